#!/usr/bin/env python3
"""Generate tests/golden/input_path.npz from the REFERENCE's own input
transforms (development container only; needs /root/reference).

hcat/transforms.py imports skimage at module level (absent here), so the
classes on the input path -- to_float (:94-116), to_tensor (:118-137),
reshape (:139-157), normalize (:257-283) and their joint_transform decorator
(:15-91) -- are taken from the reference file with `ast` at generation time
and executed in a namespace holding numpy and torch.  The chains are the ones
the reference's callers build: valscripts/main_func.py:24-29 (image:
to_float -> reshape -> normalize -> to_tensor) and the Stack pattern of
hcat/dataloader.py:79-90 with tests/transforms_test.py:22-37's joint
transforms (to_float, reshape on [image, mask, pwl]; normalize on the image;
to_tensor on all three).  Nothing from the reference is stored: the fixture
holds the raw inputs and the reference's fp16 outputs (as uint16 bits).

Usage:  python tests/golden/make_input_golden.py
"""
import ast
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import REF  # noqa: E402


def reference_transforms():
    tree = ast.parse(open(os.path.join(REF, 'hcat', 'transforms.py')).read())
    keep = {'joint_transform', 'to_float', 'to_tensor', 'reshape', 'normalize'}
    body = [n for n in tree.body if isinstance(n, (ast.FunctionDef, ast.ClassDef)) and n.name in keep]
    ns = {'np': np, 'torch': torch}
    exec(compile(ast.Module(body=body, type_ignores=[]), 'reference:hcat/transforms.py', 'exec'), ns)
    return ns


def bits(t):
    return t.contiguous().view(torch.int16).numpy().view(np.uint16)


def main():
    t = reference_transforms()
    rng = np.random.default_rng(4)
    out = {}
    # image-only chain (valscripts/main_func.py:24-29), two normalisations
    for name, (Z, Y, X, C), mean, std, dt in [
            ('img_half', (7, 19, 23, 4), [0.5] * 4, [0.5] * 4, np.uint16),
            ('img_odd', (5, 13, 9, 4), [0.31, 0.12, 0.5, 0.77], [0.23, 0.5, 0.071, 0.9], np.uint16),
            ('img_u8', (6, 11, 17, 3), [0.4, 0.2, 0.6], [0.3, 0.25, 0.5], np.uint8)]:
        hi = 65536 if dt == np.uint16 else 256
        raw = rng.integers(0, hi, size=(Z, Y, X, C)).astype(dt)
        raw.flat[:8] = [0, hi - 1, 1, hi // 2, hi // 2 - 1, 3, hi - 2, 7]
        img = raw.copy()
        for tr in [t['to_float'](), t['reshape'](), t['normalize'](mean, std), t['to_tensor']()]:
            img = tr(img)
        out[name + '.raw'] = raw
        out[name + '.mean'] = np.array(mean, dtype=np.float64)
        out[name + '.std'] = np.array(std, dtype=np.float64)
        out[name + '.out'] = bits(img)
        print(name, raw.shape, '->', tuple(img.shape), img.dtype)
    # Stack.__getitem__ pattern (hcat/dataloader.py:66-90): mask/pwl get a channel
    # axis, joint to_float + reshape, image normalize, joint to_tensor
    Z, Y, X = 6, 15, 21
    image = rng.integers(0, 65536, size=(Z, Y, X, 4)).astype(np.uint16)
    mask = (rng.random((Z, Y, X)) < 0.4).astype(np.uint8) * 255
    pwl = rng.integers(0, 65536, size=(Z, Y, X)).astype(np.uint16)
    m = np.expand_dims(mask, axis=mask.ndim)
    p = np.expand_dims(pwl, axis=pwl.ndim)
    im = image.copy()
    for jt in [t['to_float'](), t['reshape']()]:
        im, m, p = jt([im, m, p])
    im = t['normalize']([0.5] * 4, [0.5] * 4)(im)
    im, m, p = t['to_tensor']()([im, m, p])
    out['stack.image_raw'] = image
    out['stack.mask_raw'] = mask
    out['stack.pwl_raw'] = pwl
    out['stack.image'] = bits(im)
    out['stack.mask'] = bits(m)
    out['stack.pwl'] = bits(p)
    print('stack', tuple(im.shape), tuple(m.shape), tuple(p.shape))
    # the reference's error for other dtypes (to_float, :113-114)
    try:
        t['to_float']()(np.zeros((2, 2, 2, 1), dtype=np.int32))
        out['err.to_float_int32'] = np.array('none')
    except Exception as e:  # noqa: BLE001
        out['err.to_float_int32'] = np.array(type(e).__name__)
    np.savez_compressed(os.path.join(HERE, 'input_path.npz'), **out)


if __name__ == '__main__':
    main()
