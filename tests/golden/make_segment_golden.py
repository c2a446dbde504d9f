#!/usr/bin/env python3
"""Generate tests/golden/segment_small.npz from the REFERENCE's own tiled
inference functions (development container only; needs /root/reference).

hcat/segment.py and hcat/utils.py import numba, skimage, cv2, GPy and
torchvision at module level (absent here), so the three functions on the path
-- predict_segmentation_mask (segment.py:21-136), pad_image_with_reflections
and calculate_indexes (utils.py:33-124) -- are taken from the reference files
with `ast` at generation time and executed in a namespace holding what they
use: numpy, torch, `utils` (the two reference helpers) and `hcat` with
__CUDA_MEM__ (segment.py:53-54 reads hcat.__CUDA_MEM__).  The network is the
reference's own Unet_Constructor (imported as in make_golden.py), seeded, in
eval mode.  Nothing from the reference is stored: the fixture holds the
config, the input seed and the reference's outputs.

Usage:  python tests/golden/make_segment_golden.py
"""
import ast
import os
import sys
import types
from typing import List, Tuple

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

from make_golden import REF, import_reference  # noqa: E402
from oracle import inputs  # noqa: E402

# a small net whose output covers PAD + EVAL of the 4 GB table entry
# ([128, 128, 6] with PAD (128, 128, 10)), so the reference's tiling succeeds
SEG_KW = dict(image_dimensions=3, in_channels=4, out_channels=1, feature_sizes=[4, 8],
              kernel={'conv1': (3, 3, 2), 'conv2': (3, 3, 1)}, upsample_kernel=(2, 2, 2),
              max_pool_kernel=(2, 2, 1), upsample_stride=(2, 2, 1))
SHAPE = (1, 4, 160, 160, 16)
CUDA_MEM = 4.5e9       # -> '4': EVAL [128, 128, 6]
INDEX_CASES = [(128, 350, 1000, 1256), (128, 128, 160, 416), (10, 6, 8, 28), (10, 15, 16, 36),
               (128, 350, 300, 556), (2, 5, 5, 9), (4, 3, 20, 28)]


def reference_functions():
    def extract(path, names):
        tree = ast.parse(open(path).read())
        return [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in names]

    ns = {'np': np, 'torch': torch, 'Tuple': Tuple, 'List': List}
    mod = ast.Module(body=extract(os.path.join(REF, 'hcat', 'utils.py'),
                                  {'pad_image_with_reflections', 'calculate_indexes'}),
                     type_ignores=[])
    exec(compile(mod, 'reference:hcat/utils.py', 'exec'), ns)
    ns['utils'] = types.SimpleNamespace(pad_image_with_reflections=ns['pad_image_with_reflections'],
                                        calculate_indexes=ns['calculate_indexes'])
    ns['hcat'] = types.SimpleNamespace(__CUDA_MEM__=CUDA_MEM)
    mod = ast.Module(body=extract(os.path.join(REF, 'hcat', 'segment.py'),
                                  {'predict_segmentation_mask'}), type_ignores=[])
    exec(compile(mod, 'reference:hcat/segment.py', 'exec'), ns)
    return ns


def main():
    unet_mod, _ = import_reference()
    ns = reference_functions()
    torch.manual_seed(0)
    net = unet_mod.Unet_Constructor(**SEG_KW).eval()
    # non-trivial BatchNorm running statistics (eval mode uses them)
    with torch.no_grad():
        g = torch.Generator().manual_seed(5)
        for m in net.modules():
            if isinstance(m, torch.nn.BatchNorm3d):
                m.running_mean.copy_(torch.randn(m.num_features, generator=g) * 0.1)
                m.running_var.copy_(torch.rand(m.num_features, generator=g) * 0.2 + 0.05)
        net.out_conv.weight.mul_(2.0)
    state = {k: v.detach().clone() for k, v in net.state_dict().items()}
    x = torch.from_numpy(inputs.make_x(SHAPE, seed=11))
    x[0, 1, 5, 7, 2] = float('nan')
    x[0, 2, 150, 3, 13] = float('inf')
    x[0, 0, 80, 80, 0] = -float('inf')
    prob = ns['predict_segmentation_mask'](net, x.numpy().copy(), 'cpu', use_probability_map=True)
    thr = float(np.round(np.median(prob.numpy()), 3))   # a threshold that splits the volume
    msk = ns['predict_segmentation_mask'](net, x.numpy().copy(), 'cpu', use_probability_map=False,
                                          mask_cell_prob_threshold=thr)
    # reflection padding of a small odd-sized volume, and the index helper
    small = torch.from_numpy(inputs.make_x((1, 2, 7, 9, 5), seed=12))
    padded = ns['pad_image_with_reflections'](small, pad_size=(4, 6, 2))
    idx = [np.asarray(ns['calculate_indexes'](*c), dtype=np.int64) for c in INDEX_CASES]
    out = dict(shape=np.asarray(SHAPE), x_seed=np.asarray(11), cuda_mem=np.asarray(CUDA_MEM),
               prob=prob.numpy().astype(np.float32), mask=msk.numpy(),
               mask_dtype=np.asarray(str(msk.dtype)), threshold=np.asarray(thr),
               small=small.numpy(), padded=padded.numpy(),
               index_cases=np.asarray(INDEX_CASES, dtype=np.int64))
    for i, a in enumerate(idx):
        out['index_%d' % i] = a
    for k, v in state.items():
        out['state/' + k] = v.numpy()
    path = os.path.join(HERE, 'segment_small.npz')
    np.savez_compressed(path, **out)
    print('wrote', path, 'prob quantiles', np.quantile(prob.numpy(), [0, 0.1, 0.5, 0.9, 1]),
          'mask mean', float(msk.float().mean()))


if __name__ == '__main__':
    main()
