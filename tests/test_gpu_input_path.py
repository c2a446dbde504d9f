"""Input path on the GPU (csrc/ingest.hip through hcunet_amd.transforms /
dataloader): bit-exact against the reference's own outputs
(tests/golden/input_path.npz) and the oracle restatement."""
import os

import numpy as np
import pytest
import torch

import hcat.dataloader as hdl
import hcat.transforms as ht
from hcunet_amd.transforms import ingest
from oracle import input_oracle as io

pytestmark = pytest.mark.gpu
GOLD = np.load(os.path.join(os.path.dirname(__file__), 'golden', 'input_path.npz'))


def bits(t):
    return t.cpu().contiguous().view(torch.int16).numpy().view(np.uint16)


@pytest.mark.parametrize('name', ['img_half', 'img_odd', 'img_u8'])
def test_transform_chain_matches_reference(name):
    img = GOLD[name + '.raw']
    # valscripts/main_func.py:24-29
    for t in [ht.to_float(), ht.reshape(), ht.normalize(list(GOLD[name + '.mean']), list(GOLD[name + '.std'])),
              ht.to_tensor()]:
        img = t(img)
    assert img.is_cuda and img.dtype == torch.float16
    np.testing.assert_array_equal(bits(img), GOLD[name + '.out'])


def test_stack_matches_reference(tmp_path):
    # Stack reads <name>.tif, <name>.mask.tif, <name>.pwl.tif (hcat/dataloader.py:41-64);
    # np.save'd arrays under those names, read back with np.load
    for suffix, key in [('.tif', 'stack.image_raw'), ('.mask.tif', 'stack.mask_raw'), ('.pwl.tif', 'stack.pwl_raw')]:
        with open(os.path.join(tmp_path, 'vol' + suffix), 'wb') as f:
            np.save(f, GOLD[key])
    data = hdl.Stack(str(tmp_path), image_transforms=[ht.normalize([0.5] * 4, [0.5] * 4)],
                     joint_transforms=[ht.to_float(), ht.reshape()], reader=np.load)
    assert len(data) == 1
    image, mask, pwl = data[0]
    np.testing.assert_array_equal(bits(image), GOLD['stack.image'])
    np.testing.assert_array_equal(bits(mask), GOLD['stack.mask'])
    np.testing.assert_array_equal(bits(pwl), GOLD['stack.pwl'])
    got = list(data.prefetch([0, 0, 0]))
    assert len(got) == 3
    for im, m, p in got:
        np.testing.assert_array_equal(bits(im), GOLD['stack.image'])
        np.testing.assert_array_equal(bits(p), GOLD['stack.pwl'])


def test_fp16_rounding_matches_torch():
    # float64 -> fp16 as torch.as_tensor(float64, dtype=half) rounds (the
    # reference's to_tensor, hcat/transforms.py:133): float64 -> float32 -> fp16,
    # each to nearest even, over ties, near-ties, subnormals, overflow, NaN/Inf
    rng = np.random.default_rng(0)
    h = np.arange(0, 1 << 16, dtype=np.uint32).astype(np.uint16).view(np.float16)
    h = h[np.isfinite(h)].astype(np.float64)
    nxt = np.nextafter(h.astype(np.float16), np.float16(np.inf)).astype(np.float64)
    mid = (h + nxt) / 2                                  # exact ties
    vals = np.concatenate([h, mid, np.nextafter(mid, 0), np.nextafter(mid, np.inf),
                           rng.standard_normal(100000) * 10.0 ** rng.integers(-9, 6, 100000),
                           [65504.0, 65519.99, 65520.0, 1e6, -1e6, 2.0 ** -25, 2.0 ** -25 * 1.0000001,
                            2.0 ** -26, 0.0, -0.0, np.inf, -np.inf, np.nan,
                            1 + 3 * 2.0 ** -11 - 2.0 ** -30, -(1 + 3 * 2.0 ** -11 - 2.0 ** -30)]])
    vals = vals[np.isfinite(vals) | np.isinf(vals) | np.isnan(vals)]
    n = vals.size
    a = vals.reshape(1, 1, n, 1)                        # [Z=1, Y=1, X=n, C=1] float64
    v = ht.to_tensor()(a)                               # no to_float / reshape: [1,1,1,1,n]
    got = bits(v).reshape(-1)
    want = torch.as_tensor(vals, dtype=torch.half).numpy().view(np.uint16)
    # the float32 double-rounding case (just below an odd-mantissa fp16 midpoint)
    # is among the values and differs from a direct float64 -> fp16 rounding
    assert (np.float16(1 + 3 * 2.0 ** -11 - 2.0 ** -30).view(np.uint16)
            != torch.as_tensor([1 + 3 * 2.0 ** -11 - 2.0 ** -30], dtype=torch.half).numpy().view(np.uint16)[0])
    nan = np.isnan(vals)
    np.testing.assert_array_equal(got[~nan], want[~nan])
    assert np.all((got[nan] & 0x7c00) == 0x7c00) and np.all((got[nan] & 0x3ff) != 0)


def test_batched_ingest_matches_oracle():
    rng = np.random.default_rng(3)
    raw = rng.integers(0, 65536, size=(3, 16, 70, 45, 4)).astype(np.uint16)
    mean, std = [0.5, 0.4, 0.3, 0.6], [0.5, 0.25, 0.1, 0.7]
    out = ingest(raw, mean, std)
    want = np.concatenate([io.network_input(raw[b], mean, std) for b in range(3)])
    np.testing.assert_array_equal(bits(out), want.view(np.uint16))
    # the network consumes the fp16 batch directly
    assert out.shape == (3, 4, 45, 70, 16)


def test_no_reshape_layout():
    rng = np.random.default_rng(5)
    raw = rng.integers(0, 256, size=(9, 33, 40, 2)).astype(np.uint8)
    v = ht.to_tensor()(ht.to_float()(raw))              # [1, C, Z, Y, X]
    want = np.moveaxis((raw.astype(np.float64) / 256).astype(np.float16), -1, 0)[None]
    np.testing.assert_array_equal(bits(v), want.view(np.uint16))
