"""Input path (hcat/transforms.py to_float/reshape/normalize/to_tensor,
hcat/dataloader.py Stack): the oracle against the reference's own outputs
(tests/golden/input_path.npz), and the host-side behaviour of the drop-in
transforms that needs no device."""
import os

import numpy as np
import pytest

from hcunet_amd import transforms as tr
from hcunet_amd.dataloader import Stack
from oracle import input_oracle as io

GOLD = np.load(os.path.join(os.path.dirname(__file__), 'golden', 'input_path.npz'))


@pytest.mark.parametrize('name', ['img_half', 'img_odd', 'img_u8'])
def test_oracle_matches_reference(name):
    o = io.network_input(GOLD[name + '.raw'], GOLD[name + '.mean'], GOLD[name + '.std'])
    np.testing.assert_array_equal(o.view(np.uint16), GOLD[name + '.out'])


def test_oracle_stack_pattern_matches_reference():
    np.testing.assert_array_equal(io.network_input(GOLD['stack.image_raw'], [.5] * 4, [.5] * 4).view(np.uint16),
                                  GOLD['stack.image'])
    np.testing.assert_array_equal(io.network_input(GOLD['stack.mask_raw']).view(np.uint16), GOLD['stack.mask'])
    np.testing.assert_array_equal(io.network_input(GOLD['stack.pwl_raw']).view(np.uint16), GOLD['stack.pwl'])


def test_to_float_rejects_other_dtypes_like_reference():
    assert str(GOLD['err.to_float_int32']) == 'TypeError'
    with pytest.raises(TypeError):
        tr.to_float()(np.zeros((2, 2, 2, 1), dtype=np.int32))


def test_lazy_chain_records_steps_and_shapes():
    raw = np.zeros((5, 7, 9, 4), dtype=np.uint16)
    v = tr.to_float()(raw)
    v = tr.reshape()(v)
    assert v.shape == (9, 7, 5, 4)
    v = tr.normalize([0.1] * 4, [0.2] * 4)(v)
    assert v.to_float and v.reshaped and v.mean == [0.1] * 4
    with pytest.raises(ValueError):
        tr.normalize()(np.zeros((3, 3), dtype=np.float64))
    with pytest.raises(ValueError):   # joint_transform's ndim check (hcat/transforms.py:67-72)
        tr.to_float()([raw, np.zeros((5, 7, 9), dtype=np.uint16)])


def test_stack_errors_like_reference(tmp_path):
    with pytest.raises(FileExistsError):
        Stack(str(tmp_path), [], [])


def test_oracle_to_tensor_rounds_like_torch():
    # torch.as_tensor(float64, dtype=half) (hcat/transforms.py:133) rounds
    # float64 -> float32 -> fp16; values just below an odd-mantissa fp16
    # midpoint expose a direct float64 -> fp16 rounding
    import torch
    v = 1 + 3 * 2.0 ** -11 - 2.0 ** -30
    rng = np.random.default_rng(11)
    # normalize-like values: (u / 2**16 + -mean) / std with non-trivial mean/std
    u = rng.integers(0, 65536, 200000).astype(np.float64)
    vals = np.concatenate([[v, -v], (u / 2 ** 16 + -0.37) / 0.213])
    got = io.to_tensor(vals.reshape(-1, 1)).reshape(-1).view(np.uint16)
    want = torch.as_tensor(vals, dtype=torch.half).numpy().view(np.uint16)
    np.testing.assert_array_equal(got, want)
    assert np.float16(v).view(np.uint16) != got[0]


def test_stack_hands_ndarrays_to_other_transforms(tmp_path):
    """a transform that is not part of the lazy device chain (the
    reference's augmentations check isinstance(image, np.ndarray)) receives the
    array the reference's eager to_float -> reshape -> normalize would hold."""
    rng = np.random.default_rng(5)
    raw = rng.integers(0, 65536, (3, 6, 5, 4)).astype(np.uint16)
    mask = rng.integers(0, 2, (3, 6, 5)).astype(np.uint8)
    pwl = rng.integers(0, 256, (3, 6, 5)).astype(np.uint8)
    files = {'a.tif': raw, 'a.mask.tif': mask, 'a.pwl.tif': pwl}
    for n in files:
        (tmp_path / n).write_bytes(b'')
    seen = []

    class probe:
        def __call__(self, image):
            assert isinstance(image, np.ndarray)
            seen.append(image.copy())
            return image

    def reader(p):
        return files[os.path.basename(p)]

    ds = Stack(str(tmp_path), [tr.to_float(), tr.reshape(), tr.normalize([0.3] * 4, [0.7] * 4), probe()],
               [], out_transforms=[], reader=reader)
    img, m, w = ds[0]
    want = raw.astype(np.float64) / 2 ** 16
    want = want.swapaxes(2, 0)
    for c in range(4):
        want[..., c] += -0.3
        want[..., c] /= 0.7
    np.testing.assert_array_equal(seen[0], want)
    assert isinstance(img, np.ndarray)
    # the untouched mask stays lazy (raw bits, channel axis added)
    assert isinstance(m, tr.PendingVolume) and m.shape == (3, 6, 5, 1)
    np.testing.assert_array_equal(m.to_ndarray()[..., 0], mask)
