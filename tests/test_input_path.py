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
