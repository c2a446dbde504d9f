"""CPU checks of the tiled inference driver: the oracle
restatement (oracle/segment_oracle.py) against the reference's own outputs
(tests/golden/segment_small.npz, made by make_segment_golden.py), and the
driver's host logic (tile indexes, tile-size table)."""
import os

import numpy as np
import pytest
import torch

from hcunet_amd import segment as seg
from oracle import inputs, segment_oracle as so, unet_oracle as uo

GOLD = os.path.join(os.path.dirname(__file__), 'golden', 'segment_small.npz')
SEG_KW = dict(image_dimensions=3, in_channels=4, out_channels=1, feature_sizes=[4, 8],
              kernel={'conv1': (3, 3, 2), 'conv2': (3, 3, 1)}, upsample_kernel=(2, 2, 2),
              max_pool_kernel=(2, 2, 1), upsample_stride=(2, 2, 1))


def gold():
    return np.load(GOLD)


def golden_volume(g):
    x = torch.from_numpy(inputs.make_x(tuple(g['shape']), seed=int(g['x_seed'])))
    x[0, 1, 5, 7, 2] = float('nan')
    x[0, 2, 150, 3, 13] = float('inf')
    x[0, 0, 80, 80, 0] = -float('inf')
    return x


def golden_state(g):
    return {k[len('state/'):]: torch.from_numpy(g[k]) for k in g.files if k.startswith('state/')}


def test_calculate_indexes_match_reference():
    g = gold()
    for i, case in enumerate(g['index_cases']):
        ref = g['index_%d' % i].tolist()
        assert so.calculate_indexes(*[int(v) for v in case]) == ref, case
        assert seg.calculate_indexes(*[int(v) for v in case]) == ref, case


def test_reflection_pad_oracle_matches_reference():
    g = gold()
    out = so.pad_image_with_reflections(torch.from_numpy(g['small']), pad_size=(4, 6, 2))
    np.testing.assert_array_equal(out.numpy(), g['padded'])
    with pytest.raises(ValueError, match='Padding must be divisible by 2'):
        so.pad_image_with_reflections(torch.zeros(1, 1, 4, 4, 4), pad_size=(3, 2, 2))
    with pytest.raises(TypeError):
        seg.pad_image_with_reflections(np.zeros((1, 1, 4, 4, 4)), pad_size=(2, 2, 2))


def test_tile_size_table_handles_any_memory_size():
    # the reference raises KeyError unless floor(GB) is 4, 6, 8 or 11 (segment.py:52-54)
    assert seg.eval_image_size(288e9) == [350, 350, 15]   # MI355X
    assert seg.eval_image_size(11.9e9) == [350, 350, 15]
    assert seg.eval_image_size(8.2e9) == [300, 300, 10]
    assert seg.eval_image_size(7.5e9) == [300, 300, 6]
    assert seg.eval_image_size(4.5e9) == [128, 128, 6]
    assert seg.eval_image_size(2e9) == [128, 128, 6]


def test_oracle_tiled_prediction_matches_reference():
    """The oracle's tiled driver + CPU U-Net (eval) reproduces the reference's
    predict_segmentation_mask output (12 tiles of 383x383x25, NaN/Inf input)."""
    g = gold()
    spec = uo.normalize_spec(**SEG_KW)
    net = uo.OracleUnet(spec, golden_state(g))
    prob = so.predict_segmentation_mask(lambda t: net.forward(t, training=False),
                                        golden_volume(g).numpy().copy(), float(g['cuda_mem']),
                                        use_probability_map=True)
    np.testing.assert_allclose(prob.numpy(), g['prob'], rtol=0, atol=2e-6)
    thr = float(g['threshold'])
    mask = (prob.numpy() > thr).astype(np.uint8)
    near = np.abs(g['prob'] - thr) < 1e-5
    assert (mask[~near] == g['mask'][~near]).all()
