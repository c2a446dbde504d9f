"""Tiled inference driver on the GPU against the reference's own
predict_segmentation_mask output (tests/golden/segment_small.npz: 12 tiles of
383x383x25, NaN/Inf voxels, eval-mode BatchNorm with non-trivial running
statistics), plus the forward-only plan it runs on."""
import numpy as np
import pytest
import torch

from hcat.unet import Unet_Constructor
from hcunet_amd import segment as seg
from tests.test_segment_oracle import SEG_KW, gold, golden_state, golden_volume

pytestmark = pytest.mark.gpu

PROB_ATOL = 1e-5   # fp32 GPU convolutions vs the reference's fp32 CPU ones, after the sigmoid


def _net(g):
    torch.manual_seed(0)
    m = Unet_Constructor(**SEG_KW)
    m.load_state_dict(golden_state(g))
    return m.cuda().eval()


def test_tiled_probability_map_matches_reference():
    g = gold()
    m = _net(g)
    x = golden_volume(g).numpy().copy()
    prob = seg.predict_segmentation_mask(m, x, 'cuda', use_probability_map=True,
                                         total_memory=float(g['cuda_mem']))
    assert prob.device.type == 'cpu' and prob.dtype == torch.float32
    assert prob.shape == g['prob'].shape
    err = np.abs(prob.numpy() - g['prob']).max()
    assert err <= PROB_ATOL, err
    # the caller's volume is not modified (the reference cleans it in place)
    assert np.isnan(x).sum() == 1


def test_tiled_mask_matches_reference():
    g = gold()
    m = _net(g)
    thr = float(g['threshold'])
    mask = seg.predict_segmentation_mask(m, golden_volume(g).numpy().copy(), 'cuda',
                                         mask_cell_prob_threshold=thr,
                                         total_memory=float(g['cuda_mem']))
    assert mask.dtype == torch.uint8 and str(mask.dtype) == str(g['mask_dtype'])
    near = np.abs(g['prob'] - thr) < 2 * PROB_ATOL
    assert (mask.numpy()[~near] == g['mask'][~near]).all()
    assert 0.2 < mask.float().mean().item() < 0.8


def test_batched_tiles_equal_single_tiles():
    g = gold()
    m = _net(g)
    x = golden_volume(g)
    a = seg.predict_segmentation_mask(m, x, 'cuda', use_probability_map=True,
                                      total_memory=float(g['cuda_mem']))
    b = seg.predict_segmentation_mask(m, x, 'cuda', use_probability_map=True,
                                      total_memory=float(g['cuda_mem']), tiles_per_batch=1)
    assert (a - b).abs().max().item() <= 1e-6


def test_reflection_pad_on_device_matches_reference():
    g = gold()
    small = torch.from_numpy(g['small'])
    out = seg.pad_image_with_reflections(small.cuda(), pad_size=(4, 6, 2))
    assert out.is_cuda
    np.testing.assert_array_equal(out.cpu().numpy(), g['padded'])
    out16 = seg.pad_image_with_reflections(small.half(), pad_size=(4, 6, 2))
    assert out16.dtype == torch.float16 and out16.device.type == 'cpu'
    np.testing.assert_array_equal(out16.float().numpy(), torch.from_numpy(g['padded']).half().float().numpy())


def test_forward_only_plan_matches_training_plan_output():
    """Under no_grad the module runs the forward-only plan (activations in two
    ping-pong buffers); its eval output equals the full plan's bit for bit."""
    g = gold()
    m = _net(g)
    x = torch.from_numpy(np.nan_to_num(golden_volume(g).numpy()[:, :, :96, :96, :]))
    x = x.cuda()
    with torch.no_grad():
        y0 = m(x)
    y1 = m(x.clone().requires_grad_(True))
    assert torch.equal(y0, y1.detach())
    eng = m.engine()
    p_full = eng.plan(x.shape, False, forward_only=False)
    p_fwd = eng.plan(x.shape, False, forward_only=True)
    assert p_fwd.saved_bytes < p_full.saved_bytes / 2
    assert p_fwd.scratch_bytes < p_full.scratch_bytes


def test_forward_only_plan_train_mode_matches_full_plan():
    """Train-mode BatchNorm under no_grad (the tiled driver in m.train()) runs
    the forward-only plan with batch statistics: its output and the updated
    running mean / var / num_batches_tracked equal one train-mode forward of
    the full plan (the two plans may pick different convolution tilings, so
    to fp32 summation-order rounding)."""
    g = gold()
    # the tiled driver's own cleaning (NaN -> 0, Inf -> 1): batch statistics stay finite
    x = torch.from_numpy(np.nan_to_num(golden_volume(g).numpy()[:, :, :96, :96, :],
                                       nan=0.0, posinf=1.0, neginf=1.0)).cuda()
    ma, mb = _net(g).train(), _net(g).train()
    nbt0 = [int(b.num_batches_tracked) for b in ma.modules() if isinstance(b, torch.nn.BatchNorm3d)]
    with torch.no_grad():
        ya = ma(x)
    yb = mb(x.clone().requires_grad_(True)).detach()
    scale = max(yb.abs().max().item(), 1e-6)
    assert (ya - yb).abs().max().item() <= 1e-5 * scale
    bns = [(a, b) for a, b in zip(ma.modules(), mb.modules()) if isinstance(a, torch.nn.BatchNorm3d)]
    for (a, b), n0 in zip(bns, nbt0):
        assert int(a.num_batches_tracked) == int(b.num_batches_tracked) == n0 + 1
        for s in ('running_mean', 'running_var'):
            ra, rb = getattr(a, s), getattr(b, s)
            assert (ra - rb).abs().max().item() <= 1e-5 * max(rb.abs().max().item(), 1e-6), s


def test_train_mode_runs_tile_by_tile():
    """In train mode BatchNorm uses batch statistics, so tiles run one at a
    time (as the reference's loop does) and the running statistics move."""
    g = gold()
    m = _net(g).train()
    rm0 = m.down_steps[0].batch1.running_mean.clone()
    out = seg.predict_segmentation_mask(m, golden_volume(g), 'cuda', use_probability_map=True,
                                        total_memory=float(g['cuda_mem']))
    assert torch.isfinite(out).all()
    assert not torch.equal(rm0, m.down_steps[0].batch1.running_mean)
    assert int(m.down_steps[0].batch1.num_batches_tracked) == 12
