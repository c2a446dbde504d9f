"""Loss (hcat.loss.cross_entropy, method='pixel') and Adam parity on the GPU."""
import numpy as np
import pytest
import torch

from hcat.loss import cross_entropy
from hcunet_amd.optim import Adam
from oracle import inputs, unet_oracle as uo

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("pwl_kind", ["f16", "f32", "none"])
@pytest.mark.parametrize("mask_kind", ["f16", "f32", "bool"])
def test_pixel_loss(pwl_kind, mask_kind):
    pred = torch.randn(2, 1, 9, 8, 5, generator=torch.Generator().manual_seed(0)) * 3
    mask = torch.from_numpy(inputs.make_mask((2, 1, 12, 11, 7)))
    pwl = torch.from_numpy(inputs.make_pwl((2, 1, 12, 11, 7)))
    if mask_kind == 'f32':
        mask = mask.float()
    elif mask_kind == 'bool':
        mask = mask > 0.5
    if pwl_kind == 'f32':
        pwl = pwl.float()
    elif pwl_kind == 'none':
        pwl = None
    pr = pred.clone().requires_grad_(True)
    ref = uo.pixel_loss(pr, mask, pwl)
    ref.backward()
    pd = pred.cuda().requires_grad_(True)
    loss = cross_entropy(pd, mask.cuda(), None if pwl is None else pwl.cuda(), method='pixel')
    (loss * 3.0).backward()
    assert abs(loss.item() - ref.item()) <= 1e-6 * abs(ref.item()) + 1e-7
    assert (pd.grad.cpu() - 3.0 * pr.grad).abs().max().item() <= 1e-6 * pr.grad.abs().max().item() * 3


def test_loss_errors():
    pred = torch.zeros(1, 1, 4, 4, 4, device='cuda')
    with pytest.raises(ValueError):
        cross_entropy(pred, pred, pred, method='bogus')
    with pytest.raises(ValueError):
        cross_entropy(pred, torch.zeros(1, 1, 3, 4, 4, device='cuda'), None)
    with pytest.raises(IndexError):
        cross_entropy(torch.zeros(4, 4, device='cuda'), pred, pred)


def test_adam_matches_torch():
    torch.manual_seed(0)
    shapes = [(8, 4, 3, 3, 2), (8,), (16, 8, 3, 3, 1), (16,)]
    ps = [torch.randn(s) for s in shapes]
    gs = [[torch.randn(s) for s in shapes] for _ in range(3)]
    ref = [p.clone().requires_grad_(True) for p in ps]
    opt_ref = torch.optim.Adam(ref, lr=1e-3, foreach=False)
    flat = torch.cat([p.reshape(-1) for p in ps]).cuda()
    views, off = [], 0
    for p in ps:
        views.append(torch.nn.Parameter(flat[off:off + p.numel()].view_as(p)))
        views[-1].data = flat[off:off + p.numel()].view_as(p)
        off += p.numel()
    gflat = torch.zeros_like(flat)
    opt = Adam(views, lr=1e-3)
    for it in range(3):
        off = 0
        for v, g in zip(views, gs[it]):
            gflat[off:off + g.numel()].copy_(g.reshape(-1))
            v.grad = gflat[off:off + g.numel()].view_as(v)
            off += g.numel()
        for r, g in zip(ref, gs[it]):
            r.grad = g.clone()
        opt.step()
        opt_ref.step()
    torch.cuda.synchronize()
    for v, r in zip(views, ref):
        assert (v.detach().cpu() - r.detach()).abs().max().item() <= 1e-6
