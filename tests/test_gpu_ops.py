"""Per-op parity of the HIP kernels against torch CPU fp64 references of the
same op (nn.Conv3d / nn.ConvTranspose3d forward, input and weight gradients,
MaxPool3d), called through the C-ABI on channels-last device tensors."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

from hcunet_amd import _lib
from tests.helpers import desc, from_cl, max_abs, out_dims, rup4, scratch_for, stream, to_cl

pytestmark = pytest.mark.gpu

CONV_CASES = [
    # B, Cin, Cout, X, Y, Z, k, dil, groups
    (2, 4, 8, 20, 18, 7, (3, 3, 2), (1, 1, 1), 1),
    (1, 8, 8, 17, 21, 15, (3, 3, 1), (1, 1, 1), 1),
    (2, 8, 16, 13, 12, 9, (3, 3, 2), (1, 1, 1), 1),
    (1, 16, 32, 11, 10, 6, (3, 3, 2), (1, 1, 1), 1),
    (1, 32, 64, 9, 8, 5, (3, 3, 1), (1, 1, 1), 1),
    (1, 64, 128, 8, 8, 4, (3, 3, 2), (1, 1, 1), 1),
    (1, 8, 16, 12, 12, 5, (3, 3, 2), (1, 1, 1), 2),
    (1, 8, 8, 14, 13, 6, (3, 3, 1), (2, 2, 1), 1),
    (2, 6, 12, 9, 10, 6, (3, 3, 3), (1, 1, 1), 1),
    (1, 3, 5, 9, 9, 4, (1, 1, 1), (1, 1, 1), 1),
    (1, 4, 8, 10, 10, 20, (3, 3, 2), (1, 1, 1), 1),
    # wgrad8 (z tap on the column side): 8->8 at the level-0 depth, 16 columns
    # with KZ=1, two row chunks (16 input channels), ragged x/y tiles
    (1, 8, 8, 19, 21, 16, (3, 3, 2), (1, 1, 1), 1),
    (2, 8, 16, 13, 12, 9, (3, 3, 1), (1, 1, 1), 1),
    (1, 16, 8, 12, 11, 10, (3, 3, 2), (1, 1, 1), 1),
    (1, 8, 8, 11, 9, 35, (3, 3, 2), (1, 1, 1), 1),
]


def _conv_ref(B, Cin, Cout, X, Y, Z, k, dil, groups, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, Cin, X, Y, Z, generator=g, dtype=torch.float64)
    w = torch.randn(Cout, Cin // groups, *k, generator=g, dtype=torch.float64) * 0.2
    b = torch.randn(Cout, generator=g, dtype=torch.float64)
    return x, w, b


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv3d_fwd_dgrad_wgrad(case):
    B, Cin, Cout, X, Y, Z, k, dil, groups = case
    x, w, b = _conv_ref(*case)
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    y = F.conv3d(xr, wr, br, dilation=dil, groups=groups)
    gy = torch.randn(y.shape, generator=torch.Generator().manual_seed(7), dtype=torch.float64)
    y.backward(gy)
    d = desc(B, Cin, Cout, X, Y, Z, k, dil=dil, groups=groups)
    od = out_dims(d)
    assert od == tuple(y.shape[2:])
    L = _lib.lib()
    sc = scratch_for(d)
    xcl = to_cl(x)
    wd = w.float().cuda().contiguous()
    bd = b.float().cuda()
    ycl = torch.full((B, *od, rup4(Cout)), float('nan'), device='cuda')
    _lib.check(L.hcu_conv_fwd_cl(ctypes.byref(d), _lib.ptr(xcl), _lib.ptr(wd), _lib.ptr(bd),
                                 _lib.ptr(ycl), _lib.ptr(sc), sc.numel(), stream()))
    torch.cuda.synchronize()
    ours = from_cl(ycl, Cout)
    scale = y.abs().max().item()
    assert max_abs(ours, y.detach()) <= 2e-6 * scale + 1e-6, max_abs(ours, y.detach())
    if rup4(Cout) != Cout:
        assert torch.all(ycl[..., Cout:] == 0)
    # input gradient
    gcl = to_cl(gy)
    dx = torch.full((B, X, Y, Z, rup4(Cin)), float('nan'), device='cuda')
    _lib.check(L.hcu_conv_dgrad_cl(ctypes.byref(d), _lib.ptr(gcl), _lib.ptr(wd), _lib.ptr(dx),
                                   _lib.ptr(sc), sc.numel(), stream()))
    torch.cuda.synchronize()
    ref_dx = xr.grad
    assert max_abs(from_cl(dx, Cin), ref_dx) <= 2e-6 * ref_dx.abs().max().item() + 1e-6
    # weight / bias gradient
    dw = torch.full_like(wd, float('nan'))
    db = torch.full_like(bd, float('nan'))
    _lib.check(L.hcu_conv_wgrad_cl(ctypes.byref(d), _lib.ptr(xcl), _lib.ptr(gcl), _lib.ptr(dw),
                                   _lib.ptr(db), _lib.ptr(sc), sc.numel(), stream()))
    torch.cuda.synchronize()
    assert max_abs(dw.cpu(), wr.grad) <= 5e-6 * wr.grad.abs().max().item() + 1e-6
    assert max_abs(db.cpu(), br.grad) <= 5e-6 * br.grad.abs().max().item() + 1e-6


CONVT_CASES = [
    # B, Cin, Cout, X, Y, Z, k, s
    (2, 16, 8, 7, 6, 5, (2, 2, 2), (2, 2, 1)),
    (1, 128, 64, 6, 6, 11, (2, 2, 2), (2, 2, 1)),
    (1, 8, 4, 5, 4, 3, (8, 8, 2), (2, 2, 1)),
    (1, 12, 6, 4, 5, 3, (2, 2, 2), (2, 2, 2)),
    (2, 8, 5, 3, 3, 3, (3, 3, 3), (2, 2, 1)),
]


@pytest.mark.parametrize("case", CONVT_CASES)
def test_convtranspose3d_fwd_dgrad_wgrad(case):
    B, Cin, Cout, X, Y, Z, k, s = case
    g = torch.Generator().manual_seed(1)
    x = torch.randn(B, Cin, X, Y, Z, generator=g, dtype=torch.float64)
    w = torch.randn(Cin, Cout, *k, generator=g, dtype=torch.float64) * 0.2
    b = torch.randn(Cout, generator=g, dtype=torch.float64)
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x, w, b))
    y = F.conv_transpose3d(xr, wr, br, stride=s)
    gy = torch.randn(y.shape, generator=torch.Generator().manual_seed(3), dtype=torch.float64)
    y.backward(gy)
    d = desc(B, Cin, Cout, X, Y, Z, k, stride=s, transposed=1)
    od = out_dims(d)
    assert od == tuple(y.shape[2:])
    L = _lib.lib()
    sc = scratch_for(d)
    xcl = to_cl(x)
    wd = w.float().cuda().contiguous()
    bd = b.float().cuda()
    ycl = torch.full((B, *od, rup4(Cout)), float('nan'), device='cuda')
    _lib.check(L.hcu_conv_fwd_cl(ctypes.byref(d), _lib.ptr(xcl), _lib.ptr(wd), _lib.ptr(bd),
                                 _lib.ptr(ycl), _lib.ptr(sc), sc.numel(), stream()))
    torch.cuda.synchronize()
    assert max_abs(from_cl(ycl, Cout), y.detach()) <= 2e-6 * y.abs().max().item() + 1e-6
    gcl = to_cl(gy)
    dx = torch.full((B, X, Y, Z, rup4(Cin)), float('nan'), device='cuda')
    _lib.check(L.hcu_conv_dgrad_cl(ctypes.byref(d), _lib.ptr(gcl), _lib.ptr(wd), _lib.ptr(dx),
                                   _lib.ptr(sc), sc.numel(), stream()))
    torch.cuda.synchronize()
    assert max_abs(from_cl(dx, Cin), xr.grad) <= 2e-6 * xr.grad.abs().max().item() + 1e-6
    dw = torch.full_like(wd, float('nan'))
    db = torch.full_like(bd, float('nan'))
    _lib.check(L.hcu_conv_wgrad_cl(ctypes.byref(d), _lib.ptr(xcl), _lib.ptr(gcl), _lib.ptr(dw),
                                   _lib.ptr(db), _lib.ptr(sc), sc.numel(), stream()))
    torch.cuda.synchronize()
    assert max_abs(dw.cpu(), wr.grad) <= 5e-6 * wr.grad.abs().max().item() + 1e-6
    assert max_abs(db.cpu(), br.grad) <= 5e-6 * br.grad.abs().max().item() + 1e-6


@pytest.mark.parametrize("shape,k", [((2, 8, 21, 17, 5), (2, 2, 1)),
                                     ((1, 12, 9, 8, 7), (2, 2, 2)),
                                     ((1, 4, 5, 5, 5), (3, 1, 2))])
def test_maxpool_fwd(shape, k):
    x = torch.randn(*shape, generator=torch.Generator().manual_seed(2))
    ref = F.max_pool3d(x, k)
    B, C, X, Y, Z = shape
    xcl = to_cl(x)
    y = torch.empty(B, X // k[0], Y // k[1], Z // k[2], rup4(C), device='cuda')
    _lib.check(_lib.lib().hcu_maxpool_fwd_cl(B, C, X, Y, Z, (ctypes.c_int * 3)(*k), _lib.ptr(xcl),
                                             _lib.ptr(y), stream()))
    torch.cuda.synchronize()
    assert torch.equal(from_cl(y, C), ref)


# ---------------------------------------------------------------------------
# bf16 path (config 3): the same ops on bf16 channels-last activations.  The
# references use the bf16-rounded operands in fp64, so the only differences
# are fp32 accumulation and the bf16 rounding of stored outputs (2^-9
# relative): outputs within 1e-2 of max |ref|, fp32 weight gradients within
# 1e-4 relative.
def _rup8(c):
    return (c + 7) // 8 * 8


def _to_cl_bf(t):
    B, C = t.shape[:2]
    cl = t.permute(0, 2, 3, 4, 1).contiguous()
    Cs = _rup8(C)
    if Cs != C:
        cl = torch.cat([cl, torch.zeros(*cl.shape[:-1], Cs - C, dtype=cl.dtype)], -1)
    return cl.to(torch.bfloat16).cuda().contiguous()


def _bf(t):
    return t.to(torch.bfloat16).double()


BF_CONV_CASES = [
    # B, Cin, Cout, X, Y, Z, k
    (2, 4, 32, 20, 18, 7, (3, 3, 2)),
    (1, 32, 32, 17, 21, 15, (3, 3, 1)),
    (2, 32, 64, 13, 12, 9, (3, 3, 2)),
    (1, 64, 64, 11, 10, 6, (3, 3, 1)),
    (1, 128, 256, 9, 8, 5, (3, 3, 2)),
    (1, 256, 256, 10, 10, 11, (3, 3, 1)),
    (2, 512, 512, 10, 10, 11, (3, 3, 1)),
]


@pytest.mark.parametrize("case", BF_CONV_CASES)
def test_bf16_conv3d_fwd_dgrad_wgrad(case):
    B, Cin, Cout, X, Y, Z, k = case
    g = torch.Generator().manual_seed(5)
    x = _bf(torch.randn(B, Cin, X, Y, Z, generator=g, dtype=torch.float64))
    w = torch.randn(Cout, Cin, *k, generator=g, dtype=torch.float64) * (1.0 / (Cin * 9) ** 0.5)
    b = torch.randn(Cout, generator=g, dtype=torch.float64)
    wb = _bf(w)
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x, wb, b))
    y = F.conv3d(xr, wr, br)
    gy = _bf(torch.randn(y.shape, generator=torch.Generator().manual_seed(7), dtype=torch.float64))
    y.backward(gy)
    d = desc(B, Cin, Cout, X, Y, Z, k)
    d.dtype = _lib.HCU_BF16
    od = out_dims(d)
    L = _lib.lib()
    sc = scratch_for(d)
    xcl = _to_cl_bf(x)
    wd = w.float().cuda().contiguous()
    bd = b.float().cuda()
    ycl = torch.full((B, *od, _rup8(Cout)), float('nan'), device='cuda', dtype=torch.bfloat16)
    _lib.check(L.hcu_conv_fwd_cl(ctypes.byref(d), _lib.ptr(xcl), _lib.ptr(wd), _lib.ptr(bd),
                                 _lib.ptr(ycl), _lib.ptr(sc), sc.numel(), stream()))
    torch.cuda.synchronize()
    ours = ycl[..., :Cout].permute(0, 4, 1, 2, 3).double().cpu()
    assert max_abs(ours, y.detach()) <= 1e-2 * y.abs().max().item(), max_abs(ours, y.detach())
    gcl = _to_cl_bf(gy)
    dx = torch.full((B, X, Y, Z, _rup8(Cin)), float('nan'), device='cuda', dtype=torch.bfloat16)
    _lib.check(L.hcu_conv_dgrad_cl(ctypes.byref(d), _lib.ptr(gcl), _lib.ptr(wd), _lib.ptr(dx),
                                   _lib.ptr(sc), sc.numel(), stream()))
    torch.cuda.synchronize()
    ref_dx = xr.grad
    got = dx[..., :Cin].permute(0, 4, 1, 2, 3).double().cpu()
    assert max_abs(got, ref_dx) <= 1e-2 * ref_dx.abs().max().item(), max_abs(got, ref_dx)
    dw = torch.full_like(wd, float('nan'))
    db = torch.full_like(bd, float('nan'))
    _lib.check(L.hcu_conv_wgrad_cl(ctypes.byref(d), _lib.ptr(xcl), _lib.ptr(gcl), _lib.ptr(dw),
                                   _lib.ptr(db), _lib.ptr(sc), sc.numel(), stream()))
    torch.cuda.synchronize()
    assert max_abs(dw.cpu(), wr.grad) <= 1e-4 * wr.grad.abs().max().item(), max_abs(dw.cpu(), wr.grad)
    assert max_abs(db.cpu(), br.grad) <= 1e-4 * br.grad.abs().max().item()


BF_CONVT_CASES = [
    (2, 64, 32, 7, 6, 5, (2, 2, 2), (2, 2, 1)),
    (1, 512, 256, 8, 8, 11, (2, 2, 2), (2, 2, 1)),
    (1, 128, 64, 6, 6, 11, (2, 2, 2), (2, 2, 1)),
]


@pytest.mark.parametrize("case", BF_CONVT_CASES)
def test_bf16_convtranspose3d_fwd_dgrad_wgrad(case):
    B, Cin, Cout, X, Y, Z, k, s = case
    g = torch.Generator().manual_seed(1)
    x = _bf(torch.randn(B, Cin, X, Y, Z, generator=g, dtype=torch.float64))
    w = torch.randn(Cin, Cout, *k, generator=g, dtype=torch.float64) * (1.0 / Cin ** 0.5)
    b = torch.randn(Cout, generator=g, dtype=torch.float64)
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x, _bf(w), b))
    y = F.conv_transpose3d(xr, wr, br, stride=s)
    gy = _bf(torch.randn(y.shape, generator=torch.Generator().manual_seed(3), dtype=torch.float64))
    y.backward(gy)
    d = desc(B, Cin, Cout, X, Y, Z, k, stride=s, transposed=1)
    d.dtype = _lib.HCU_BF16
    od = out_dims(d)
    L = _lib.lib()
    sc = scratch_for(d)
    xcl = _to_cl_bf(x)
    wd = w.float().cuda().contiguous()
    bd = b.float().cuda()
    ycl = torch.full((B, *od, _rup8(Cout)), float('nan'), device='cuda', dtype=torch.bfloat16)
    _lib.check(L.hcu_conv_fwd_cl(ctypes.byref(d), _lib.ptr(xcl), _lib.ptr(wd), _lib.ptr(bd),
                                 _lib.ptr(ycl), _lib.ptr(sc), sc.numel(), stream()))
    torch.cuda.synchronize()
    ours = ycl[..., :Cout].permute(0, 4, 1, 2, 3).double().cpu()
    assert max_abs(ours, y.detach()) <= 1e-2 * y.abs().max().item(), max_abs(ours, y.detach())
    gcl = _to_cl_bf(gy)
    dx = torch.full((B, X, Y, Z, _rup8(Cin)), float('nan'), device='cuda', dtype=torch.bfloat16)
    _lib.check(L.hcu_conv_dgrad_cl(ctypes.byref(d), _lib.ptr(gcl), _lib.ptr(wd), _lib.ptr(dx),
                                   _lib.ptr(sc), sc.numel(), stream()))
    torch.cuda.synchronize()
    got = dx[..., :Cin].permute(0, 4, 1, 2, 3).double().cpu()
    assert max_abs(got, xr.grad) <= 1e-2 * xr.grad.abs().max().item(), max_abs(got, xr.grad)
    dw = torch.full_like(wd, float('nan'))
    db = torch.full_like(bd, float('nan'))
    _lib.check(L.hcu_conv_wgrad_cl(ctypes.byref(d), _lib.ptr(xcl), _lib.ptr(gcl), _lib.ptr(dw),
                                   _lib.ptr(db), _lib.ptr(sc), sc.numel(), stream()))
    torch.cuda.synchronize()
    assert max_abs(dw.cpu(), wr.grad) <= 1e-4 * wr.grad.abs().max().item(), max_abs(dw.cpu(), wr.grad)
    assert max_abs(db.cpu(), br.grad) <= 1e-4 * br.grad.abs().max().item()
