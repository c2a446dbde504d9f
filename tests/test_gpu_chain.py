"""Single-op layer chains (hcunet_amd.chain, hcu_chain_* C-ABI) vs the same
op in torch on the CPU (fp64 autograd): forward, input gradient and
weight / bias gradients of Conv3d with stride / padding / dilation (the
r_unet.py layers, including dilated 5^3 kernels that run on their dilation
sub-lattices), ConvTranspose3d with padding (crop) and Conv3d + BatchNorm +
ReLU + MaxPool sequences."""
import copy

import pytest
import torch
import torch.nn as nn

from hcunet_amd.chain import Chain, FlatParams

pytestmark = pytest.mark.gpu


class _Holder(nn.Module):
    def __init__(self, *mods):
        super().__init__()
        self.m = nn.ModuleList(mods)


def _run(mods, ops, x, need_dx=True, training=True):
    """GPU chain vs CPU fp64 torch of the same modules; returns errors."""
    gpu = [copy.deepcopy(m).float() for m in mods]
    cpu = [m.double() for m in mods]
    xc = x.double().clone().requires_grad_(need_dx)
    y = xc
    for op, m in zip(ops, cpu):
        if op == 'pool':
            y = m(y)
        elif op == 'bnrelu':
            y = torch.relu(m(y))
        else:
            y = m(y)
    g = torch.randn(y.shape, dtype=torch.float64, generator=torch.Generator().manual_seed(9))
    (y * g).sum().backward()
    holder = _Holder(*gpu).cuda()
    for m in holder.m:
        m.zero_grad(set_to_none=True)
    flat = FlatParams(holder)
    spec = []
    i = 0
    while i < len(ops):
        op, m = ops[i], holder.m[i]
        if op in ('conv', 'conv_fold'):
            bn = holder.m[i + 1] if i + 1 < len(ops) and ops[i + 1] == 'bnrelu' else None
            spec.append(('conv', m, bn, op == 'conv_fold'))
            i += 2 if bn is not None else 1
        elif op == 'convt':
            spec.append(('convt', m))
            i += 1
        elif op == 'pool':
            spec.append(('pool', tuple(m.kernel_size) if not isinstance(m.kernel_size, int)
                         else (m.kernel_size,) * 3))
            i += 1
    ch = Chain(flat, x.shape[1], spec)
    xg = x.float().cuda().requires_grad_(need_dx)
    out = ch(xg, training, False)
    (out * g.float().cuda()).sum().backward()
    torch.cuda.synchronize()
    errs = {'out': ((out.detach().cpu().double() - y.detach()).abs().max().item(), y.abs().max().item())}
    if need_dx:
        errs['dx'] = ((xg.grad.cpu().double() - xc.grad).abs().max().item(), xc.grad.abs().max().item())
    for (k, p), (_, q) in zip(holder.named_parameters(), [(k, q) for k, q in
                                                           _Holder(*cpu).named_parameters()]):
        errs[k] = ((p.grad.cpu().double() - q.grad).abs().max().item(), q.grad.abs().max().item())
    return errs


def _check(errs, rel=2e-5, cancelled=()):
    """cancelled: biases feeding a train-mode BatchNorm -- their exact gradient
    is 0 and fp32 returns rounding noise: absolute 1e-4."""
    bad = {k: v for k, v in errs.items()
           if (v[0] > 1e-4 if k in cancelled else v[0] > rel * max(v[1], 1e-3))}
    assert not bad, bad


@pytest.mark.parametrize('k,s,p,d,cin,cout,shape', [
    (3, 2, 1, 1, 4, 10, (1, 4, 24, 24, 10)),      # RDCNet.strided_conv (r_unet.py:213)
    (3, 1, 1, 1, 10, 10, (1, 10, 12, 12, 5)),     # RDCNet.out_conv (:215)
    (1, 1, 0, 1, 20, 10, (1, 20, 12, 12, 5)),     # RDCBlock.conv (:372)
    (5, 1, 2, 1, 10, 10, (1, 10, 12, 12, 5)),     # StackedDilation.conv1 (:348)
    (5, 1, 6, 3, 10, 10, (1, 10, 12, 12, 5)),     # conv3: dilation 3 (sub-lattices)
    (5, 1, 10, 5, 10, 10, (1, 10, 16, 14, 7)),    # conv5: dilation 5
    (3, 1, 1, 1, 9, 16, (1, 9, 16, 16, 4)),       # RecursiveUnet Down conv (:262)
])
def test_conv_chain(k, s, p, d, cin, cout, shape):
    conv = nn.Conv3d(cin, cout, k, stride=s, padding=p, dilation=d)
    x = torch.randn(shape, generator=torch.Generator().manual_seed(1))
    _check(_run([conv], ['conv'], x, need_dx=(s == 1)))


@pytest.mark.parametrize('k,s,p,cin,cout,shape', [
    ((4, 4, 4), (2, 2, 2), (1, 1, 1), 10, 5, (1, 10, 12, 12, 5)),   # RDCNet.transposed_conv (:216)
    ((6, 6, 5), (2, 2, 1), (2, 2, 2), 64, 32, (1, 64, 4, 4, 4)),    # RecursiveUnet up_conv (:319)
    ((2, 2, 2), (2, 2, 1), (0, 0, 0), 16, 8, (2, 16, 5, 6, 3)),     # Unet_Constructor up_conv
])
def test_convt_chain(k, s, p, cin, cout, shape):
    ct = nn.ConvTranspose3d(cin, cout, k, stride=s, padding=p)
    x = torch.randn(shape, generator=torch.Generator().manual_seed(2))
    _check(_run([ct], ['convt'], x))


def test_down_pool_chain():
    mods = [nn.Conv3d(9, 16, 3, padding=1), nn.BatchNorm3d(16), nn.Conv3d(16, 16, 3, padding=1),
            nn.BatchNorm3d(16), nn.MaxPool3d((2, 2, 1))]
    x = torch.randn((1, 9, 16, 16, 4), generator=torch.Generator().manual_seed(4))
    _check(_run(mods, ['conv', 'bnrelu', 'conv', 'bnrelu', 'pool'], x), rel=1e-4,
           cancelled=('m.0.bias', 'm.2.bias'))


def _to_cl(t, cs, dtype):
    """NCXYZ -> [B, X, Y, Z, cs] with zero padding channels."""
    v = t.permute(0, 2, 3, 4, 1)
    return torch.nn.functional.pad(v, (0, cs - t.shape[1])).to(dtype).contiguous()


@pytest.mark.parametrize('bf16', [False, True])
def test_channels_last_boundaries_and_parts(bf16):
    """Chain in_cl / out_cl / in_part (the RDCNet recurrence's hand-over,
    include/hcunet.h hcu_chain_spec): a 1x1 Conv3d (2C -> C, C = 10) on the
    channel-wise cat of two padded channels-last tensors, then a dilated 5^3
    Conv3d (its sub-lattice form) channels-last in and out, against the same
    two chains on NCXYZ tensors: outputs, the gradients of both inputs and
    every weight / bias gradient, to the precision of the compute dtype."""
    from hcunet_amd.chain import cl_channels
    torch.manual_seed(3)
    C = 10
    c1 = nn.Conv3d(2 * C, C, 1)
    c2 = nn.Conv3d(C, C, 5, dilation=4, padding=8)
    shape = (1, C, 40, 36, 12)
    a = torch.randn(shape)
    b = torch.randn(shape)
    g = torch.randn(shape)
    dt = torch.bfloat16 if bf16 else torch.float32
    cs = cl_channels(C, bf16)
    res = {}
    for mode in ('nc', 'cl'):
        holder = _Holder(copy.deepcopy(c1), copy.deepcopy(c2)).cuda()
        flat = FlatParams(holder)
        m1, m2 = holder.m
        if mode == 'nc':
            k1 = Chain(flat, 2 * C, [('conv', m1, None, False)])
            k2 = Chain(flat, C, [('conv', m2, None, False)])
            xa, xb = a.cuda().requires_grad_(True), b.cuda().requires_grad_(True)
            y = k2(k1(torch.cat((xa, xb), 1), True, bf16), True, bf16)
            (y * g.cuda()).sum().backward()
            res[mode] = (y.detach().cpu(), xa.grad.cpu(), xb.grad.cpu(),
                         [p.grad.cpu() for p in holder.parameters()])
        else:
            k1 = Chain(flat, 2 * C, [('conv', m1, None, False)], in_cl=True, out_cl=True, in_part=C)
            k2 = Chain(flat, C, [('conv', m2, None, False)], in_cl=True, out_cl=True)
            xa = _to_cl(a.cuda(), cs, dt).requires_grad_(True)
            xb = _to_cl(b.cuda(), cs, dt).requires_grad_(True)
            y = k2(k1(torch.cat((xa, xb), -1), True, bf16), True, bf16)
            assert y.shape == (1,) + shape[2:] + (cs,) and y.dtype == dt
            assert not y[..., C:].any()   # padding channels stay zero
            (y.float() * _to_cl(g.cuda(), cs, torch.float32)).sum().backward()
            back = lambda t: t[..., :C].float().permute(0, 4, 1, 2, 3).cpu()   # noqa: E731
            assert not xa.grad[..., C:].any() and not xb.grad[..., C:].any()
            res[mode] = (back(y.detach()), back(xa.grad), back(xb.grad),
                         [p.grad.cpu() for p in holder.parameters()])
    tol = 3e-2 if bf16 else 1e-4
    (y0, da0, db0, g0), (y1, da1, db1, g1) = res['nc'], res['cl']
    for name, u, v in [('out', y0, y1), ('dA', da0, da1), ('dB', db0, db1)] + \
            [('grad%d' % i, u, v) for i, (u, v) in enumerate(zip(g0, g1))]:
        err = (u.float() - v.float()).abs().max().item()
        assert err <= tol * max(u.abs().max().item(), 1e-6), (name, err, u.abs().max().item())


@pytest.mark.parametrize('in_cl,swap', [(False, True), (True, True), (True, False)])
def test_convt_chain_bf16_padded_phase_columns(in_cl, swap, monkeypatch):
    """RDCNet's ConvTranspose3d (10 -> 5, k4, s2, p1; r_unet.py:216) on the
    bf16 path, where its 5 output channels are padded to 8 columns per stride
    phase (GConvArgs::cph: zero weights and bias in the padded columns), and
    its weight gradient taken as the Conv3d weight gradient of the
    input-gradient convolution (swap; HCU_CONVT_NOSWAP=1: the (tap, co)
    column form), against fp64 torch on the same bf16-representable input,
    weights and upstream gradient: output and input gradient to bf16 storage
    precision, weight / bias gradients (fp32 accumulation of exact products)
    to 2e-3."""
    from hcunet_amd.chain import cl_channels
    if not swap:
        monkeypatch.setenv('HCU_CONVT_NOSWAP', '1')
    torch.manual_seed(6)
    ct = nn.ConvTranspose3d(10, 5, 4, stride=2, padding=1)
    with torch.no_grad():
        ct.weight.copy_(ct.weight.bfloat16().float())
    x = torch.randn((1, 10, 20, 18, 6), generator=torch.Generator().manual_seed(7)).bfloat16().float()
    ref = copy.deepcopy(ct).double()
    xr = x.double().requires_grad_(True)
    y = ref(xr)
    g = torch.randn(y.shape, generator=torch.Generator().manual_seed(8)).bfloat16().double()
    (y * g).sum().backward()
    holder = _Holder(copy.deepcopy(ct)).cuda()
    ch = Chain(FlatParams(holder), 10, [('convt', holder.m[0])], in_cl=in_cl)
    if in_cl:
        xg = _to_cl(x.cuda(), cl_channels(10, True), torch.bfloat16).requires_grad_(True)
    else:
        xg = x.cuda().requires_grad_(True)
    out = ch(xg, True, True)
    assert out.shape == y.shape and out.dtype == torch.float32
    (out * g.float().cuda()).sum().backward()
    torch.cuda.synchronize()
    dx = xg.grad[..., :10].float().permute(0, 4, 1, 2, 3) if in_cl else xg.grad
    if in_cl:
        assert not xg.grad[..., 10:].any()
    m = holder.m[0]
    for name, got, want, tol in [('out', out.detach(), y.detach(), 1e-2), ('dx', dx, xr.grad, 1e-2),
                                 ('dW', m.weight.grad, ref.weight.grad, 2e-3),
                                 ('db', m.bias.grad, ref.bias.grad, 2e-3)]:
        err = (got.cpu().double() - want).abs().max().item()
        assert err <= tol * want.abs().max().item(), (name, err, want.abs().max().item())


@pytest.mark.parametrize('cin,cout,part', [(50, 10, 10), (20, 10, 10), (16, 16, 0)])
def test_pointwise_conv_chain_bf16(cin, cout, part):
    """The streaming 1x1x1 kernels (pwconv.hip) of the bf16 chains: RDCNet's
    mixing convolutions (StackedDilation.out_conv 50 -> 10 and RDCBlock.conv
    20 -> 10 on channel parts of 10 channels in 16 slots, r_unet.py:354-374)
    and a plain 16 -> 16 one, channels-last in and out, against fp64 torch on
    the same bf16-representable input, weights and upstream gradient: output
    and input gradient to bf16 storage precision, weight / bias gradients to
    2e-3; every padding slot of the output and of the input gradient 0."""
    from hcunet_amd.chain import cl_channels
    torch.manual_seed(11)
    conv = nn.Conv3d(cin, cout, 1)
    with torch.no_grad():
        conv.weight.copy_(conv.weight.bfloat16().float())
    shape = (1, cin, 24, 20, 6)
    x = torch.randn(shape, generator=torch.Generator().manual_seed(12)).bfloat16().float()
    ref = copy.deepcopy(conv).double()
    xr = x.double().requires_grad_(True)
    y = ref(xr)
    g = torch.randn(y.shape, generator=torch.Generator().manual_seed(13)).bfloat16().double()
    (y * g).sum().backward()
    holder = _Holder(copy.deepcopy(conv)).cuda()
    m = holder.m[0]
    if part:
        ps = cl_channels(part, True)
        xin = torch.cat([_to_cl(x[:, i:i + part].cuda(), ps, torch.bfloat16) for i in range(0, cin, part)], -1)
        ch = Chain(FlatParams(holder), cin, [('conv', m, None, False)], in_cl=True, out_cl=True, in_part=part)
    else:
        ps = cl_channels(cin, True)
        xin = _to_cl(x.cuda(), ps, torch.bfloat16)
        ch = Chain(FlatParams(holder), cin, [('conv', m, None, False)], in_cl=True, out_cl=True)
    xin = xin.requires_grad_(True)
    out = ch(xin, True, True)
    cs = cl_channels(cout, True)
    assert out.shape == (1,) + shape[2:] + (cs,) and out.dtype == torch.bfloat16
    assert not out[..., cout:].any()
    (out.float() * _to_cl(g.float().cuda(), cs, torch.float32)).sum().backward()
    torch.cuda.synchronize()
    got_y = out[..., :cout].float().permute(0, 4, 1, 2, 3)
    if part:
        parts = xin.grad.reshape(xin.shape[:-1] + (cin // part, ps))
        assert not parts[..., part:].any()
        dx = parts[..., :part].reshape(xin.shape[:-1] + (cin,)).float().permute(0, 4, 1, 2, 3)
    else:
        dx = xin.grad[..., :cin].float().permute(0, 4, 1, 2, 3)
    for name, got, want, tol in [('out', got_y, y.detach(), 1e-2), ('dx', dx, xr.grad, 1e-2),
                                 ('dW', m.weight.grad, ref.weight.grad, 2e-3),
                                 ('db', m.bias.grad, ref.bias.grad, 2e-3)]:
        err = (got.cpu().double() - want).abs().max().item()
        assert err <= tol * want.abs().max().item(), (name, err, want.abs().max().item())
