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
