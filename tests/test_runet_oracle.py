"""The r_unet.py oracle restatement (oracle/runet_oracle.py) pinned to the
reference's own outputs, losses and gradients (tests/golden/runet_*.npz,
made by running /root/reference/hcat/r_unet.py): CPU, fp32 and fp64."""
import os

import numpy as np
import pytest
import torch

from hcat.r_unet import RDCNet, RecursiveUnet
from oracle import inputs, loss_oracle as lo, runet_oracle as ro

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def _summary(t):
    t = t.detach().double().reshape(-1)
    idx = (inputs.splitmix64(99, 64) % np.uint64(t.numel())).astype(np.int64)
    return np.concatenate([[t.sum().item(), t.norm().item(), t.abs().max().item()],
                           t[torch.from_numpy(idx)].numpy()])


def _step(fwd, net, g, dtype):
    s = ro.state_of(net, dtype)
    x = torch.from_numpy(inputs.make_x(tuple(g['x_shape']))).to(dtype)
    out = fwd(s, x)
    oshape = tuple(out.shape)
    mshape = (oshape[0], 1) + oshape[2:]
    mask = torch.from_numpy(inputs.make_mask(mshape)).to(dtype)
    pwl = torch.from_numpy(inputs.make_pwl(mshape))
    vec = torch.from_numpy(g['vec']).to(dtype)
    loss = lo.cross_entropy(out[:, 0:1], mask, pwl, method='pixel') + lo.MSELoss(out[:, 2:], vec)
    loss.backward()
    return s, out.detach(), loss.item()


@pytest.mark.parametrize('tag,dtype,tol', [('f32', torch.float32, 1e-5), ('f64', torch.float64, 1e-10)])
def test_rdcnet_oracle_matches_reference(tag, dtype, tol):
    g = np.load(os.path.join(GOLD, 'runet_rdc.npz'))
    torch.manual_seed(int(g['seed']))
    net = RDCNet(4, 5)
    s, out, loss = _step(ro.rdcnet_forward, net, g, dtype)
    np.testing.assert_allclose(out.numpy(), g[tag + '.out'], rtol=0, atol=tol * 10)
    assert abs(loss - float(g[tag + '.loss'])) <= tol * 10
    for k, _ in net.named_parameters():
        ref = g[tag + '.grad.' + k]
        np.testing.assert_allclose(s[k].grad.numpy(), ref, rtol=0, atol=tol * max(1.0, np.abs(ref).max()),
                                   err_msg=k)


@pytest.mark.parametrize('tag,dtype,tol', [('f32', torch.float32, 1e-4), ('f64', torch.float64, 1e-9)])
def test_recursive_unet_oracle_matches_reference(tag, dtype, tol):
    g = np.load(os.path.join(GOLD, 'runet_rec.npz'))
    torch.manual_seed(int(g['seed']))
    net = RecursiveUnet(image_dimensions=3)
    s, out, loss = _step(lambda st, x: ro.runet_forward(st, x, training=True), net, g, dtype)
    np.testing.assert_allclose(out.numpy(), g[tag + '.out'], rtol=0, atol=tol)
    assert abs(loss - float(g[tag + '.loss'])) <= tol
    for k, _ in net.named_parameters():
        ref = g[tag + '.grad.' + k]
        np.testing.assert_allclose(_summary(s[k].grad), ref, rtol=0, atol=tol * max(1.0, np.abs(ref).max()),
                                   err_msg=k)
    for k, _ in net.named_buffers():
        np.testing.assert_allclose(s[k].double().numpy(), g[tag + '.buf.' + k], rtol=0, atol=tol, err_msg=k)
