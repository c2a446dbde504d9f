#!/usr/bin/env python3
"""Generate tests/golden/runet_*.npz and unet_blocks.npz from the REFERENCE
implementation itself (development container only; /root/reference).

hcat/r_unet.py imports only torch: it is imported through the
same namespace shim as make_golden.py, with torch.Tensor.cuda patched to the
identity for the CPU run (the reference hard-codes .cuda() at r_unet.py:141,
152, 223).  Nothing from the reference is copied: the fixtures hold the
reference modules' own seeded initial weights, the seeded inputs and the
reference's outputs / losses / gradients (fp32 and fp64 runs), and the
BatchNorm running statistics after the training forward.

Training step recorded (reference pattern tests/r_unet_test.py:48-56):
  out = net(x); loss = cross_entropy(out[:, 0:1], mask, pwl, method='pixel')
  + MSELoss(out[:, 2:], vector); loss.backward().

Usage:  python tests/golden/make_runet_golden.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import importlib  # noqa: E402

from make_golden import import_reference  # noqa: E402
from oracle import inputs  # noqa: E402


def import_runet():
    unet, loss = import_reference()
    torch.Tensor.cuda = lambda self, *a, **k: self   # CPU run of the reference's .cuda() calls
    runet = importlib.import_module('hcat.r_unet')
    return runet, unet, loss


def run(net, loss_mod, x, mask, pwl, vec, dtype, train=True, noise=None):
    net = net.to(dtype).train(train)
    xx = torch.from_numpy(x).to(dtype)
    if noise is not None:   # (seed, relative amplitude): sensitivity probe
        gen = torch.Generator().manual_seed(noise[0])
        xx = xx * (1 + noise[1] * torch.randn(xx.shape, generator=gen, dtype=dtype))
    net.zero_grad()
    out = net(xx)
    lp = loss_mod.cross_entropy(out[:, 0:1], torch.from_numpy(mask).to(dtype),
                                torch.from_numpy(pwl), method='pixel')
    lv = loss_mod.MSELoss(out[:, 2:], torch.from_numpy(vec).to(dtype))
    loss = lp + lv
    loss.backward()
    grads = {k: p.grad.detach().clone() for k, p in net.named_parameters()}
    bufs = {k: b.detach().clone() for k, b in net.named_buffers()}
    return out.detach(), loss.detach(), grads, bufs


def summary(t):
    """Size-independent digest: sum, L2 norm, max|.|, 64 hashed samples."""
    t = t.detach().double().reshape(-1)
    idx = (inputs.splitmix64(99, 64) % np.uint64(t.numel())).astype(np.int64)
    return np.concatenate([[t.sum().item(), t.norm().item(), t.abs().max().item()],
                           t[torch.from_numpy(idx)].numpy()])


def record(name, make, shape, seed, full=True, eval_too=False, sens=0):
    """full=False: weights and gradients as digests (summary) -- the weights are
    re-created on the GPU side from the same seed (the drop-in modules
    reproduce torch's default initialisation in the reference's order)."""
    runet, unet, loss = import_runet()
    torch.manual_seed(seed)
    net = make(runet)
    state = {k: v.detach().clone() for k, v in net.state_dict().items()}
    x = inputs.make_x(shape)
    with torch.no_grad():
        oshape = tuple(make(runet).eval()(torch.from_numpy(x)).shape)
    mshape = (oshape[0], 1) + oshape[2:]
    mask = inputs.make_mask(mshape)
    pwl = inputs.make_pwl(mshape)
    vec = (inputs.make_x((oshape[0], oshape[1] - 2) + oshape[2:]) * 0.5).astype(np.float32)
    rec = {'x_shape': np.array(shape), 'out_shape': np.array(oshape)}
    rec['seed'] = np.array(seed)
    for k, v in state.items():
        rec['init.' + k] = v.numpy() if full else summary(v)
    for tag, dt in (('f32', torch.float32), ('f64', torch.float64)):
        net = make(runet)
        net.load_state_dict(state)
        out, ls, grads, bufs = run(net, loss, x, mask, pwl, vec, dt)
        rec[tag + '.out'] = out.numpy()
        rec[tag + '.loss'] = np.array(ls.item())
        for k, g in grads.items():
            rec[tag + '.grad.' + k] = g.numpy() if full else summary(g)
        for k, b in bufs.items():
            rec[tag + '.buf.' + k] = b.numpy()
    # eval mode (BatchNorm on the running statistics): the gradients no longer
    # pass ten steps of batch statistics, so they are not noise-amplified
    for tag, dt in ((('e32', torch.float32), ('e64', torch.float64)) if eval_too else ()):
        net = make(runet)
        net.load_state_dict(state)
        out, ls, grads, _ = run(net, loss, x, mask, pwl, vec, dt, train=False)
        rec[tag + '.out'] = out.numpy()
        rec[tag + '.loss'] = np.array(ls.item())
        for k, g in grads.items():
            rec[tag + '.grad.' + k] = g.numpy() if full else summary(g)
    # sensitivity envelope of the train-mode gradients: the reference's own
    # fp32 run with the input perturbed by 1e-6 relative noise (the size of a
    # reordered fp32 reduction's rounding), `sens` seeds; per tensor the
    # largest digest relative L2 against the unperturbed fp64 run
    for k in (grads.keys() if sens else ()):
        rec['sens.grad.' + k] = np.array(0.0)
    for s in range(sens):
        net = make(runet)
        net.load_state_dict(state)
        _, _, grads, _ = run(net, loss, x, mask, pwl, vec, torch.float32, noise=(100 + s, 1e-6))
        for k, g in grads.items():
            d, d64 = summary(g), rec['f64.grad.' + k]
            d64 = d64 if not full else summary(torch.from_numpy(d64))
            r = np.linalg.norm(d - d64) / max(np.linalg.norm(d64), 1e-12)
            rec['sens.grad.' + k] = np.maximum(rec['sens.grad.' + k], r)
    rec['vec'] = vec
    path = os.path.join(HERE, name + '.npz')
    np.savez_compressed(path, **rec)
    print('wrote', path, 'out', oshape, 'loss', rec['f32.loss'], 'f64', rec['f64.loss'])


def record_blocks():
    """Down / Up blocks of a reference Unet_Constructor called on their own
    (hcat/unet.py:263-266, 309-315), train mode, fp32 and fp64."""
    _, unet, _ = import_runet()
    kw = dict(image_dimensions=3, in_channels=4, out_channels=1, feature_sizes=[4, 8, 16],
              kernel={'conv1': (3, 3, 2), 'conv2': (3, 3, 1)}, upsample_kernel=(2, 2, 2),
              max_pool_kernel=(2, 2, 1), upsample_stride=(2, 2, 1))
    torch.manual_seed(5)
    net = unet.Unet_Constructor(**kw)
    state = {k: v.detach().clone() for k, v in net.state_dict().items()}
    xd = inputs.make_x((2, 4, 20, 18, 5))
    xu = inputs.make_x((2, 16, 6, 7, 3))
    skip = (2, 8, 14, 16, 6)
    rec = {'xd_shape': np.array(xd.shape), 'xu_shape': np.array(xu.shape), 'skip': np.array(skip)}
    for k, v in state.items():
        rec['init.' + k] = v.numpy()
    for tag, dt in (('f32', torch.float32), ('f64', torch.float64)):
        net = unet.Unet_Constructor(**kw)
        net.load_state_dict(state)
        net = net.to(dt).train()
        d, u = net.down_steps[0], net.up_steps[0]
        xdt = torch.from_numpy(xd).to(dt).requires_grad_(True)
        od = d(xdt)
        gd = torch.from_numpy(inputs.make_x(tuple(od.shape))).to(dt)
        (od * gd).sum().backward()
        rec[tag + '.down.out'] = od.detach().numpy()
        rec[tag + '.down.dx'] = xdt.grad.numpy()
        for k, p in d.named_parameters():
            rec[tag + '.down.grad.' + k] = p.grad.numpy()
        for k, b in d.named_buffers():
            rec[tag + '.down.buf.' + k] = b.numpy()
        xut = torch.from_numpy(xu).to(dt).requires_grad_(True)
        ou = u(xut, torch.zeros(skip, dtype=dt))
        gu = torch.from_numpy(inputs.make_x(tuple(ou.shape))).to(dt)
        (ou * gu).sum().backward()
        rec[tag + '.up.out'] = ou.detach().numpy()
        rec[tag + '.up.dx'] = xut.grad.numpy()
        for k, p in u.named_parameters():
            rec[tag + '.up.grad.' + k] = p.grad.numpy()
        for k, b in u.named_buffers():
            rec[tag + '.up.buf.' + k] = b.numpy()
    path = os.path.join(HERE, 'unet_blocks.npz')
    np.savez_compressed(path, **rec)
    print('wrote', path)


if __name__ == '__main__':
    record('runet_rdc', lambda m: m.RDCNet(4, 5), (1, 4, 24, 24, 10), 0)
    record('runet_rec', lambda m: m.RecursiveUnet(image_dimensions=3), (1, 4, 16, 16, 4), 1, full=False,
           eval_too=True, sens=16)
    record_blocks()
