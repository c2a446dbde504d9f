#!/usr/bin/env python3
"""Per-parameter gradient error of one GPU training step vs the fp64/fp32
oracle (debug aid): prints err/tol for every parameter."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests.test_gpu_unet import CONFIGS, _build, _mask_pwl, _oshape, _bn_cancelled  # noqa
from hcat.loss import cross_entropy  # noqa
from oracle import unet_oracle as uo  # noqa

name = sys.argv[1] if len(sys.argv) > 1 else 'l5_min'
kw, shape = CONFIGS[name]
m, spec, state, x = _build(kw, shape)
osh = _oshape(spec, state, x)
ref32 = uo.train_step(spec, state, x, *_mask_pwl(osh), dtype=torch.float32)
ref64 = uo.train_step(spec, state, x, *_mask_pwl(osh), dtype=torch.float64)
mask, pwl = _mask_pwl(osh)
m = m.cuda().train()
out = m(torch.from_numpy(x).cuda())
loss = cross_entropy(out, torch.from_numpy(mask).cuda(), torch.from_numpy(pwl).cuda())
loss.backward()
torch.cuda.synchronize()
print('out err', (out.detach().cpu().double() - ref32['out'].double()).abs().max().item())
for n, p in m.named_parameters():
    g = p.grad.detach().cpu().double()
    g64 = ref64['grads'][n].double()
    g32 = ref32['grads'][n].double()
    err = (g - g64).abs().max().item()
    noise = (g32 - g64).abs().max().item()
    idx = (g - g64).abs().argmax().item()
    nrm = g64.norm().item()
    rl2 = (g - g64).norm().item() / max(nrm, 1e-30)
    rl32 = (g32 - g64).norm().item() / max(nrm, 1e-30)
    print('%-32s err %.3e  ref32-noise %.3e  max|g| %.3e  ratio %.2f  relL2 %.2e ref32 %.2e' % (
        n, err, noise, g64.abs().max().item(), err / max(noise, 1e-30), rl2, rl32))

if len(sys.argv) > 2:
    n = sys.argv[2]
    p = dict(m.named_parameters())[n]
    d = (p.grad.detach().cpu().double() - ref64['grads'][n].double()).abs()
    d32 = (ref32['grads'][n].double() - ref64['grads'][n].double()).abs()
    print('per output channel max err:', [round(v, 7) for v in d.reshape(d.shape[0], -1).max(1).values.tolist()])
    print('per output channel max ref32 noise:', [round(v, 7) for v in d32.reshape(d.shape[0], -1).max(1).values.tolist()])
