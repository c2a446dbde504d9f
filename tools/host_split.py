"""Host enqueue time of each phase of one training step, enqueued onto an
idle, synchronised queue (no backpressure): zero_grad, forward, loss,
backward, allreduce, optimizer step.   python tools/host_split.py [--config 2]"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
import hcunet_amd  # noqa: E402
from hcat.loss import cross_entropy  # noqa: E402
from hcat.unet import Unet_Constructor  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--config', default='2')
ap.add_argument('--steps', type=int, default=15)
args = ap.parse_args()
cfg = bench.CONFIGS[args.config]
dev = torch.device('cuda', 0)
torch.manual_seed(0)
m = Unet_Constructor(**cfg['kw']).to(dev).train()
opt = hcunet_amd.optim.Adam(m.parameters(), lr=1e-3)
x, mask, pwl = bench.synth_inputs(cfg['batch'], 1000, dev)
bf16 = cfg['dtype'] == 'bf16'
from hcunet_amd import _lib  # noqa: E402
L = _lib.lib()
native = {}


def _wrap(name):
    f = getattr(L, name)
    native[name] = []

    def w(*a):
        t0 = time.perf_counter()
        r = f(*a)
        native[name].append((time.perf_counter() - t0) * 1e3)
        return r
    setattr(L, name, w)


for _n in ('hcu_unet_forward', 'hcu_unet_backward', 'hcu_adam_step', 'hcu_loss_pixel_fwd'):
    _wrap(_n)
ph = {k: [] for k in ('zero_grad', 'forward', 'loss', 'backward', 'allreduce', 'adam', 'total')}
for it in range(args.steps + 3):
    torch.cuda.synchronize()
    t = [time.perf_counter()]
    opt.zero_grad()
    t.append(time.perf_counter())
    with torch.autocast('cuda', dtype=torch.bfloat16, enabled=bf16):
        out = m(x)
        t.append(time.perf_counter())
        loss = cross_entropy(out, mask, pwl, method='pixel')
    t.append(time.perf_counter())
    loss.backward()
    t.append(time.perf_counter())
    hcunet_amd.dist.allreduce_gradients(m)
    t.append(time.perf_counter())
    opt.step()
    t.append(time.perf_counter())
    if it >= 3:
        for k, a, b in zip(list(ph)[:-1], t[:-1], t[1:]):
            ph[k].append((b - a) * 1e3)
        ph['total'].append((t[-1] - t[0]) * 1e3)
torch.cuda.synchronize()
zg = []
for _ in range(20):
    for p in m.parameters():
        p.grad = torch.zeros_like(p)
    t0 = time.perf_counter()
    opt.zero_grad()
    zg.append((time.perf_counter() - t0) * 1e3)
print('zero_grad alone (grads attached, no sync before): median %.3f ms' % statistics.median(zg))
for k, v in native.items():
    if v:
        print('  native %-20s calls/step %.1f  median %.3f ms' % (k, len(v) / (args.steps + 3), statistics.median(v)))
print('config %s host enqueue per phase, idle queue (median ms over %d steps):' % (args.config, args.steps))
for k, v in ph.items():
    print('  %-10s %.3f' % (k, statistics.median(v)))
