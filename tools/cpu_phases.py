#!/usr/bin/env python3
"""Host-side (CPU) time of each phase of the training step, without syncs:
how long Python + the launch path take to enqueue each part of the step."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from hcat.loss import cross_entropy  # noqa: E402
from hcat.unet import Unet_Constructor  # noqa: E402
import hcunet_amd  # noqa: E402


def main():
    cfg = bench.CONFIGS['2']
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    m = Unet_Constructor(**cfg['kw']).to(dev).train()
    opt = hcunet_amd.optim.Adam(m.parameters(), lr=1e-3)
    x, mask, pwl = bench.synth_inputs(cfg['batch'], 1000, dev)
    acc = {}
    for it in range(30):
        t = [time.perf_counter()]
        opt.zero_grad()
        t.append(time.perf_counter())
        out = m(x)
        t.append(time.perf_counter())
        loss = cross_entropy(out, mask, pwl, method='pixel')
        t.append(time.perf_counter())
        loss.backward()
        t.append(time.perf_counter())
        opt.step()
        t.append(time.perf_counter())
        if it >= 10:
            for k, name in enumerate(['zero_grad', 'forward', 'loss', 'backward', 'adam']):
                acc[name] = acc.get(name, 0.0) + (t[k + 1] - t[k]) * 1e6 / 20
    torch.cuda.synchronize()
    print('host us per phase:', {k: round(v, 1) for k, v in acc.items()}, 'total', round(sum(acc.values()), 1))


if __name__ == '__main__':
    main()
