#!/usr/bin/env python3
"""Per-layer kernel-time breakdown of the config-2 training step (HIP events
around every library launch, tagged by network layer and phase).

  python tools/layer_profile.py [--steps K] [--json out.json]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from hcat.loss import cross_entropy  # noqa: E402
from hcat.unet import Unet_Constructor  # noqa: E402
import hcunet_amd  # noqa: E402
from hcunet_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--config', default='2')
    ap.add_argument('--json', default=None)
    a = ap.parse_args()
    cfg = bench.CONFIGS[a.config]
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    m = Unet_Constructor(**cfg['kw']).to(dev).train()
    opt = hcunet_amd.optim.Adam(m.parameters(), lr=1e-3)
    x, mask, pwl = bench.synth_inputs(cfg['batch'], 1000, dev)

    bf16 = cfg.get('dtype') == 'bf16'

    def step():
        opt.zero_grad()
        with torch.autocast('cuda', dtype=torch.bfloat16, enabled=bf16):
            loss = cross_entropy(m(x), mask, pwl, method='pixel')
        loss.backward()
        opt.step()
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    L = _lib.lib()
    L.hcu_timing_enable(a.steps * 1024)
    L.hcu_timing_detail(1)
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    rep = _lib.timing_report()
    L.hcu_timing_disable()
    rows = []
    for k, v in rep.items():
        kern, _, tag = k.partition('@')
        rows.append(dict(kernel=kern, tag=tag or '-', n=v['count'] / a.steps, us=v['ms'] * 1e3 / a.steps,
                         gflops=v['flops'] / a.steps / 1e9, mb=v['bytes'] / a.steps / 1e6))
    rows.sort(key=lambda r: -r['us'])
    tot = sum(r['us'] for r in rows)
    print('total kernel time per step: %.1f us, launches %d' % (tot, sum(r['n'] for r in rows)))
    print('%-34s %-14s %5s %9s %6s %8s %8s' % ('kernel', 'layer', 'n', 'us', '%', 'TF/s', 'GB/s'))
    for r in rows:
        tf = r['gflops'] / r['us'] * 1e3 if r['us'] > 0 else 0   # GF/us = PF/s
        gb = r['mb'] / r['us'] * 1e3 if r['us'] > 0 else 0       # MB/us = TB/s
        print('%-34s %-14s %5.1f %9.1f %6.2f %8.2f %8.1f' % (r['kernel'][:34], r['tag'], r['n'], r['us'],
                                                            100 * r['us'] / tot, tf, gb))
    by_phase = {}
    for r in rows:
        ph = r['tag'].split('.')[-1]
        by_phase[ph] = by_phase.get(ph, 0) + r['us']
    print('by phase:', {k: round(v, 1) for k, v in sorted(by_phase.items(), key=lambda kv: -kv[1])})
    if a.json:
        with open(a.json, 'w') as f:
            json.dump(rows, f, indent=1)


if __name__ == '__main__':
    main()
