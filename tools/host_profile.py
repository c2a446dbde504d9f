#!/usr/bin/env python3
"""Host-side cost of one training step (what the CPU spends enqueueing
zero_grad / forward / loss / backward / Adam), with cProfile.

  python tools/host_profile.py [--config 2] [--steps 30]
"""
import argparse
import cProfile
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import hcunet_amd  # noqa: E402
from hcat.loss import cross_entropy  # noqa: E402
from hcat.unet import Unet_Constructor  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='2')
    ap.add_argument('--steps', type=int, default=30)
    a = ap.parse_args()
    cfg = bench.CONFIGS[a.config]
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    model = Unet_Constructor(**cfg['kw']).to(dev).train()
    opt = hcunet_amd.optim.Adam(model.parameters(), lr=1e-3)
    x, mask, pwl = bench.synth_inputs(cfg['batch'], 1000, dev)
    bf16 = cfg['dtype'] == 'bf16'

    def step():
        opt.zero_grad()
        with torch.autocast('cuda', dtype=torch.bfloat16, enabled=bf16):
            out = model(x)
            loss = cross_entropy(out, mask, pwl, method='pixel')
        loss.backward()
        opt.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    # host enqueue time with the GPU far behind (no sync inside)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    print('host enqueue %.3f ms/step, wall %.3f ms/step' % (t_enq / a.steps * 1e3, t_all / a.steps * 1e3))
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.steps):
        step()
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats('tottime').print_stats(25)


if __name__ == '__main__':
    main()
