"""Host slack of the config-2 train step: the same loop as bench.py with a
host-side busy wait of S ms inserted at one point of every step.  If the step
time stays flat as S grows, the GPU is the bottleneck; the S at which it starts
to grow is the host's slack.  Also times the host enqueue of each phase.

  python tools/host_slack.py [--config 2] [--where end|mid] [--sleeps 0,0.3,0.6]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import hcunet_amd  # noqa: E402
from hcat.loss import cross_entropy  # noqa: E402
from hcat.unet import Unet_Constructor  # noqa: E402


def spin(ms):
    t = time.perf_counter() + ms * 1e-3
    while time.perf_counter() < t:
        pass


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='2')
    ap.add_argument('--steps', type=int, default=30)
    ap.add_argument('--sleeps', default='0,0.2,0.4,0.6,0.8,1.0')
    ap.add_argument('--where', default='end', choices=['end', 'mid'])
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    cfg = bench.CONFIGS[args.config]
    torch.manual_seed(0)
    model = Unet_Constructor(**cfg['kw']).to(dev).train()
    opt = hcunet_amd.optim.Adam(model.parameters(), lr=1e-3)
    x, mask, pwl = bench.synth_inputs(cfg['batch'], 1000, dev)
    bf16 = cfg['dtype'] == 'bf16'
    ph = {'fwd': 0.0, 'bwd': 0.0, 'opt': 0.0}

    def step(s_ms):
        t0 = time.perf_counter()
        opt.zero_grad()
        with torch.autocast('cuda', dtype=torch.bfloat16, enabled=bf16):
            out = model(x)
            loss = cross_entropy(out, mask, pwl, method='pixel')
        t1 = time.perf_counter()
        if args.where == 'mid':
            spin(s_ms)
        t2 = time.perf_counter()
        loss.backward()
        t3 = time.perf_counter()
        opt.step()
        if args.where == 'end':
            spin(s_ms)
        t4 = time.perf_counter()
        ph['fwd'] += t1 - t0
        ph['bwd'] += t3 - t2
        ph['opt'] += t4 - t3 - (s_ms * 1e-3 if args.where == 'end' else 0)

    for s in [float(v) for v in args.sleeps.split(',')]:
        for _ in range(5):
            step(s)
        torch.cuda.synchronize()
        for k in ph:
            ph[k] = 0.0
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step(s)
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / args.steps * 1e3
        print('spin %.2f ms (%s): %.3f ms/step  host fwd %.3f bwd %.3f opt %.3f ms' %
              (s, args.where, el, ph['fwd'] / args.steps * 1e3, ph['bwd'] / args.steps * 1e3,
               ph['opt'] / args.steps * 1e3), flush=True)


if __name__ == '__main__':
    main()
