#!/usr/bin/env python3
"""Weight-gradient microbenchmark: one Conv3d wgrad (+ finalize) per call through
the C-ABI at the config-2 level shapes, per-kernel HIP-event times.

  python tools/wgrad_bench.py [--reps 20]   (HCU_W8_DBG / HCU_NO_WGRAD8 select variants)
"""
import argparse
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hcunet_amd import _lib  # noqa: E402
from tests.helpers import desc, out_dims, scratch_for, stream  # noqa: E402

SHAPES = {   # name: B, Cin, Cout, X, Y, Z, k
    'c3.d0.c2': (4, 32, 32, 254, 254, 15, (3, 3, 1)),    # config 3 (bf16 with --bf16)
    'c3.d1.c2': (4, 64, 64, 125, 125, 13, (3, 3, 1)),
    'c3.d1.c1': (4, 32, 64, 127, 127, 14, (3, 3, 2)),
    'd0.c1': (2, 4, 8, 256, 256, 16, (3, 3, 2)),
    'd0.c2': (2, 8, 8, 254, 254, 15, (3, 3, 1)),
    'd1.c1': (2, 8, 16, 127, 127, 14, (3, 3, 2)),
    'd1.c2': (2, 16, 16, 125, 125, 13, (3, 3, 1)),
    'd2.c2': (2, 32, 32, 59, 59, 13, (3, 3, 1)),       # the deep fp32 levels (wgrad3)
    'd3.c1': (2, 32, 64, 28, 28, 13, (3, 3, 2)),
    'd3.c2': (2, 64, 64, 26, 26, 12, (3, 3, 1)),
    'd4.c1': (2, 64, 128, 12, 12, 12, (3, 3, 2)),
    'd4.c2': (2, 128, 128, 10, 10, 11, (3, 3, 1)),
    'u1.c1': (2, 32, 32, 24, 24, 12, (3, 3, 2)),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('--only', default=None)
    ap.add_argument('--bf16', action='store_true')
    a = ap.parse_args()
    L = _lib.lib()
    for name, (B, Cin, Cout, X, Y, Z, k) in SHAPES.items():
        if a.only and name not in a.only.split(','):
            continue
        d = desc(B, Cin, Cout, X, Y, Z, k)
        q = 4
        if a.bf16:
            d.dtype = _lib.HCU_BF16
            q = 8
        od = out_dims(d)
        cs_in, cs_out = (Cin + q - 1) // q * q, (Cout + q - 1) // q * q
        dt = torch.bfloat16 if a.bf16 else torch.float32
        x = torch.randn(B, X, Y, Z, cs_in, device='cuda').to(dt)
        gy = torch.randn(B, *od, cs_out, device='cuda').to(dt)
        dw = torch.empty(Cout, Cin, *k, device='cuda')
        db = torch.empty(Cout, device='cuda')
        sc = scratch_for(d)
        args = (ctypes.byref(d), _lib.ptr(x), _lib.ptr(gy), _lib.ptr(dw), _lib.ptr(db), _lib.ptr(sc), sc.numel(),
                stream())
        for _ in range(3):
            _lib.check(L.hcu_conv_wgrad_cl(*args))
        torch.cuda.synchronize()
        L.hcu_timing_enable(a.reps * 8)
        for _ in range(a.reps):
            _lib.check(L.hcu_conv_wgrad_cl(*args))
        torch.cuda.synchronize()
        rep = _lib.timing_report()
        L.hcu_timing_disable()
        flops = 2.0 * B * od[0] * od[1] * od[2] * Cin * Cout * k[0] * k[1] * k[2]
        for kern, v in sorted(rep.items(), key=lambda kv: -kv[1]['ms']):
            us = v['ms'] * 1e3 / v['count']
            extra = ' %.1f TF/s useful' % (flops / us / 1e6) if 'finalize' not in kern else ''
            print('%-6s %-28s %8.1f us%s' % (name, kern, us, extra))


if __name__ == '__main__':
    main()
