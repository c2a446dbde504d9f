#!/usr/bin/env python3
"""Convolution microbenchmark: forward and input gradient of one Conv3d per
call through the C-ABI at the config-2 level shapes, per-kernel HIP-event times
(variant builds via HCU_LIB_PATH).

  python tools/conv_bench.py [--reps 20] [--only d0.c2] [--bf16]
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

SHAPES = {   # name: B, Cin, Cout, X, Y, Z, k  (config 2)
    'd0.c1': (2, 4, 8, 256, 256, 16, (3, 3, 2)),
    'd0.c2': (2, 8, 8, 254, 254, 15, (3, 3, 1)),
    'd1.c1': (2, 8, 16, 127, 127, 14, (3, 3, 2)),
    'd1.c2': (2, 16, 16, 125, 125, 13, (3, 3, 1)),
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
        y = torch.empty(B, *od, cs_out, device='cuda', dtype=dt)
        gy = torch.randn(B, *od, cs_out, device='cuda').to(dt)
        dx = torch.empty_like(x)
        w = torch.randn(Cout, Cin, *k, device='cuda')
        bias = torch.randn(Cout, device='cuda')
        sc = scratch_for(d)
        fwd = (ctypes.byref(d), _lib.ptr(x), _lib.ptr(w), _lib.ptr(bias), _lib.ptr(y), _lib.ptr(sc), sc.numel(),
               stream())
        bwd = (ctypes.byref(d), _lib.ptr(gy), _lib.ptr(w), _lib.ptr(dx), _lib.ptr(sc), sc.numel(), stream())
        vox = B * od[0] * od[1] * od[2]
        mb = (x.numel() + y.numel()) * x.element_size() / 1e6
        for what, fn, args in (('fwd', L.hcu_conv_fwd_cl, fwd), ('dgrad', L.hcu_conv_dgrad_cl, bwd)):
            for _ in range(3):
                _lib.check(fn(*args))
            torch.cuda.synchronize()
            L.hcu_timing_enable(a.reps * 8)
            for _ in range(a.reps):
                _lib.check(fn(*args))
            torch.cuda.synchronize()
            rep = _lib.timing_report()
            L.hcu_timing_disable()
            if hasattr(L, 'hcu_debug_conv8_phases'):
                ph = (ctypes.c_ulonglong * 8)()
                for _ in range(3):
                    _lib.check(fn(*args))
                torch.cuda.synchronize()
                L.hcu_debug_conv8_phases(ph)   # zero
                _lib.check(fn(*args))
                torch.cuda.synchronize()
                L.hcu_debug_conv8_phases(ph)
                t = max(1, ph[5])
                print('   phases (cycles per tile of wave 0): halo->LDS %.0f  barrier %.0f  issue %.0f  mfma %.0f  '
                      'epilogue %.0f | prologue %.0f lifetime %.0f  (tiles %d)' %
                      (ph[0] / t, ph[1] / t, ph[2] / t, ph[3] / t, ph[4] / t, ph[6] / t, ph[7] / t, ph[5]))
            for kern, v in sorted(rep.items(), key=lambda kv: -kv[1]['ms']):
                if 'prep' in kern:
                    continue
                us = v['ms'] * 1e3 / v['count']
                print('%-6s %-5s %-34s %8.1f us  %6.2f TB/s (%.0f MB, %.2f Mvox)' %
                      (name, what, kern, us, mb / us, mb, vox / 1e6), flush=True)


if __name__ == '__main__':
    main()
