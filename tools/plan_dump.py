#!/usr/bin/env python3
"""Prints every kernel plan of a bench configuration (host only, no GPU needed):
the bconv tilings (HCU_CONV2_LOG) and the weight-gradient kernels
(HCU_PLAN_LOG), from the persistent tuning table (HCU_BCONV_TUNE=1).

  python tools/plan_dump.py [--config 2|3]
"""
import argparse
import ctypes
import os
import sys

os.environ.setdefault('HCU_BCONV_TUNE', '1')
os.environ.setdefault('HCU_CONV2_LOG', '1')
os.environ.setdefault('HCU_PLAN_LOG', '1')
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from hcat.unet import Unet_Constructor  # noqa: E402
from hcunet_amd import unet as U  # noqa: E402
from hcunet_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='2')
    a = ap.parse_args()
    cfg = bench.CONFIGS[a.config]
    m = Unet_Constructor(**cfg['kw'])
    spec = U.spec_struct(m)
    spec.compute_dtype = _lib.HCU_BF16 if cfg['dtype'] == 'bf16' else _lib.HCU_F32
    p = U._Plan(spec, cfg['batch'], *bench.TILE)
    print('saved %.1f MB scratch %.1f MB' % (p.saved_bytes / 1e6, p.scratch_bytes / 1e6))
    sys.stderr.flush()


if __name__ == '__main__':
    main()
