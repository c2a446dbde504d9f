"""Bitwise comparison of two library builds on the same training steps (the
child process of tests/test_gpu_modes.py, 3 steps of a 5-level net):
  python tools/cmp_libs.py LIB_A LIB_B [--bf16] [--kw config3]"""
import argparse
import os
import pathlib
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from tests import test_gpu_modes as tm  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('a')
ap.add_argument('b')
ap.add_argument('--bf16', action='store_true')
ap.add_argument('--wide', action='store_true', help='feature_sizes [32..512] (config-3 widths)')
ap.add_argument('--env-a', default='', help='K=V[,K=V] for run a only (A/B of an environment switch)')
ap.add_argument('--env-b', default='', help='K=V[,K=V] for run b only')
args = ap.parse_args()


def _kv(spec):
    return dict(kv.split('=', 1) for kv in spec.split(',') if kv)
kw = tm.KW.replace('[8, 16, 32, 64, 128]', '[32, 64, 128, 256, 512]') if args.wide else tm.KW
env = {'HCU_TEST_BF16': '1' if args.bf16 else '0'}
tmp = pathlib.Path(tempfile.mkdtemp())
ra = tm._run(tmp, 'a', dict(env, HCU_LIB_PATH=args.a, **_kv(args.env_a)), kw=kw)
rb = tm._run(tmp, 'b', dict(env, HCU_LIB_PATH=args.b, **_kv(args.env_b)), kw=kw)
diff = [(it, k, (x.double() - y.double()).abs().max().item())
        for it in range(3) for k, (x, y) in enumerate(zip(ra[it], rb[it])) if not torch.equal(x, y)]
print('bitwise equal' if not diff else 'DIFFERENT: %d tensors, first %s' % (len(diff), diff[:5]))
