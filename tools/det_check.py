#!/usr/bin/env python3
"""Run-to-run determinism of the training step (forward + pixel loss +
backward, 3 iterations) in fresh processes, per environment setting: each arm
runs twice and every output / gradient is compared bitwise.

  python tools/det_check.py [--bf16] 'ENV_A' ['ENV_B' ...]
"""
import argparse
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'tests'))

import torch  # noqa: E402

from test_gpu_modes import CHILD, KW  # noqa: E402


def run(env_extra, bf16, tag, tmp):
    out = os.path.join(tmp, tag + '.pt')
    env = dict(os.environ)
    env.update(env_extra)
    env['HCU_BCONV_TUNE'] = '0'
    env['HCU_TEST_BF16'] = '1' if bf16 else '0'
    kw = KW.replace('[8, 16, 32, 64, 128]', '[16, 32, 64, 128]') if bf16 else KW
    r = subprocess.run([sys.executable, '-c', CHILD % dict(root=ROOT, out=out, kw=kw, shape=(2, 4, 188, 188, 6))],
                       env=env, capture_output=True, text=True, timeout=300)
    if r.returncode:
        print(r.stderr[-2000:])
        raise SystemExit(1)
    return torch.load(out, weights_only=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--bf16', action='store_true')
    ap.add_argument('arms', nargs='+')
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as tmp:
        for k, arm in enumerate(a.arms):
            env = dict(kv.split('=', 1) for kv in arm.split())
            r1 = run(env, a.bf16, 'a%d_1' % k, tmp)
            r2 = run(env, a.bf16, 'a%d_2' % k, tmp)
            bad = [(it, j, (x - y).abs().max().item()) for it in range(3)
                   for j, (x, y) in enumerate(zip(r1[it], r2[it])) if not torch.equal(x, y)]
            print('arm %d [%s] bf16=%d: %s' % (k, arm, a.bf16, 'deterministic' if not bad else 'DIFFERS %r' % bad[:6]))
            sys.stdout.flush()


if __name__ == '__main__':
    main()
