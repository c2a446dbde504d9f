#!/usr/bin/env python3
"""Accounts for every kernel dispatch of a rocprofv3 run (its SQLite output,
`--kernel-trace --output-format rocpd`): which kernels are not this
library's (hcu::) kernels, and whether they fall inside a training step.

Steps are delimited by the optimizer: a step ends with its adam_kernel
dispatch, and step k spans from the end of step k-1's adam_kernel to the end
of its own (the first step from its first kernel).  Dispatches before the
first step (model set-up: parameter and input uploads) and after the last
(the loss read-back) are reported separately.

  python tools/kernel_audit.py gpurun_out/<run>/run_results.db
"""
import collections
import sqlite3
import sys


def main(path):
    c = sqlite3.connect(path)
    rows = list(c.execute('select name, start, end from kernels order by start'))
    ends = [e for n, s, e in rows if 'adam_kernel' in n]
    if not ends:
        print('no adam_kernel dispatch: not a training run')
        return 1
    first = next(s for n, s, e in rows if 'hcu' in n and 'adam' not in n)
    before, after = collections.Counter(), collections.Counter()
    inside = collections.Counter()
    for n, s, e in rows:
        short = n.split('(')[0][:70]
        if s < first:
            before[short] += 1
        elif s > ends[-1]:
            after[short] += 1
        elif 'hcu' not in n:
            inside[short] += 1
    nsteps = len(ends)
    print('%d dispatches, %d steps (adam_kernel)' % (len(rows), nsteps))
    print('before the first step (set-up):')
    for k, v in before.most_common():
        print('  %5d  %s' % (v, k))
    print('after the last step:')
    for k, v in after.most_common():
        print('  %5d  %s' % (v, k))
    print('non-hcu kernels inside the steps (count, per step):')
    if not inside:
        print('  none')
    for k, v in inside.most_common():
        print('  %5d  %6.2f  %s' % (v, v / nsteps, k))
    return 0


if __name__ == '__main__':
    sys.exit(main(sys.argv[1]))
