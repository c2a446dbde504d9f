#!/usr/bin/env python3
"""Per-kernel averages of every counter in rocprofv3 --pmc CSV output.

  python tools/pmc_summary.py DIR [DIR ...] [--top N] [--match SUBSTR]
"""
import argparse
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import short_name  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('dirs', nargs='+')
    ap.add_argument('--top', type=int, default=25)
    ap.add_argument('--match', default='')
    a = ap.parse_args()
    vals = {}   # kernel -> counter -> [values]
    for d in a.dirs:
        for fn in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
            with open(fn, newline='') as f:
                for row in csv.DictReader(f):
                    k = short_name(row.get('Kernel_Name', '?'))
                    if a.match and a.match not in k:
                        continue
                    vals.setdefault(k, {}).setdefault(row['Counter_Name'], []).append(
                        float(row['Counter_Value']))
    ctrs = sorted({c for v in vals.values() for c in v})
    order = sorted(vals, key=lambda k: -max(sum(x) for x in vals[k].values()))
    print('%-34s' % 'kernel' + ''.join('%16s' % c[:16] for c in ctrs))
    for k in order[:a.top]:
        print('%-34s' % k[:34] + ''.join(
            '%16.4g' % (sum(vals[k][c]) / len(vals[k][c]) if c in vals[k] else float('nan'))
            for c in ctrs))


if __name__ == '__main__':
    main()
