#!/usr/bin/env python3
"""Per-kernel duration summary from a rocprofv3 results database (rocpd sqlite).

  python tools/rocpd_stats.py path/to/run_results.db [--top N] [--filter substr]
"""
import argparse
import sqlite3
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('db')
    ap.add_argument('--top', type=int, default=30)
    ap.add_argument('--filter', default=None)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute('select s.kernel_name, d.start, d.end, d.group_segment_size from rocpd_kernel_dispatch d '
                     'join rocpd_info_kernel_symbol s on d.kernel_id = s.id').fetchall()
    agg = {}
    for name, s, e, lds in rows:
        if a.filter and a.filter not in name:
            continue
        agg.setdefault(name, []).append((e - s) / 1e3)
    tot = sum(sum(v) for v in agg.values())
    print('%-70s %6s %10s %10s %10s %6s' % ('kernel', 'calls', 'total_us', 'avg_us', 'med_us', '%'))
    for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:a.top]:
        print('%-70s %6d %10.1f %10.2f %10.2f %6.2f' % (name[:70], len(v), sum(v), sum(v) / len(v),
                                                      statistics.median(v), 100 * sum(v) / tot))


if __name__ == '__main__':
    main()
