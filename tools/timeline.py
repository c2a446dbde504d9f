#!/usr/bin/env python3
"""Step timeline of a graphed training step from a rocprofv3 rocpd database.

  rocprofv3 --kernel-trace -d OUT -- python3 bench.py --steps 10 --no-kernel-timing ...
  python tools/timeline.py OUT/.../*_results.db [--marker adam_kernel] [--gaps 25]

Splits the dispatch stream into steps at the marker kernel (the step's last
launch), then for the last complete step reports: wall time, busy time (union
of kernel intervals over all queues), per-queue busy time, the idle gaps of the
critical (marker's) queue with the kernels either side, and the share of the
step spent in kernels shorter than 10 us.
"""
import argparse
import glob
import sqlite3


def load(db):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute('pragma table_info(rocpd_kernel_dispatch)')]
    qcol = 'queue_id' if 'queue_id' in cols else ('stream_id' if 'stream_id' in cols else None)
    q = ('select s.kernel_name, d.start, d.end, %s from rocpd_kernel_dispatch d '
         'join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start' % (('d.' + qcol) if qcol else '0'))
    return [(n, s, e, qq) for n, s, e, qq in c.execute(q).fetchall()]


def short(n):
    n = n.split('(')[0]
    return n[:48]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('db', nargs='+')
    ap.add_argument('--marker', default='adam_kernel')
    ap.add_argument('--gaps', type=int, default=25)
    ap.add_argument('--all', action='store_true', help='every kernel of the step, all queues, by start')
    a = ap.parse_args()
    dbs = []
    for d in a.db:
        dbs += glob.glob(d) if any(ch in d for ch in '*?[') else [d]
    rows = []
    for d in dbs:
        rows += load(d)
    rows.sort(key=lambda r: r[1])
    ends = [i for i, r in enumerate(rows) if a.marker in r[0]]
    if len(ends) < 3:
        print('fewer than 3 marker kernels found')
        return
    i0, i1 = ends[-2] + 1, ends[-1] + 1
    step = rows[i0:i1]
    t0 = rows[ends[-2]][2]
    t1 = rows[ends[-1]][2]
    wall = (t1 - t0) / 1e3
    iv = sorted((s, e) for _, s, e, _ in step)
    busy, cs, ce = 0, None, None
    for s, e in iv:
        s = max(s, t0)
        if cs is None:
            cs, ce = s, e
        elif s > ce:
            busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        busy += ce - cs
    print('step wall %.1f us, busy (union over queues) %.1f us, idle %.1f us, %d launches'
          % (wall, busy / 1e3, wall - busy / 1e3, len(step)))
    queues = {}
    for n, s, e, q in step:
        queues.setdefault(q, []).append((n, s, e))
    for q, ks in sorted(queues.items(), key=lambda kv: -len(kv[1])):
        print('queue %s: %d launches, kernel time %.1f us' % (q, len(ks), sum(e - s for _, s, e in ks) / 1e3))
    small = [(e - s) for _, s, e, _ in step if e - s < 10000]
    print('kernels < 10 us: %d launches, %.1f us' % (len(small), sum(small) / 1e3))
    mq = rows[ends[-1]][3]
    ks = queues[mq]
    gaps = []
    prev_e, prev_n = t0, '<step start>'
    for n, s, e in ks:
        gaps.append(((s - prev_e) / 1e3, prev_n, n))
        prev_e, prev_n = max(prev_e, e), n
    tot = sum(g for g, _, _ in gaps if g > 0)
    print('critical queue %s: gaps total %.1f us over %d launches (mean %.2f us)'
          % (mq, tot, len(ks), tot / max(1, len(ks))))
    for g, p, n in sorted(gaps, key=lambda x: -x[0])[:a.gaps]:
        print('  gap %7.1f us  after %-48s before %s' % (g, short(p), short(n)))
    # stream attribution by kernel family: the weight-gradient branch runs on
    # the executor's side stream
    side_keys = ('wgrad', 'chansum', 'reduce_partials', 'outconv_wfinalize')
    main_ev = [(s_, e_, n) for n, s_, e_, _ in step if not any(k in n for k in side_keys)]
    side_ev = [(s_, e_, n) for n, s_, e_, _ in step if any(k in n for k in side_keys)]
    if side_ev:
        bwd0 = min(s_ for s_, _, n in side_ev)
        mb = [(s_, e_, n) for s_, e_, n in main_ev if s_ >= bwd0 and 'adam' not in n]
        print('backward from first side-stream kernel: main busy %.1f us (ends at +%.1f), side busy %.1f us '
              '(ends at +%.1f), adam starts at +%.1f'
              % (sum(e_ - s_ for s_, e_, _ in mb) / 1e3, (max(e_ for _, e_, _ in mb) - bwd0) / 1e3 if mb else 0,
                 sum(e_ - s_ for s_, e_, _ in side_ev) / 1e3, (max(e_ for _, e_, _ in side_ev) - bwd0) / 1e3,
                 (max(s_ for s_, _, n in main_ev if 'adam' in n) - bwd0) / 1e3))
    if a.all:
        qn = {q: i for i, q in enumerate(sorted(queues, key=lambda q: -len(queues[q])))}
        print('\nall kernels (queue index, start offset us, end offset us, duration us):')
        for n, s, e, q in sorted(step, key=lambda r: r[1]):
            print('  q%d %8.1f %8.1f %7.1f  %s' % (qn[q], (s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3, short(n)))
        return
    print('\ncritical-queue sequence (us: start offset, duration):')
    for n, s, e in ks:
        print('  %8.1f %7.1f  %s' % ((s - t0) / 1e3, (e - s) / 1e3, short(n)))


if __name__ == '__main__':
    main()
