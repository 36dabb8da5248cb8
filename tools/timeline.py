"""Timeline of a rocprofv3 kernel trace: per step, how long the GPU ran
something, how much two streams overlapped, and the idle gaps.

    python tools/timeline.py <kernel_trace.csv> [--marker bench_gen_get]

A step starts at every other marker kernel (one per connection; two
connections per GET step).  For each complete step: wall span, busy time
(union of kernel intervals), overlap (time with >= 2 kernels running),
idle time, and the kernels' summed durations by name.
"""

import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('csv')
    ap.add_argument('--marker', default='bench_gen_get')
    ap.add_argument('--per-step', type=int, default=2,
                    help='marker launches per step (connections)')
    ap.add_argument('--last', type=int, default=4, help='steps shown')
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']),
                         r['Kernel_Name'], r.get('Queue_Id') or
                         r.get('Stream_Id') or '0'))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if a.marker in r[2]]
    starts = [rows[marks[j]][0] for j in range(0, len(marks), a.per_step)]
    steps = list(zip(starts, starts[1:]))[-a.last:]
    for s0, s1 in steps:
        ks = [r for r in rows if s0 <= r[0] < s1]
        ev = []
        for b, e, _, _ in ks:
            ev.append((b, 1))
            ev.append((e, -1))
        ev.sort()
        busy = over = 0
        cur = 0
        last = s0
        for t, d in ev:
            if cur >= 1:
                busy += t - last
            if cur >= 2:
                over += t - last
            cur += d
            last = t
        span = s1 - s0
        by = collections.Counter()
        for b, e, n, _ in ks:
            by[n.split('(')[0][:48]] += e - b
        print('step %.1f us: busy %.1f, >=2 running %.1f, idle %.1f, '
              'kernels %d, summed %.1f us' % (
                  span / 1e3, busy / 1e3, over / 1e3, (span - busy) / 1e3,
                  len(ks), sum(by.values()) / 1e3))
        for n, d in by.most_common(14):
            print('   %8.1f  %s' % (d / 1e3, n))


if __name__ == '__main__':
    main()
