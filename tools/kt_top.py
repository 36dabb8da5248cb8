"""Longest kernel dispatches of a rocprofv3 kernel trace (CSV):
python tools/kt_top.py <kernel_trace.csv> [N]"""
import csv
import sys


def main():
    path = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            try:
                d = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
            except (KeyError, ValueError):
                continue
            rows.append((d, int(r['Start_Timestamp']),
                         r.get('Kernel_Name', '')[:90],
                         r.get('Correlation_Id', '')))
    if not rows:
        print('no rows')
        return
    t0 = min(r[1] for r in rows)
    rows.sort(reverse=True)
    for d, s, name, cid in rows[:k]:
        print('%10.1f us  at %10.1f us  %s  %s' % (d / 1e3, (s - t0) / 1e3,
                                                  name, cid))


if __name__ == '__main__':
    main()
