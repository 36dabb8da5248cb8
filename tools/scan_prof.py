"""Summarise a rocprofv3 kernel trace of tools/microbench/scan_bench.py:
per scan-kernel median duration, bucketed by grid size (i.e. by n)."""

import collections
import csv
import statistics
import sys


def main(path):
    rows = collections.defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r['Kernel_Name']
            if 'scan_' not in name:
                continue
            short = name.split('(')[0].replace('void ', '').replace('zk::', '')
            grid = int(r['Grid_Size_X']) // int(r['Workgroup_Size_X'])
            dur = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
            rows[(short, grid)].append(dur)
    print('| kernel | workgroups | calls | median us |')
    print('|---|---|---|---|')
    for (k, g), v in sorted(rows.items(), key=lambda x: (x[0][1], x[0][0])):
        print('| `%s` | %d | %d | %.2f |'
              % (k, g, len(v), statistics.median(v)))


if __name__ == '__main__':
    main(sys.argv[1])
