"""Join the PMC passes of tools/pmc_passes.sh into one per-kernel table:
median duration (kernel trace), HBM-side bytes fetched / written
(FETCH_SIZE / WRITE_SIZE, KiB per dispatch), achieved GB/s, and the SQ
instruction mix.  Usage: pmc_summary.py gpurun_out/pmc_get [out.md]."""

import collections
import csv
import glob
import os
import statistics
import sys


def _short(name):
    n = name.split('(')[0].replace('void ', '')
    return n.replace('zk::', '')[:48]


def _load(d):
    """{kernel: {counter: [values per dispatch], '_dur': [ns]}}"""
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'),
                       recursive=True):
        per = collections.defaultdict(dict)
        for r in csv.DictReader(open(f)):
            key = (r['Kernel_Name'], r['Dispatch_Id'])
            per[key][r['Counter_Name']] = float(r['Counter_Value'])
        for (k, _), cs in per.items():
            for c, v in cs.items():
                out[_short(k)][c].append(v)
    for f in glob.glob(os.path.join(d, '**', '*kernel_trace.csv'),
                       recursive=True):
        for r in csv.DictReader(open(f)):
            dur = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
            out[_short(r['Kernel_Name'])]['_dur'].append(dur)
    return out


def main(d, dst=None):
    data = _load(d)
    rows = []
    for k, cs in data.items():
        if not cs.get('_dur') or k.startswith('at::') or 'native' in k:
            continue
        dur = statistics.median(cs['_dur']) / 1e3
        med = {c: statistics.median(v) for c, v in cs.items() if v}
        rows.append((dur, k, med))
    rows.sort(reverse=True)
    lines = ['| kernel | median us | fetch KiB | write KiB | GB/s | VALU | '
             'LDS | VMEM rd/wr | LDS bank confl | MFMA |',
             '|---|---|---|---|---|---|---|---|---|---|']
    for dur, k, m in rows[:24]:
        fk = m.get('FETCH_SIZE', 0.0)
        wk = m.get('WRITE_SIZE', 0.0)
        gbs = (fk + wk) * 1024 / (dur * 1e3) if dur > 0 else 0
        lines.append('| `%s` | %.1f | %.0f | %.0f | %.0f | %.0f | %.0f | '
                     '%.0f/%.0f | %.0f | %.0f |' % (
                         k, dur, fk, wk, gbs, m.get('SQ_INSTS_VALU', 0),
                         m.get('SQ_INSTS_LDS', 0),
                         m.get('SQ_INSTS_VMEM_RD', 0),
                         m.get('SQ_INSTS_VMEM_WR', 0),
                         m.get('SQ_LDS_BANK_CONFLICT', 0),
                         m.get('SQ_INSTS_MFMA', 0)))
    txt = '\n'.join(lines) + '\n'
    if dst:
        open(dst, 'w').write(txt)
    print(txt)


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
