"""fs_link's repair phases on the link-repair test streams
(tests/test_frame_repair.py): scan time, chain counters and, with
ZKMI_FS_DBG=1, fs_link's phase clock (chases, link check, recount).  Run
under ``rocprofv3 --kernel-trace --stats`` for the per-kernel split.

  ZKMI_FS_DBG=1 python tools/microbench/fl_probe.py [--case phantom]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..',
                                'tests'))
from zkmi.ops import _lib  # noqa: E402
from zkmi.ops import batch as B  # noqa: E402
import test_frame_repair as T  # noqa: E402


def stream(case):
    rng = np.random.default_rng(9)
    if case == 'phantom':
        return T._create_replies(1 << 20, zxid0=0x2E0000 - 500000), 256, 1
    if case == 'period':
        return T._set_replies(1 << 20), 256, 1
    if case == 'clean':
        return T._create_replies(1 << 20, zxid0=0x500000), 256, 1
    if case.startswith('dense'):
        lens = rng.integers(96, 249, 150000)
        buf, starts = T._stream(rng, lens, payload='plausible')
        return (buf, starts), 256, int(case[5:] or 1)
    if case == 'nospec':
        lens = np.random.default_rng(11).integers(88, 1113, 60000)
        return T._stream(np.random.default_rng(11), lens), 2048, 1
    raise SystemExit('unknown case')


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--case', default='phantom')
    ap.add_argument('--reps', type=int, default=5)
    ap.add_argument('--dbg', action='store_true', help='ZKMI_FS_DBG=1')
    a = ap.parse_args()
    if a.dbg:
        os.environ['ZKMI_FS_DBG'] = '1'     # read at the first scan
    (buf, starts), win, group = stream(a.case)
    dev = torch.device('cuda', 0)
    d = torch.from_numpy(buf).to(dev)
    sc = B.FrameScanner(len(starts) + 16, dev, window=win, group=group)
    nospec = a.case == 'nospec'
    sc.scan(d, len(buf), nospec=nospec)
    torch.cuda.synchronize()
    sc.chain_stats()
    for r in range(a.reps):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        ft = sc.scan(d, len(buf), nospec=nospec)
        e1.record()
        torch.cuda.synchronize()
        line = '%s rep %d: %.3f ms %r' % (a.case, r, e0.elapsed_time(e1),
                                         sc.chain_stats())
        if os.environ.get('ZKMI_FS_DBG'):
            tiles = (len(buf) + 4095) // 4096
            dd = _lib.lib().frame_scan_dbg(tiles + 1).cpu().numpy()
            raw = dd.reshape(-1)[8 * tiles:8 * tiles + 8]
            path = int(raw[4]) >> 56
            c = raw.astype(np.float64)
            c[4] = float(int(raw[4]) & ((1 << 56) - 1))
            us = lambda x, y: (c[y] - c[x]) / 100.0 if c[x] and c[y] \
                else -1.0                                       # noqa: E731
            line += (' fs_link: to chase %.1f us, chases %.1f us, check %.1f'
                     ' us, chase->end %.1f us, total %.1f us, path %d' % (
                         us(5, 0), us(0, 1), us(2, 3), us(3, 4), us(5, 4),
                         path))
        print(line, flush=True)
    r = ft.host_result()
    off = ft.off[:r['frames']].cpu().numpy()
    print('exact', r['frames'] == len(starts) and
          np.array_equal(off, starts + 4))


if __name__ == '__main__':
    main()
