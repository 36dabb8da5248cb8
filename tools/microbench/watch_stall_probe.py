"""The watch workload's slow step: which K1 path its R1 notification scan
took.  Eager watch steps with K1's chain counters read after each; at the
first step slower than 5x the running median: the chain counters, fs_link's
phase clock (ZKMI_FS_DBG=1: start, chases, links checked, end | path), the
stream saved to gpurun_out/watch_stall_stream.npz, then three re-scans of
the same bytes, timed, with their counters.

  ZKMI_FS_DBG=1 python tools/microbench/watch_stall_probe.py --steps 130
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from zkmi.bench import synthetic as S  # noqa: E402
from zkmi.ops import _lib  # noqa: E402


def fs_clock(cap_bytes):
    """fs_link's phase clock row (the debug buffer's row past the tiles of
    the scanned buffer's capacity)."""
    tiles = (cap_bytes + 4095) // 4096
    try:
        host = _lib.lib().frame_scan_dbg(tiles + 1).numpy().reshape(-1)
    except RuntimeError:
        return None                   # ZKMI_FS_DBG not set
    row = host[tiles * 8:(tiles + 1) * 8]
    t0 = row[5]
    return {'path': int(row[4]) >> 56,
            'us': [round((int(v) & ((1 << 56) - 1)) / 100.0 - t0 / 100.0, 1)
                   if v else None for v in row[:5]]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=130)
    a = ap.parse_args()
    dev = torch.device('cuda', 0)
    n = 1 << 20
    tree = S.GpuTree(1000000, 100, device=dev, seed=0, watch_cap=2 * n)
    pipe = S.WatchPipeline(tree, n, seed=0)
    acc = torch.zeros(64, dtype=torch.int64, device=dev)
    pipe.nscan.chain_stats()
    times = []
    for s in range(a.steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pipe.step(acc=acc)
        torch.cuda.synchronize()
        ms = 1e3 * (time.perf_counter() - t0)
        st = pipe.nscan.chain_stats()
        med = float(np.median(times)) if times else ms
        times.append(ms)
        if s < 5 or ms < 5 * med:
            if s % 10 == 0:
                print('step %d %.2f ms %r' % (s, ms, st), flush=True)
            continue
        nb = int(pipe.nrx.item()) if hasattr(pipe.nrx, 'item') \
            else int(pipe.nrx)
        print('SLOW step %d %.2f ms (median %.2f) stats %r stream %d B '
              'zxid %d' % (s, ms, med, st, nb, int(tree.counters[1].item())),
              flush=True)
        print('fs_link clock', fs_clock(pipe.rx.numel()), flush=True)
        buf = pipe.rx[:nb].clone()
        out = os.path.join(ROOT, 'gpurun_out')
        os.makedirs(out, exist_ok=True)
        np.savez_compressed(os.path.join(out, 'watch_stall_stream.npz'),
                            buf=buf.cpu().numpy())
        for r in range(3):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            ft = pipe.nscan.scan(buf, nb)
            torch.cuda.synchronize()
            print('rescan %d %.3f ms frames %d stats %r clock %r' % (
                r, 1e3 * (time.perf_counter() - t1), int(ft.count[0].item()),
                pipe.nscan.chain_stats(), fs_clock(pipe.rx.numel())),
                flush=True)
        break
    print('done', int(acc.sum().item()), 'median %.3f ms max %.3f ms' % (
        float(np.median(times)), max(times)), flush=True)


if __name__ == '__main__':
    main()
