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
    """fs_link's debug rows past the tiles of the scanned buffer's
    capacity: every block's entry and check-done clocks, the common path's
    bases start / end (us from the earliest block entry; 100 MHz clock)."""
    tiles = (cap_bytes + 4095) // 4096
    try:
        host = _lib.lib().frame_scan_dbg(tiles + 6).numpy().reshape(-1)
    except RuntimeError:
        return None                   # ZKMI_FS_DBG not set
    rows = host[tiles * 8:(tiles + 6) * 8]
    blk = rows[8:40].reshape(16, 2).astype(np.int64)
    live = blk[:, 0] > 0
    if not live.any():
        return None
    t0 = int(blk[live, 0].min())
    us = lambda v: round((int(v) - t0) / 100.0, 2)     # noqa: E731
    return {'block_entry': [us(v) for v in blk[live, 0]],
            'block_check_done': [us(v) for v in blk[live, 1]],
            'bases': [us(rows[40]) if rows[40] else None,
                      us(rows[41]) if rows[41] else None],
            'repair_path': int(rows[4]) >> 56}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=130)
    ap.add_argument('--gc', choices=('on', 'off', 'freeze'), default='on',
                    help='the Python collector during the steps')
    ap.add_argument('--all', action='store_true',
                    help='every step (no stop at the first slow one)')
    ap.add_argument('--prelaunch', type=int, default=0,
                    help='tiny kernel launches before the steps (is the '
                         'slow step the process\'s N-th launch?)')
    ap.add_argument('--seed', type=int, default=0)
    a = ap.parse_args()
    import gc
    gcs = []            # (step, generation, ms) of every collection
    times = []          # (filled by the step loop below)

    def on_gc(phase, info, box={}):
        if phase == 'start':
            box['t'] = time.perf_counter()
        else:
            gcs.append((len(times), info['generation'],
                        1e3 * (time.perf_counter() - box.get('t', 0))))
    gc.callbacks.append(on_gc)
    dev = torch.device('cuda', 0)
    n = 1 << 20
    tree = S.GpuTree(1000000, 100, device=dev, seed=0, watch_cap=2 * n)
    pipe = S.WatchPipeline(tree, n, seed=a.seed)
    if a.prelaunch:
        x = torch.zeros(1, device=dev)
        t0 = time.perf_counter()
        worst = 0.0
        for k in range(a.prelaunch):
            t1 = time.perf_counter()
            x.add_(1)
            if k % 256 == 255:
                torch.cuda.synchronize()
            worst = max(worst, time.perf_counter() - t1)
        torch.cuda.synchronize()
        print('prelaunch %d launches %.1f ms, slowest launch call %.2f ms'
              % (a.prelaunch, 1e3 * (time.perf_counter() - t0),
                 1e3 * worst), flush=True)
    acc = torch.zeros(64, dtype=torch.int64, device=dev)
    pipe.nscan.chain_stats()
    # a CUDA event after each of the step's launches-worth of host calls
    # (the pipeline's own methods wrapped), to time its phases on the GPU
    marks = []

    def mark(name):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        marks.append((name, e))

    def wrap(obj, meth, name):
        f = getattr(obj, meth)

        def g(*args, **kw):
            r = f(*args, **kw)
            mark(name)
            return r
        setattr(obj, meth, g)
    for sc, nm in ((pipe.server.scanner, 'req_scan'), (pipe.rscan, 'rep_scan'),
                   (pipe.nscan, 'note_scan')):
        wrap(sc, 'scan', nm)
    wrap(pipe.server, 'serve', 'serve')
    wrap(pipe.fan, 'gather_slots', 'gather')
    del times[:]
    prev_seg = (0, 0, 0)
    if a.gc == 'off':
        gc.disable()
    elif a.gc == 'freeze':
        gc.collect()
        gc.freeze()
    for s in range(a.steps):
        torch.cuda.synchronize()
        marks.clear()
        mark('start')
        t0 = time.perf_counter()
        pipe.step(acc=acc)
        mark('end')
        torch.cuda.synchronize()
        ms = 1e3 * (time.perf_counter() - t0)
        phases = [(marks[j][0], round(marks[j - 1][1].elapsed_time(
            marks[j][1]), 3)) for j in range(1, len(marks))]
        st = pipe.nscan.chain_stats()
        mst = torch.cuda.memory_stats(dev)
        seg = (mst.get('segment.all.allocated', 0),
               mst.get('reserved_bytes.all.current', 0),
               mst.get('num_alloc_retries', 0))
        if s > 0 and seg != prev_seg:
            print('step %d %.2f ms: allocator segments %d (+%d), reserved '
                  '%.1f MB, retries %d' % (s, ms, seg[0], seg[0] - prev_seg[0],
                                           seg[1] / 1e6, seg[2]), flush=True)
        prev_seg = seg
        med = float(np.median(times)) if times else ms
        times.append(ms)
        slow_gc = [g for g in gcs if g[0] == s and g[2] > 5]
        if slow_gc:
            print('step %d %.2f ms: collections %r' % (s, ms, slow_gc),
                  flush=True)
        if ms >= 5 * med and s >= 5 and a.all:
            print('SLOW step %d %.2f ms: GPU phases %r' % (s, ms, phases),
                  flush=True)
        if s < 5 or ms < 5 * med or a.all:
            if s % 10 == 0:
                print('step %d %.2f ms %r' % (s, ms, st), flush=True)
            continue
        nb = int(pipe.nrx.item()) if hasattr(pipe.nrx, 'item') \
            else int(pipe.nrx)
        print('SLOW step %d %.2f ms (median %.2f) stats %r stream %d B '
              'zxid %d' % (s, ms, med, st, nb, int(tree.counters[1].item())),
              flush=True)
        print('GPU phases (ms since the mark before):', phases, flush=True)
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
    print('done', int(acc.sum().item()), 'median %.3f ms max %.3f ms '
          '(step %d); gc %s: %d collections, gen2 %r' % (
              float(np.median(times[1:])), max(times[1:]),
              int(np.argmax(times[1:])) + 1, a.gc, len(gcs),
              [(g[0], round(g[2], 1)) for g in gcs if g[1] == 2]),
          flush=True)


if __name__ == '__main__':
    main()
