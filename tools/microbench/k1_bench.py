"""K1 microbenchmark: the frame scan alone over the GET workload's own
request and reply streams (one 512K-request connection, the bench's
shape), timed per scan, checked frame by frame against the host codec's
framing, with the per-tile phase clock when ZKMI_FS_DBG=1.

    python tools/microbench/k1_bench.py [--data-dist LO-HI] [--reps N]

Prints one line per stream: scan us, GB/s, frames, tiles, chain stats
(tiles without a speculated entry / re-walked / repair rounds / looked
up) and, with ZKMI_FS_DBG, the phase medians (us) of fs_tile."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
from zkmi import codec, consts  # noqa: E402
from zkmi.bench import synthetic as S  # noqa: E402
from zkmi.ops import _lib  # noqa: E402
from zkmi.ops import batch as B  # noqa: E402


def host_frames(buf, n):
    raw = buf[:n].cpu().numpy().tobytes()
    frames, stop, bad = codec.scan_frames(raw, 0, len(raw), consts.MAX_PACKET)
    off = np.fromiter((o for o, _ in frames), np.int64, len(frames))
    ln = np.fromiter((l for _, l in frames), np.int64, len(frames))
    return off, ln, stop, bad


def walked(tiles, group):
    """A group's walked tiles (all but its first): medians / p90 (us) of
    the wait for the tile's load (+ its LDS store), the chain walk through
    it and the records, and the frames walked per tile."""
    if group <= 1:
        return ''
    d = _lib.lib().frame_scan_dbg(tiles + 1).cpu().numpy().reshape(-1)
    d = d[:8 * tiles].reshape(tiles, 8)
    rows = np.array([t for t in range(tiles) if t % group and d[t, 3]])
    if len(rows) == 0:
        return ''
    c = d[rows].astype(np.float64)
    us = 1.0 / 100.0
    cols = {'load+store': (c[:, 1] - c[:, 0]) * us,
            'walk': (c[:, 2] - c[:, 1]) * us,
            'records': (c[:, 3] - c[:, 2]) * us}
    out = ' '.join('%s %.2f/%.2f' % (k, np.median(v), np.percentile(v, 90))
                   for k, v in cols.items())
    return out + ' frames/tile %d' % int(np.median(c[:, 5]))


def phases(tiles, step=1):
    """Per-tile phase medians / p90 (us) of fs_tile's clock: stage, node
    detection, map build (successors + pointer jumping), publish, wait for
    the tile before, chain; with the node counts and jumping rounds."""
    d = _lib.lib().frame_scan_dbg(tiles + 1).cpu().numpy().reshape(-1)
    d = d[:8 * tiles].reshape(tiles, 8)[::step]
    c = d.astype(np.float64)
    t0 = c[:, 0].min()
    us = 1.0 / 100.0            # 100 MHz wall clock
    cols = {'start': (c[:, 0] - t0) * us, 'stage': (c[:, 6] - c[:, 0]) * us,
            'detect': (c[:, 4] - c[:, 6]) * us,
            'build': (c[:, 7] - c[:, 4]) * us,
            'publish': (c[:, 1] - c[:, 7]) * us,
            'wait': (c[:, 2] - c[:, 1]) * us,
            'chain': (c[:, 3] - c[:, 2]) * us,
            'end': (c[:, 3] - t0) * us}
    out = ' '.join('%s %.2f/%.2f' % (k, np.median(v), np.percentile(v, 90))
                   for k, v in cols.items())
    nodes = d[:, 5] & 0xFFFF
    rounds = (d[:, 5] >> 16) & 0xFF
    done = (d[:, 5] >> 24) & 1
    out += ('\n         nodes p50 %d p90 %d max %d (>512: %d tiles) rounds '
            'p50 %d max %d, map chain %.1f%%' % (
                np.median(nodes), np.percentile(nodes, 90), nodes.max(),
                int((nodes > 512).sum()), np.median(rounds), rounds.max(),
                100.0 * done.mean()))
    return out


def bench(tag, buf, n_dev, window, reps, group=1):
    dev = buf.device
    n = int(n_dev.item())
    cap = n // 8 + 64
    sc = B.FrameScanner(cap, dev, window=window, group=group)
    ft = sc.scan(buf, n_dev)
    torch.cuda.synchronize()
    off, ln, stop, bad = host_frames(buf, n)
    got = int(ft.result[0].item())
    ok = got == len(off)
    if ok:
        ok = (np.array_equal(ft.off[:got].cpu().numpy(), off) and
              np.array_equal(ft.length[:got].cpu().numpy().astype(np.int64),
                             ln) and int(ft.result[1].item()) == stop)
    sc.chain_stats()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for _ in range(3):
        sc.scan(buf, n_dev)
    ev[0].record()
    for _ in range(reps):
        sc.scan(buf, n_dev)
    ev[1].record()
    torch.cuda.synchronize()
    us = ev[0].elapsed_time(ev[1]) * 1e3 / reps
    st = sc.chain_stats()
    tiles = (n + 4095) // 4096
    line = ('%-8s g%d %8.1f us %6.2f GB/s frames %d tiles %d exact %s '
            'stats %s' % (tag, sc.group, us, n / us / 1e3, got, tiles, ok,
                          {k: v // (reps + 3) for k, v in st.items()}))
    if os.environ.get('ZKMI_FS_DBG'):
        sc.scan(buf, n_dev)
        torch.cuda.synchronize()
        line += '\n         ' + phases(tiles, sc.group)
        wl = walked(tiles, sc.group)
        if wl:
            line += '\n         walked tiles: ' + wl
    print(line, flush=True)
    return ok


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--data-dist', default=None)
    ap.add_argument('--batch', type=int, default=1 << 19)
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('--req-group', type=int, default=1,
                    help='tiles a wave takes on the request stream')
    ap.add_argument('--win-max', type=int, default=None,
                    help='batch.FS_WINDOW_AUTO_MAX for this run (the largest '
                         'window chosen without long-frame mode)')
    ap.add_argument('--workload', default='get',
                    help='get, mix (create / set / delete replies) or storm '
                         '(EPHEMERAL|SEQUENTIAL creates, --batch 1M for the '
                         "bench's shape)")
    ap.add_argument('--zxid', type=lambda x: int(x, 0), default=None,
                    help='the tree zxid the GET replies carry (their header '
                         'bytes: length-like words for some ranges)')
    ap.add_argument('--group', type=int, default=None,
                    help='tiles a wave takes on the reply stream (1, 2, 4)')
    a = ap.parse_args()
    dev = torch.device('cuda', 0)
    if a.win_max is not None:
        B.FS_WINDOW_AUTO_MAX = a.win_max
    dist = None
    if a.data_dist:
        lo, hi = a.data_dist.split('-')
        dist = (int(lo), int(hi))
    tree = S.GpuTree(1_000_000, 100, device=dev, seed=0, data_dist=dist)
    if a.workload == 'mix':
        tree = S.GpuTree(1_000_000, 100, device=dev, seed=0,
                         spare=(2 * a.batch + 8192) / 1e6 + 0.05)
    if a.workload == 'storm':
        tree = S.GpuTree(1_000_000, 100, device=dev, seed=0, hash_factor=2,
                         spare=(3 * a.batch + 8192) / 1e6 + 0.05)
    if a.zxid is not None:
        tree.counters[_lib.TC_ZXID] = a.zxid
    if a.workload in ('mix', 'storm'):
        if a.workload == 'mix':
            pipe = S.MixPipeline(tree, 2 * a.batch, 100, seed=1)
        else:
            pipe = S.StormPipeline(tree, a.batch)
        for _ in range(2):
            pipe.step()
        drv = pipe.drv
        tx, srv, rwin = drv.tx, drv.server, drv.rwindow
        rgroup = drv.rscanner.group
    else:
        pipe = S.GetPipeline(tree, a.batch, seed=1)
        for _ in range(2):
            pipe.step()
        tx, srv, rwin = pipe.tx, pipe.server, pipe.rwindow
        rgroup = pipe.rscanner.group
    torch.cuda.synchronize()
    req_n = srv.scanner.table.result[1:2].clone()
    rx, rtotal = srv.result[0], srv.result[1]
    ok = bench('request', tx, req_n, srv.window, a.reps, a.req_group)
    group = rgroup if a.group is None else a.group
    ok &= bench('reply', rx, rtotal.reshape(1)[:1].clone(), rwin, a.reps,
                group)
    print('ALL EXACT' if ok else 'MISMATCH', flush=True)
    sys.exit(0 if ok else 1)


if __name__ == '__main__':
    main()
