"""Which watch step's R1 notification scan needs the long repair, and what
its stream looks like: eager watch steps with K1's chain counters read
after each, then, for the first step whose scan had tiles without a
speculated entry, the per-tile node counts of its stream (host numpy; the
map holds 512 nodes) and the bytes of the first such tile.

  python tools/microbench/watch_k1_probe.py --steps 120
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from zkmi.bench import synthetic as S  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--steps', type=int, default=120)
a = ap.parse_args()
dev = torch.device('cuda', 0)
n = 1 << 20
tree = S.GpuTree(1000000, 100, device=dev, seed=0, watch_cap=2 * n)
pipe = S.WatchPipeline(tree, n, seed=0)
acc = torch.zeros(64, dtype=torch.int64, device=dev)
pipe.nscan.chain_stats()
for s in range(a.steps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pipe.step(acc=acc)
    torch.cuda.synchronize()
    ms = 1e3 * (time.perf_counter() - t0)
    st = pipe.nscan.chain_stats()
    if s > 0 and (st['no_spec'] or st['rewalked'] or ms > 10):
        print('step %d %.2f ms %r window %d zxid %d' % (
            s, ms, st, pipe.nscan.window, int(tree.counters[1].item())),
            flush=True)
        nb = int(pipe.nrx.item()) if hasattr(pipe.nrx, 'item') \
            else int(pipe.nrx)
        buf = pipe.rx[:nb].cpu().numpy()
        u = buf.astype(np.uint32)
        w = u[:-3] << 24 | u[1:-2] << 16 | u[2:-1] << 8 | u[3:]
        W = pipe.nscan.window
        pos = np.arange(len(w)) % 4096
        node = ((w >= 16) & (w <= W - 4)) | \
            ((pos < W) & (w >= 16) & (w <= 1 << 20))
        per = np.add.reduceat(node.astype(np.int64),
                              np.arange(0, len(w), 4096))
        print('stream %d B, tiles %d, nodes per tile p50 %d p99 %d max %d, '
              'tiles over 512: %d' % (nb, len(per), np.median(per),
                                      np.percentile(per, 99), per.max(),
                                      int((per > 512).sum())), flush=True)
        over = np.nonzero(per > 512)[0]
        t = int(over[0]) if len(over) else int(np.argmax(per))
        print('tile %d bytes:' % t)
        print(buf[t * 4096:t * 4096 + 512].tobytes().hex(), flush=True)
        break
print('done', int(acc.sum().item()), flush=True)
