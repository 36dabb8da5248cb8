"""Where the storm's session expiry (csrc/kernels/tree.hip tree_expire_k)
spends its time: per removed node, the hash lookup + tombstone, the
backward shift over the hole and the whole thread, from the kernel's
optional phase clocks (zk_tree_expire_debug), over the expiries of a few
storm steps (BASELINE config 5 shape).

  python tools/microbench/expire_probe.py [--steps 4]

Prints per expiry: removed nodes, the launch span, and p50 / p90 / p99 of
each phase, split by start time into the launch's quarters (the later
workgroups start once earlier ones retire).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from zkmi.bench import synthetic as S  # noqa: E402
from zkmi.ops import _lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--steps', type=int, default=4)
ap.add_argument('--batch', type=int, default=1 << 20)
ap.add_argument('--nodes', type=int, default=1000000)
ap.add_argument('--ndirs', type=int, default=1024)
a = ap.parse_args()
dev = torch.device('cuda', 0)
spare = (a.batch * 3 + 8192) / a.nodes
tree = S.GpuTree(a.nodes, 100, device=dev, seed=0, spare=spare + 0.05,
                 hash_factor=2)
pipe = S.StormPipeline(tree, a.batch, ndirs=a.ndirs)
acc = torch.zeros(64, dtype=torch.int64, device=dev)
for _ in range(3):
    pipe.step(acc=acc)
torch.cuda.synchronize()
L = _lib.lib()
buf = torch.zeros(4 * tree.cap, dtype=torch.int32, device=dev)
L.tree_expire_debug(buf)


def pct(v, q):
    return float(np.percentile(v, q)) if len(v) else float('nan')


for s in range(a.steps):
    buf.zero_()
    pipe.step(acc=acc)
    torch.cuda.synchronize()
    d = buf.view(-1, 4).cpu().numpy()
    rows = d[d[:, 3] > 0].astype(np.int64)
    if len(rows) == 0:
        print('step %d: no expiry' % s, flush=True)
        continue
    start = (rows[:, 0] - rows[:, 0].min()) & 0xFFFFFFFF
    us = 1.0 / 100.0
    end = start + rows[:, 3]
    print('step %d removed %d span %.1f us' % (s, len(rows),
                                               end.max() * us), flush=True)
    span = max(int(start.max()), 1)
    for qi in range(4):
        sel = (start * 4 // (span + 1)) == qi
        r = rows[sel]
        if not len(r):
            continue
        ph = {'lookup+tomb': r[:, 1] * us, 'shift': r[:, 2] * us,
              'thread': r[:, 3] * us}
        print('  q%d start %6.1f us n %7d | ' % (qi, start[sel].min() * us,
                                                 len(r)) +
              ' | '.join('%s %.2f/%.2f/%.2f' % (k, pct(v, 50), pct(v, 90),
                                                pct(v, 99))
                         for k, v in ph.items()), flush=True)
L.tree_expire_debug(torch.empty(0, dtype=torch.int32, device=dev))
ok = int(acc[0].item())
print('replies ok %d' % ok, flush=True)
