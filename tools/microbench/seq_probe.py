"""Where seq_group_k's time goes on the storm step (BASELINE config 5): the
kernel's per-chunk phase clocks (csrc/kernels/tree.hip, zk_tree_seq_debug),
summarised over the 1024-request chunks of one numbering pass.

  python tools/microbench/seq_probe.py [--steps 6]

Phases per chunk (one 1024-thread workgroup): parse (frame header, flags
and parent path; an extra barrier closes it), the group key's table probe
and the group ticket, the chunk-local ids in LDS, the rank / count / bitmap
tail — split into the launch's first resident round of workgroups and the
later ones.  Also the whole launch span.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))))

import torch  # noqa: E402

from zkmi.bench import synthetic as S  # noqa: E402
from zkmi.ops import _lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--steps', type=int, default=6)
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
pipe.step(acc=acc)
# (room for servers sized past the batch: 5 int64 per chunk of 4 batches)
nch = 4 * ((a.batch + 1023) // 1024)
buf = torch.zeros(5 * nch, dtype=torch.int64, device=dev)
L = _lib.lib()
L.tree_seq_debug(buf)


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * len(v)))] if v else float('nan')


for s in range(a.steps):
    buf.zero_()
    pipe.step(acc=acc)
    torch.cuda.synchronize()
    d = buf.view(nch, 5).cpu().tolist()
    rows = [r for r in d if r[0] and r[3]]
    if not rows:
        print('step %d: no numbered chunk' % s)
        continue
    t0 = min(r[0] for r in rows)
    us = lambda x: x / 100.0   # noqa: E731  (100 MHz ticks)
    span = us(max(r[3] for r in rows) - t0)
    print('step %d chunks %d span %.1f us' % (s, len(rows), span))
    # the first resident round of workgroups against the later ones
    for tag, sel in (('first', lambda r: us(r[0] - t0) < 10),
                     ('later', lambda r: us(r[0] - t0) >= 10)):
        rr = [r for r in rows if sel(r)]
        if not rr:
            continue
        ph = {'start': [us(r[0] - t0) for r in rr],
              'parse': [us(r[4] - r[0]) for r in rr],
              'key+ticket': [us(r[1] - r[4]) for r in rr],
              'ids': [us(r[2] - r[1]) for r in rr],
              'tail': [us(r[3] - r[2]) for r in rr]}
        print('  %-5s %4d chunks | ' % (tag, len(rr)) + ' | '.join(
            '%s p50 %.2f p90 %.2f' % (k, pct(v, .5), pct(v, .9))
            for k, v in ph.items()), flush=True)
L.tree_seq_debug(torch.empty(0, dtype=torch.int64, device=dev))
