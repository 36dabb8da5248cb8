"""Per-chunk step times of a write workload over a long run (the bench's
sustained window disagreed with its timed window): replays of the captured
cycle, timed in chunks of 50, with the tree counters after each chunk.

  python tools/microbench/sustain_probe.py --workload mix --steps 800
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))))

import torch  # noqa: E402

from zkmi.bench import synthetic as S  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--workload', default='mix')
ap.add_argument('--steps', type=int, default=800)
ap.add_argument('--chunk', type=int, default=50)
ap.add_argument('--batch', type=int, default=1 << 20)
ap.add_argument('--nodes', type=int, default=1000000)
ap.add_argument('--eager', action='store_true')
ap.add_argument('--no-compact', action='store_true',
                help='no free-ring compaction after each batch')
ap.add_argument('--hash-factor', type=int, default=8)
ap.add_argument('--sort-free', type=int, default=0,
                help='sort the pending free ring after every N chunks '
                '(0: never): tests the free-ring locality hypothesis')
ap.add_argument('--zxid', type=lambda x: int(x, 0), default=None,
                help='start the tree at this zxid')
a = ap.parse_args()
dev = torch.device('cuda', 0)
w = a.workload
if w == 'watch':
    tree = S.GpuTree(a.nodes, 100, device=dev, seed=0, watch_cap=2 * a.batch)
    pipe = S.WatchPipeline(tree, a.batch, seed=0)
else:
    spare = (a.batch + 8192) / a.nodes
    scratch = (a.batch // 2 + 64) * (80 + 112) if w in ('chain', 'nest') else 0
    tree = S.GpuTree(a.nodes, 100, device=dev, seed=0, spare=spare + 0.05,
                     scratch=scratch, hash_factor=a.hash_factor,
                     compact_free=not a.no_compact)
    pipe = {'mix': lambda: S.MixPipeline(tree, a.batch, 100, seed=0),
            'nest': lambda: S.NestPipeline(tree, a.batch, seed=0),
            'chain': lambda: S.ChainPipeline(tree, a.batch, 100, seed=0)}[w]()
if a.zxid is not None:
    tree.counters[1] = a.zxid                # TC_ZXID
acc = torch.zeros(64, dtype=torch.int64, device=dev)
for _ in range(3):
    pipe.step(acc=acc)
run = lambda: pipe.step(acc=acc)   # noqa: E731
if not a.eager:
    g = pipe.capture(acc)
    run = g.replay
torch.cuda.synchronize()
acc.zero_()
done = 0
chunks = 0
print('workload', w, 'per step', getattr(pipe, 'n', a.batch), flush=True)
while done < a.steps:
    if a.sort_free and chunks % a.sort_free == 0:
        torch.cuda.synchronize()
        n_sorted = tree.sort_free()
        print('sorted %d free entries' % n_sorted, flush=True)
    chunks += 1
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.chunk):
        run()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    done += a.chunk
    ok = int(acc.sum().item())
    pend, near = tree.free_order()
    print('steps %5d  %.3f ms/step  ok %d  free pending %d  one-apart %.3f '
          ' counters %s' % (done, 1e3 * dt / a.chunk, ok, pend, near,
                            tree.counters.cpu().tolist()), flush=True)
