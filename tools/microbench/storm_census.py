"""Storm (BASELINE config 5) over a long run: step time per chunk of
captured replays and the hash index census after each chunk (entries in
use, tombstones; GpuTree.digest), so the index's growth under
never-reused SEQUENTIAL names is seen directly.

  python tools/microbench/storm_census.py --steps 1000 --hash-factor 2

The storm runs with no index rebuild (its expiry reclaims the index,
csrc/kernels/tree.hip ht_shift); ``rehashes`` counts any that happen.
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
ap.add_argument('--steps', type=int, default=1000)
ap.add_argument('--chunk', type=int, default=100)
ap.add_argument('--batch', type=int, default=1 << 20)
ap.add_argument('--nodes', type=int, default=1000000)
ap.add_argument('--ndirs', type=int, default=1024)
ap.add_argument('--hash-factor', type=int, default=2)
a = ap.parse_args()
dev = torch.device('cuda', 0)
spare = (a.batch * 3 + 8192) / a.nodes
tree = S.GpuTree(a.nodes, 100, device=dev, seed=0, spare=spare + 0.05,
                 hash_factor=a.hash_factor)
print('hash entries', tree.hcap, 'node slots', tree.cap, flush=True)
pipe = S.StormPipeline(tree, a.batch, ndirs=a.ndirs)
acc = torch.zeros(64, dtype=torch.int64, device=dev)
for _ in range(3):
    pipe.step(acc=acc)
g = pipe.capture(acc)
torch.cuda.synchronize()
acc.zero_()
done = 0
rehash = tree.rehash
nre = [0]


def counted():
    nre[0] += 1
    rehash()


tree.rehash = counted
while done < a.steps:
    k = min(a.chunk, a.steps - done)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        g.replay()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    done += k
    d, live, used, tomb = tree.digest()
    print('steps %5d  %.4f ms/step  live %d  entries %d  tombstones %d '
          '(%.2f%% of the table)  rehashes %d' % (
              done, dt / k * 1e3, live, used, tomb, 100.0 * used / tree.hcap,
              nre[0]), flush=True)
ok = int(acc[0].item())
want = pipe.n * a.steps
print('replies ok %d of %d' % (ok, want), flush=True)
if ok != want:
    print('diagnose', pipe.diagnose())
    sys.exit(1)
