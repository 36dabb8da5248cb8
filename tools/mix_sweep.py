"""Mix-workload sweep (bench --workload mix internals): step time vs number
of parent directories, to separate parent-Stat contention from the rest of
the create/set/delete path.  Usage: python tools/mix_sweep.py [ndirs ...]"""

import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from zkmi.bench import synthetic as S  # noqa: E402


def run(ndirs, batch=1 << 20, steps=10):
    tree = S.GpuTree(1_000_000, 100, spare=(batch + 8192) / 1e6 + 0.05 +
                     ndirs / 1e6)
    pipe = S.MixPipeline(tree, batch, 100, ndirs=ndirs)
    for _ in range(3):
        pipe.step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        pipe.step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / steps
    print('ndirs %6d: %.3f ms/step, %.0f M ops/s' % (ndirs, dt * 1e3,
                                                    pipe.n / dt / 1e6),
          flush=True)
    del pipe, tree
    torch.cuda.empty_cache()


if __name__ == '__main__':
    for nd in [int(x) for x in sys.argv[1:]] or [64, 1024, 16384, 65536]:
        run(nd)
