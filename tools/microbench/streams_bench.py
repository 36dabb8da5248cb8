"""Per-step time of the get pipeline vs the number of concurrent pipelined
connections (HIP streams) per GPU, at a fixed 1M-request batch."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
from zkmi.bench import synthetic as S  # noqa: E402


def run(tree, batch, streams, steps=20, warmup=3):
    p = S.GetPipeline(tree, batch, seed=1, streams=streams)
    acc = torch.zeros(1, dtype=torch.int64, device=tree.device)
    for _ in range(warmup):
        p.step(acc=acc)
    torch.cuda.synchronize()
    acc.zero_()
    t = time.perf_counter()
    for _ in range(steps):
        p.step(acc=acc)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / steps
    ok = int(acc.item())
    assert ok == batch * steps, (ok, batch * steps)
    return dt


def main():
    dev = torch.device('cuda', 0)
    tree = S.GpuTree(1_000_000, 100, device=dev, seed=0)
    batch = int(os.environ.get('BATCH', 1 << 20))
    for k in [int(x) for x in os.environ.get('STREAMS', '1,2,3,4').split(',')]:
        dt = run(tree, batch, k)
        print('streams=%d batch=%d  %.3f ms/step  %.1f M ops/s'
              % (k, batch, dt * 1e3, batch / dt / 1e6), flush=True)


if __name__ == '__main__':
    main()
