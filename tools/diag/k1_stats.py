"""K1 one-pass chain counters for the benchmark's request and reply streams
(how many tiles took a speculated entry vs waited, repairs, restarts)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))))
import torch  # noqa: E402

from zkmi.bench import synthetic as S  # noqa: E402


def main():
    dev = torch.device('cuda', 0)
    tree = S.GpuTree(1_000_000, 100, device=dev)
    pipe = S.GetPipeline(tree, 1 << 19)
    for _ in range(3):
        ok = pipe.step()
    torch.cuda.synchronize()
    print('ok', int(ok.item()), 'of', 3 << 19)
    print('request stream', pipe.server.scanner.chain_stats())
    print('reply stream  ', pipe.rscanner.chain_stats())
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(10):
        pipe.step()
    torch.cuda.synchronize()
    print('ms/step (1 connection, 512K)', (time.perf_counter() - t) * 100)


if __name__ == '__main__':
    main()
