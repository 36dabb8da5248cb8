"""Diagnostic: K1 chain statistics of the GET pipeline's request and reply
scans (tiles without a speculated entry / re-walked / repair rounds) and
the time of one scan, for several data sizes."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
from zkmi.bench import synthetic as S  # noqa: E402


def main():
    dev = torch.device('cuda', 0)
    for kw in ({'data_bytes': 100}, {'data_bytes': 512},
               {'data_bytes': 0, 'data_dist': (0, 1024)}):
        tree = S.GpuTree(1_000_000, device=dev, **kw)
        p = S.GetPipeline(tree, 1 << 19)
        for _ in range(3):
            p.step()
        torch.cuda.synchronize()
        idx, rep, rx, ft = p.last
        rs = p.rscanner
        print(kw, 'req', p.server.scanner.chain_stats(), 'reply',
              rs.chain_stats(), 'window', rs.window, flush=True)
        n = int(ft.result[1].item())
        for _ in range(3):
            rs.scan(rx, n)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            rs.scan(rx, n)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 10
        print('   reply scan %.1f us for %.1f MB (%.2f TB/s)' % (
            dt * 1e6, n / 1e6, n / dt / 1e12), rs.chain_stats(), flush=True)
        del p, tree
        torch.cuda.empty_cache()


if __name__ == '__main__':
    main()
