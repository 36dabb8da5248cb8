"""Prefix-scan engine microbenchmark: MFMA byte-plane vs shuffle scan
(csrc/kernels/scan.hip) over record-size-like inputs.  Prints one line per
(engine, dtype, n, value range) with the per-scan time (CUDA events, median
of 50) and the effective HBM rate (read input + write int64 prefix)."""

import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
from zkmi.ops import _lib, batch as B  # noqa: E402


def bench(x, reps=50):
    for _ in range(5):
        B.exclusive_scan(x)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        B.exclusive_scan(x)
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts)


def main():
    dev = torch.device('cuda', 0)
    for n in (1 << 16, 1 << 20, 1 << 22, 1 << 24):
        for dt in (torch.int32, torch.int64):
            for hi in (200, 60000):
                x = torch.randint(0, hi, (n,), dtype=dt, device=dev)
                for mode, name in ((_lib.SCAN_SHFL, 'shfl'),
                                   (_lib.SCAN_MFMA_W1, 'mfw1'),
                                   (_lib.SCAN_MFMA_W4, 'mfw4')):
                    _lib.set_scan_mode(mode)
                    us = bench(x)
                    gbs = n * (x.element_size() + 8) / us / 1e3
                    print('scan %-4s %-5s n=%-9d hi=%-6d %9.1f us  %7.1f GB/s'
                          % (name, str(dt)[6:], n, hi, us, gbs), flush=True)
    _lib.set_scan_mode(_lib.SCAN_MFMA)


if __name__ == '__main__':
    main()
