"""Diagnostic: K1 over large random streams with reply-like frame sizes,
against the host framer."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
from zkmi.ops import batch as B  # noqa: E402


def stream(nf, lo, hi, seed):
    rng = np.random.default_rng(seed)
    lens = rng.integers(lo, hi + 1, nf).astype(np.int64)
    starts = np.zeros(nf, np.int64)
    np.cumsum(lens[:-1] + 4, out=starts[1:])
    total = int(starts[-1] + lens[-1] + 4)
    buf = rng.integers(0, 256, total, dtype=np.uint8)
    for k in range(4):                      # big-endian length words
        buf[starts + k] = ((lens >> (8 * (3 - k))) & 0xff).astype(np.uint8)
    return buf, starts, lens


def main():
    dev = torch.device('cuda', 0)
    for nf, lo, hi, win in ((500_000, 88, 1112, 2048),
                            (500_000, 88, 1112, 1024),
                            (500_000, 88, 300, 512),
                            (200_000, 88, 1112, 2048)):
        for seed in range(3):
            buf, starts, lens = stream(nf, lo, hi, seed)
            d = torch.from_numpy(buf).to(dev)
            sc = B.FrameScanner(nf + 16, dev, window=win)
            ft = sc.scan(d, len(buf))
            r = ft.host_result()
            off = ft.off[:min(r['frames'], nf)].cpu().numpy()
            want = starts + 4
            first = -1
            m = min(len(off), nf)
            neq = np.nonzero(off[:m] != want[:m])[0]
            if len(neq):
                first = int(neq[0])
            print(nf, lo, hi, win, seed, r, 'first mismatch', first,
                  sc.chain_stats(), flush=True)
            if first >= 0:
                j = first
                print('  want', want[j - 2:j + 3].tolist(), 'got',
                      off[j - 2:j + 3].tolist(), 'tile', want[j] // 4096,
                      flush=True)


if __name__ == '__main__':
    main()
