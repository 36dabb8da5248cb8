"""Diagnostic: GET pipeline over variable-size data; per data range, the
fraction of correct replies and the first wrong ones."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
from zkmi.bench import synthetic as S  # noqa: E402


def main():
    dev = torch.device('cuda', 0)
    for lo, hi in ((0, 200), (0, 400), (0, 600), (0, 1024), (900, 1024),
                   (300, 340)):
        tree = S.GpuTree(20000, 0, fanout=100, device=dev, data_dist=(lo, hi))
        p = S.GetPipeline(tree, 8192)
        ok = int(p.step().item())
        idx, rep, rx, ft = p.last
        n = 8192
        want = tree.data_len[idx]
        bad = ((rep.status[:n] != 0) | (rep.err[:n] != 0) |
               (rep.pay_len[:n] != want)).nonzero().flatten()[:5].tolist()
        print('range', lo, hi, 'ok', ok, 'frames', ft.host_result(),
              'first bad', [(i, int(rep.status[i]), int(rep.err[i]),
                             int(rep.pay_len[i]), int(want[i]))
                            for i in bad], flush=True)


if __name__ == '__main__':
    main()
