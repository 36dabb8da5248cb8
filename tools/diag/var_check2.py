"""Diagnostic: variable-size GET at bench scale (1M nodes, 1M batch)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
from zkmi.bench import synthetic as S  # noqa: E402


def run(nodes, batch, streams, dd, pad):
    dev = torch.device('cuda', 0)
    tree = S.GpuTree(nodes, 0, device=dev, data_dist=dd, name_pad=pad)
    p = S.GetPipeline(tree, batch, streams=streams)
    acc = torch.zeros(1, dtype=torch.int64, device=dev)
    for _ in range(3):
        p.step(acc=acc)
    sub = p.subs[0] if p.subs else p
    idx, rep, rx, ft = sub.last
    n = sub.batch
    want = tree.data_len[idx]
    bad = ((rep.status[:n] != 0) | (rep.err[:n] != 0) |
           (rep.pay_len[:n] != want))
    nb = int(bad.sum())
    first = bad.nonzero().flatten()[:4].tolist()
    print(nodes, batch, streams, dd, pad, 'ok', int(acc.item()), '/',
          3 * batch, 'sub0 bad', nb, 'frames', ft.host_result(),
          [(i, int(rep.status[i]), int(rep.err[i]), int(rep.pay_len[i]),
            int(want[i])) for i in first], flush=True)
    del p, tree
    torch.cuda.empty_cache()


if __name__ == '__main__':
    run(1_000_000, 1 << 20, 2, (0, 1024), (0, 16))
    run(1_000_000, 1 << 20, 1, (0, 1024), None)
    run(1_000_000, 1 << 18, 1, (0, 1024), None)
    run(100_000, 1 << 16, 1, (0, 1024), None)
