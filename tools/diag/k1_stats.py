"""Diagnostic: K1 chain statistics (tiles without a speculated entry, tiles
re-walked by fs_link, repair rounds) per step of the GET pipeline, for the
request and the reply stream of each connection."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
from zkmi.bench import synthetic as S  # noqa: E402

dev = torch.device('cuda', 0)
batch = 1 << 20
for tag, kw in (('get100', dict(data_bytes=100)),
                ('var0-1024', dict(data_bytes=100, data_dist=(0, 1024)))):
    tree = S.GpuTree(1_000_000, **kw, device=dev, seed=0)
    pipe = S.GetPipeline(tree, batch, seed=1, streams=2)
    for k in range(4):
        pipe.step()
        torch.cuda.synchronize()
        st = [(p.server.scanner.chain_stats(), p.rscanner.chain_stats())
              for p in pipe.subs]
        print(tag, 'step', k, ' | '.join('req %s rep %s' % (a, b)
                                         for a, b in st), flush=True)
    del pipe, tree
    torch.cuda.empty_cache()
