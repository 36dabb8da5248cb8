import sys, torch
sys.path.insert(0, '.')
from zkmi.bench.synthetic import GpuTree, NestPipeline
dev = torch.device('cuda', 0)
CASES = ((20000, 7 * 1024, 64), (20000, 7 * 1024, 1024),
         (200000, 7 * 16384, 1024), (1000000, 7 * 149796, 1024))
for nodes, batch, ndirs in CASES:
    tree = GpuTree(nodes, 100, fanout=1000 if nodes >= 200000 else 100,
                   device=dev, spare=(batch + 8192) / nodes + 0.05,
                   scratch=(batch // 2 + 64) * 192)
    pipe = NestPipeline(tree, batch, ndirs=ndirs)
    for s in range(3):
        ok = int(pipe.step().item())
        rb, rep = pipe.last
        n = rb.n
        err = rep.err[:n].view(-1, 7).cpu()
        hist = [dict(zip(*[x.tolist() for x in
                           torch.unique(err[:, c], return_counts=True)]))
                for c in range(7)]
        print(nodes, batch, ndirs, 'step', s, ok, '/', n, hist,
              pipe.drv.server.order_stats(), flush=True)
