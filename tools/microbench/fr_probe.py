"""Forced-route capture probe (one rank, one GPU): which part of the
two-connection sharded step breaks stream capture.

  --mode copy    the all-to-all replaced by a device copy (what a one-rank
                 all_to_all_single moves), no RCCL in the graph
  --mode origin  the collectives issued from the capture's origin stream
  --mode comm    the collectives on the pipeline's comm stream (default)
"""
import argparse
import socket

import torch
import torch.distributed as dist

from zkmi.bench.synthetic import GpuTree
from zkmi.parallel.sharded import ShardedGetPipeline

ap = argparse.ArgumentParser()
ap.add_argument('--mode', default='comm')
ap.add_argument('--streams', type=int, default=2)
a = ap.parse_args()
dev = torch.device('cuda', 0)
s = socket.socket()
s.bind(('127.0.0.1', 0))
port = s.getsockname()[1]
s.close()
dist.init_process_group('nccl', device_id=dev, rank=0, world_size=1,
                        init_method='tcp://127.0.0.1:%d' % port)
tree = GpuTree(20000, 100, fanout=100, device=dev, seed=0, shard=(0, 1))
n = 8192
pipe = ShardedGetPipeline(tree, n, seed=3, streams=a.streams, force_route=True)
if a.mode == 'copy':
    pipe.a2a = lambda out, inp: out.copy_(inp)
elif a.mode == 'origin':
    origin = {}
    real = pipe.a2a

    def a2a(out, inp):
        o = origin.get('s')
        if o is None:
            return real(out, inp)
        cur = torch.cuda.current_stream(dev)
        o.wait_stream(cur)
        with torch.cuda.stream(o):
            dist.all_to_all_single(out, inp)
        cur.wait_stream(o)
        return out
    pipe.a2a = a2a
    pipe.comm = None
acc = torch.zeros(64, dtype=torch.int64, device=dev)
for _ in range(2):
    pipe.step(acc=acc)
torch.cuda.synchronize()
print('eager ok', int(acc.sum().item()) == 2 * n, flush=True)
if a.mode == 'origin':
    # capture by hand so the origin stream is known
    for c in pipe.subs:
        c.device_seed()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    st = torch.cuda.Stream(dev)
    with torch.cuda.graph(g, stream=st, capture_error_mode='thread_local'):
        origin['s'] = st
        pipe.step(acc=acc)
else:
    g = pipe.capture(acc)
torch.cuda.synchronize()
print('captured', flush=True)
acc.zero_()
for _ in range(3):
    g.replay()
torch.cuda.synchronize()
print('replay ok', int(acc.sum().item()) == 3 * n, flush=True)
g = pipe = None
import gc
gc.collect()
torch.cuda.synchronize()
dist.destroy_process_group()
print('done', flush=True)
