"""R2 on the GPU (zkmi/parallel/sharded.py, csrc/kernels/route.hip): reads
routed to the rank owning the path's hash shard, bytes moved with
all_to_all.  The multi-rank case runs two ranks on one GPU with gloo
collectives (RCCL needs one GPU per rank) and checks the routed replies
byte for byte against serving the same requests from an unsharded tree."""

import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_router_matches_host_hash(gpu):
    """route.hip's owners equal the host FNV-1a mirror; the split is stable
    and grouped by owner."""
    from zkmi.bench.synthetic import GpuTree, path_owner
    from zkmi.parallel.sharded import ShardedGetPipeline
    tree = GpuTree(20000, 37, fanout=100, device=gpu, seed=0)
    pipe = ShardedGetPipeline(tree, 5000)
    pipe.step()
    from zkmi.ops import _lib
    L = _lib.lib()
    for W in (3, 8):
        pipe.rws = torch.empty(L.route_workspace(5000, W),
                               dtype=torch.int64, device=gpu)
        cnt = torch.empty(W, dtype=torch.int64, device=gpu)
        L.route_requests(5000, W, pipe.poff, pipe.plen, tree.path_arena,
                         pipe.idx, pipe.xid, pipe.owner, pipe.idx_s,
                         pipe.xid_s, pipe.poff_s, pipe.plen_s, cnt, pipe.rws)
        arena = tree.path_arena.cpu().numpy().tobytes()
        po, pl = pipe.poff.cpu().tolist(), pipe.plen.cpu().tolist()
        want = path_owner([arena[o:o + n] for o, n in zip(po, pl)], W)
        assert pipe.owner.cpu().numpy().tolist() == want.tolist()
        order = np.argsort(want, kind='stable')
        assert pipe.idx_s.cpu().numpy().tolist() == \
            pipe.idx.cpu().numpy()[order].tolist()
        assert cnt.cpu().tolist() == np.bincount(want, minlength=W).tolist()


def test_sharded_get_one_rank(gpu):
    from zkmi.bench.synthetic import GpuTree
    from zkmi.parallel.sharded import ShardedGetPipeline
    tree = GpuTree(20000, 37, fanout=100, device=gpu, seed=0, shard=(0, 1))
    pipe = ShardedGetPipeline(tree, 4096)
    for _ in range(3):
        assert int(pipe.step().item()) == 4096


def _mask_zxid(stream):
    """Reply frames with the header zxid zeroed: each GPU server's zxid
    advances with the batches it served, the bodies must match exactly."""
    from zkmi import jute
    frames, _, bad = jute.scan_frames(stream)
    assert bad < 0
    return [b'%s\0\0\0\0\0\0\0\0%s' % (stream[o:o + 4], stream[o + 12:o + n])
            for o, n in frames]


def _rank(rank, world, port, q):
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from zkmi.bench.synthetic import GpuTree, GpuServer
        from zkmi.ops import batch as B
        from zkmi.parallel.sharded import ShardedGetPipeline
        dev = torch.device('cuda', 0)
        n = 3000
        tree = GpuTree(20000, 37, fanout=100, device=dev, seed=0,
                       shard=(rank, world), ctime_ms=1 << 40)
        pipe = ShardedGetPipeline(tree, n, seed=5, coll_device='cpu')
        oks = [int(pipe.step().item()) for _ in range(3)]
        rep, crx, ft = pipe.last
        got = bytes(crx.cpu().numpy().tobytes())
        # the same (routed-order) requests served by an unsharded replica
        full = GpuTree(20000, 37, fanout=100, device=dev, seed=0,
                       ctime_ms=1 << 40)
        srv = GpuServer(full, n, n * 300)
        rb = B.RequestBatch(n, pipe.opcode, pipe.xid_s, pipe.zero32,
                            pipe.poff_s, pipe.plen_s, pipe.zero64,
                            pipe.zero32, pipe.zero32, tree.path_arena,
                            tree.slab, pipe.acl_off, pipe.acl_len,
                            pipe.acl_arena)
        tx, _, total, _ = B.encode_requests(rb, B.XidTable(bits=14,
                                                           device=dev))
        out, rtotal, _, _ = srv.serve(tx, total)
        want = bytes(out[:int(rtotal.item())].cpu().numpy().tobytes())
        q.put((rank, oks, _mask_zxid(got) == _mask_zxid(want), len(got),
               dict(pipe.stats)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 3])
def test_sharded_get_multi_rank_gloo(gpu, world):
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    assert all(p.exitcode == 0 for p in procs)
    res = {}
    for _ in range(world):
        r = q.get(timeout=5)
        res[r[0]] = r[1:]
    for rank, (oks, same, nbytes, st) in res.items():
        assert oks == [3000] * 3, (rank, oks)
        assert same and nbytes > 3000 * 100, rank
        # most reads are remote: bytes really moved between the ranks
        assert st['remote_reqs'] > 3 * 3000 * (world - 1) / world * 0.8
        assert st['bytes_sent'] > 0 and st['bytes_recv'] > 0
