"""BASELINE config 5 across GPUs (zkmi/bench/synthetic.py StormPipeline
with a process group): the members hold one replicated tree (every
member applies every member's write batch, in rank order, so sequential
names and zxids agree); each rank's session is born on its own member,
replicated to every member (R3 all-gather into the replicated session
tables), resumed on the NEXT member (the ConnectRequests go there through
an all-gather, the answers come back the same way) with the same id and
password, its second batch created there; its first batch survives the
move and both go at its expiry, which every member applies; the expired
session's resume is refused on any member.  After a move the client reads
its first batch (written through member r) on member r+1: every node is
there, owned by its session (write visibility across members).  Everything
is checked on the device (the pipeline's reply / handshake / removed-count
checks).

Every member's tree digest (path, czxid, mzxid, version, cversion, owner,
data of every live znode) must agree at the end.

Runs world 2 and 3 with gloo on one GPU (ranks share it; RCCL needs one GPU
per rank).  Reference: lib/zk-session.js:265-339 (reattach to another
backend), test/multi-node.test.js:107-165 (a write through one server is
read on another), :233-350 (the ephemeral survives the failover),
test/nasty.test.js:40-103."""

import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _rank(rank, world, port, q, steps, n):
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from zkmi.bench.synthetic import GpuTree, StormPipeline
        dev = torch.device('cuda', 0)
        # every member starts from the same tree (one replicated tree)
        tree = GpuTree(20000, 37, fanout=100, device=dev, seed=0,
                       spare=1.5)
        pipe = StormPipeline(tree, n, ndirs=64, coll_device='cpu')
        oks = [int(pipe.step().item()) for _ in range(steps)]
        # the last step moved the session to the next member: its first
        # batch, written through this member, read there
        found = int(pipe.cross_read().item())
        # the replicated tables: every member knows every live session
        sids = pipe.sessions.sid[pipe.sessions.state == 1].cpu().tolist()
        # one tree: every member's zxid counter agrees
        zx = int(tree.counters[1].item())
        # one tree, byte for byte: every znode's path (the SEQUENTIAL names
        # included), czxid, mzxid, version, cversion, owner and data
        dig = tree.digest()[:2]
        q.put((rank, oks, dict(pipe.stats), bool(pipe.hs_ok.item()),
               sorted({s >> 56 for s in sids}), found, zx, dig))
    except BaseException as e:          # reported by the parent
        q.put((rank, repr(e), None, None, None, None, None, None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 3])
def test_storm_sessions_move_between_members(gpu, world):
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    steps, n = 9, 2048
    procs = [ctx.Process(target=_rank, args=(r, world, port, q, steps, n))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    res = {}
    for _ in range(world):
        r = q.get(timeout=10)
        res[r[0]] = r[1:]
    assert all(p.exitcode == 0 for p in procs), res
    zxids, digests = set(), set()
    for rank, (oks, st, hs_ok, members, found, zx, dig) in res.items():
        assert oks == [n] * steps, (rank, oks)
        assert hs_ok
        # steps 1..9 after the birth in __init__: 5 resumes, all on the
        # next member; 4 births; 4 generations expired (two batches of
        # every member's session on every member), 4 expired resumes
        # refused; every member applied every member's batches
        assert st == {'born': 5, 'resumed': 5, 'expired': 4,
                      'expired_resume_refused': 4, 'cross_rank_resumes': 5,
                      'replicated_writes': (steps + 1) * world * n}, \
            (rank, st)
        # every member's live sessions are in every member's table
        assert members == list(range(1, world + 1)), (rank, members)
        assert found == n, (rank, found)
        zxids.add(zx)
        digests.add(tuple(dig))
    assert len(zxids) == 1, zxids
    # the members re-execute every batch: with SEQUENTIAL numbers assigned
    # in stream order they build the same tree (round 5's atomic numbering
    # named the same creates differently on each member)
    assert len(digests) == 1, digests
