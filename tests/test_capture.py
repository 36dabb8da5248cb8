"""The write workloads as HIP graphs (bench.py captures one step, or one
per rotation, after the warmup and times replays): a replay draws new xids
from the device-side xid counter and every reply is checked on the device,
exactly as in eager steps.  The tree stays steady across replays (nodes
recycled through the free ring).  The watch workload captures a cycle of
steps (its node sets are host draws per step).  Storm steps stay eager:
the session a step serves and the one it expires are host scalars handed
to the serve and expire kernels, and the hash rebuild is a host decision."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _tree(gpu, scratch=0, **kw):
    from zkmi.bench.synthetic import GpuTree
    return GpuTree(20000, 37, fanout=100, device=gpu, spare=1.0,
                   scratch=scratch, **kw)


def _replays(pipe, gpu, eager=3, replays=6):
    acc = torch.zeros(64, dtype=torch.int64, device=gpu)
    for _ in range(eager):
        pipe.step(acc=acc)
    torch.cuda.synchronize()
    assert int(acc.sum().item()) == eager * pipe.n
    g = pipe.capture(acc)
    torch.cuda.synchronize()
    acc.zero_()
    torch.cuda.synchronize()
    for _ in range(replays):
        g.replay()
    torch.cuda.synchronize()
    return int(acc.sum().item())


def test_mix_replays_three_rotations(gpu):
    from zkmi.bench.synthetic import MixPipeline
    from zkmi.ops import _lib
    tree = _tree(gpu)
    pipe = MixPipeline(tree, 3 * 4096, ndirs=64)
    hw = int(tree.counters[_lib.TC_NODES].item())
    assert _replays(pipe, gpu, replays=7) == 7 * pipe.n
    # (creates, sets, deletes kept rotating: the tree did not grow)
    assert int(tree.counters[_lib.TC_NODES].item()) <= hw + pipe.m
    # and eager steps go on after the replays
    assert int(pipe.step().item()) == pipe.n


def _pending_free(tree):
    from zkmi.ops import _lib
    c = tree.counters.cpu().tolist()
    h, pub = c[_lib.TC_FREE_HEAD], c[_lib.TC_FREE_PUB]
    assert c[_lib.TC_FREE_TAIL] == pub
    idx = torch.arange(h, pub, device=tree.device) % tree.free_list.numel()
    return tree.free_list[idx].cpu().tolist()


@pytest.mark.parametrize('hash_factor', [2, 8])
def test_mix_free_ring_compacted(gpu, hash_factor):
    """compact_free: after every served batch the free ring's pending
    entries are exactly the free nodes, ascending (csrc/kernels/tree.hip
    free_count_k / free_scatter_k), eager and replayed; every reply still
    checks out and the tree stays steady.  Wider hash tables (bench.py
    --hash-factor) serve the same."""
    from zkmi.bench.synthetic import MixPipeline
    from zkmi.ops import _lib
    tree = _tree(gpu, compact_free=True, hash_factor=hash_factor)
    assert tree.compact_free
    pipe = MixPipeline(tree, 3 * 4096, ndirs=64)
    acc = torch.zeros(64, dtype=torch.int64, device=gpu)
    for k in range(4):
        pipe.step(acc=acc)
        torch.cuda.synchronize()
        pend = _pending_free(tree)
        assert pend == sorted(pend)
        nn = min(int(tree.counters[_lib.TC_NODES].item()), tree.cap)
        free = torch.nonzero(tree.node_parent[:nn] == -2).flatten()
        assert pend == free.cpu().tolist(), k
    assert int(acc.sum().item()) == 4 * pipe.n
    hw = int(tree.counters[_lib.TC_NODES].item())
    assert _replays(pipe, gpu, eager=2, replays=6) == 6 * pipe.n
    pend = _pending_free(tree)
    assert pend == sorted(pend) and len(pend) > 0
    assert int(tree.counters[_lib.TC_NODES].item()) <= hw + pipe.m


def test_chain_replays(gpu):
    from zkmi.bench.synthetic import ChainPipeline
    tree = _tree(gpu, scratch=1 << 22)
    pipe = ChainPipeline(tree, 4 * 2048, data_bytes=100, ndirs=64)
    assert _replays(pipe, gpu) == 6 * pipe.n


def test_nest_replays(gpu):
    from zkmi.bench.synthetic import NestPipeline
    tree = _tree(gpu, scratch=1 << 22)
    pipe = NestPipeline(tree, 7 * 1024, ndirs=64)
    assert _replays(pipe, gpu) == 6 * pipe.n


def test_watch_replays_a_cycle(gpu):
    """Arm, write-fired notifications and their decode + check, replayed:
    every replay's notifications all arrive and check out (the watches
    re-arm every step, so a cycle's node sets can repeat)."""
    from zkmi.bench.synthetic import GpuTree, WatchPipeline
    tree = GpuTree(20000, 37, fanout=100, device=gpu, seed=0,
                   watch_cap=8192)
    pipe = WatchPipeline(tree, 3000)
    assert pipe.capturable
    assert _replays(pipe, gpu, eager=2, replays=11) == 11 * pipe.n
