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


def _tree(gpu, scratch=0):
    from zkmi.bench.synthetic import GpuTree
    return GpuTree(20000, 37, fanout=100, device=gpu, spare=1.0,
                   scratch=scratch)


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
