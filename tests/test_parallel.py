"""Multi-process tests of the node layer (zkmi.parallel, R1-R4) on the gloo
backend, world_size 2 — the same code runs on RCCL ("nccl") on MI355X.
Both ranks talk to one in-process fake server owned by the parent."""

import os
import socket
import sys
import time
import traceback

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, mport, zport, scenario, errq):
    try:
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.join(ROOT, 'tests'))
        import torch.distributed as dist
        dist.init_process_group('gloo', init_method='tcp://127.0.0.1:%d'
                                % mport, rank=rank, world_size=world)
        from zkhelpers import client, wait_for
        from zkmi.parallel import SessionGroup, owner_of
        c = client([{'address': '127.0.0.1', 'port': zport}],
                   session_timeout=4000)
        c.wait_connected(10)
        g = SessionGroup(c)
        globals()['_scn_' + scenario](rank, world, c, g, dist, wait_for,
                                      owner_of, zport)
        dist.barrier()
        dist.destroy_process_group()
    except BaseException:
        errq.put((rank, traceback.format_exc()))
        raise


def _run(scenario, world=2):
    from zkmi.server import FakeZKServer
    zk = FakeZKServer(tick_ms=250)
    try:
        ctx = mp.get_context('spawn')
        errq = ctx.SimpleQueue()
        mp.start_processes(_worker, args=(world, _free_port(), zk.port,
                                          scenario, errq),
                           nprocs=world, join=True, start_method='spawn')
        return zk
    except Exception:
        msgs = []
        while not errq.empty():
            msgs.append('rank %d:\n%s' % errq.get())
        raise AssertionError('\n'.join(msgs) or 'worker failed')
    finally:
        zk.shutdown()


# -- scenarios (run inside each rank) ----------------------------------------

def _scn_metrics(rank, world, c, g, dist, wait_for, owner_of, zport):
    for i in range(rank + 1):
        c.call_sync('ping')
    tot = g.allreduce_metrics(extra={'pings': rank + 1})
    assert tot['pings'] == sum(range(1, world + 1))
    assert tot['zookeeper_events{evtype="session"}'] == world
    assert tot['zookeeper_events{evtype="connect"}'] >= world


def _scn_batched_get(rank, world, c, g, dist, wait_for, owner_of, zport):
    if rank == 0:
        for i in range(6):
            c.call_sync('create', '/bg%d' % i, b'v%d' % i, {})
    dist.barrier()
    mine = ['/bg%d' % i for i in range(rank, rank + 5)] + ['/nope']
    res = g.batched_get(mine)
    for p, r in zip(mine, res):
        if p == '/nope':
            assert getattr(r, 'code', None) == 'NO_NODE'
        else:
            assert r[0] == ('v' + p[3:]).encode(), (p, r)
            assert r[1].dataLength == len(r[0])
    # 2 ranks x 6 requested paths -> 7 unique (bg0..bg5, /nope), each
    # fetched once on the node
    assert g.stats['batched_get_unique'] == 7
    assert g.stats['batched_get_requested'] == 12


def _scn_batched_get_timeout(rank, world, c, g, dist, wait_for, owner_of,
                             zport):
    """A rank whose session never answers: its reads fail with
    OPERATION_TIMEOUT on every rank, and the collective still completes (no
    rank is left blocked in the second all-gather)."""
    if rank == 0:
        for i in range(8):
            c.call_sync('create', '/bt%d' % i, b'v%d' % i, {})
    dist.barrier()
    paths = ['/bt%d' % i for i in range(8)]
    owners = set(owner_of(p, world) for p in paths)
    assert owners == set(range(world))       # both ranks own some paths
    if rank == 1:
        c.get = lambda path, cb: None          # replies never come
    res = g.batched_get(paths, timeout=0.5)
    for p, r in zip(paths, res):
        if owner_of(p, world) == 1:
            assert getattr(r, 'code', None) == 'OPERATION_TIMEOUT', (p, r)
        else:
            assert r[0] == ('v' + p[3:]).encode(), (p, r)


def _scn_watch_fanout(rank, world, c, g, dist, wait_for, owner_of, zport):
    path = '/fan'
    if rank == 0:
        c.call_sync('create', path, b'a', {})
    dist.barrier()
    seen = []
    g.watcher(path).on('dataChanged', lambda d, s: seen.append(d))
    # the owner's initial arm publishes the current data
    _tick_until(g, dist, lambda: len(seen) >= 1)
    assert seen == [b'a'], seen
    dist.barrier()
    if rank == 0:
        c.call_sync('set', path, b'b', -1)
    _tick_until(g, dist, lambda: len(seen) >= 2)
    assert seen == [b'a', b'b'], seen


def _scn_watch_kinds(rank, world, c, g, dist, wait_for, owner_of, zport):
    """Every event kind crosses the fan-out as wire frames (NOTIFICATION +
    the forwarded GET_CHILDREN2 / EXISTS reply) and arrives with its
    values on every rank."""
    path = '/wk'
    if rank == 0:
        c.call_sync('create', path, b'p', {})
    dist.barrier()
    kids, gone = [], []
    g.watcher(path).on('childrenChanged', lambda ch, st: kids.append(
        (sorted(ch), st.numChildren))).on('deleted', lambda: gone.append(1))
    _tick_until(g, dist, lambda: len(kids) >= 1)
    assert kids == [([], 0)], kids
    dist.barrier()
    if rank == 0:
        c.call_sync('create', path + '/c1', b'', {})
    _tick_until(g, dist, lambda: len(kids) >= 2)
    assert kids[-1] == (['c1'], 1), kids
    dist.barrier()
    if rank == 0:
        c.call_sync('delete', path + '/c1', -1)
        c.call_sync('delete', path, -1)
    _tick_until(g, dist, lambda: len(gone) >= 1)
    assert g.fan.stats['decoded_host'] >= 2 * len(kids)


def _tick_until(g, dist, cond, rounds=200):
    """tick() is a collective: every rank must call it the same number of
    times, so the stop decision is all-reduced."""
    import torch
    for _ in range(rounds):
        g.tick()
        flag = torch.tensor([1 if cond() else 0])
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if flag.item():
            return
        time.sleep(0.02)
    raise AssertionError('condition not reached')


def _scn_session_failover(rank, world, c, g, dist, wait_for, owner_of,
                          zport):
    if rank == 0:
        c.call_sync('create', '/owner', b'r0', {'flags': ['EPHEMERAL']})
        c.watcher('/owner').on('deleted', lambda *a: None)
    dist.barrier()
    cred = g.broadcast_session(0)
    assert cred['sessionId'] != 0 and len(cred['passwd']) == 16
    assert '/owner' in cred['watches'].get('createdOrDeleted', [])
    dist.barrier()
    if rank == 0:
        c.abandon()                  # rank 0 "dies" without closing
    dist.barrier()
    if rank == 1:
        from zkhelpers import client
        c2 = client([{'address': '127.0.0.1', 'port': zport}],
                    session_timeout=4000, session=cred)
        c2.wait_connected(10)
        assert c2.getSession().getSessionId() == '%016x' % (
            cred['sessionId'] & 0xffffffffffffffff)
        st = c2.call_sync('stat', '/owner')
        assert st.ephemeralOwner == cred['sessionId']
        time.sleep(4.5)              # longer than the session timeout
        assert c2.call_sync('get', '/owner')[0] == b'r0'
        c2.close_sync(10)            # closing the adopted session frees it
        c3 = client([{'address': '127.0.0.1', 'port': zport}])
        c3.wait_connected(10)
        assert wait_for(lambda: _missing(c3, '/owner'), 5)
        c3.close_sync(10)


def _missing(c, p):
    try:
        c.call_sync('stat', p)
        return False
    except Exception as e:
        return getattr(e, 'code', None) == 'NO_NODE'


# -- tests --------------------------------------------------------------------

@pytest.mark.parametrize('scenario', ['metrics', 'batched_get',
                                      'batched_get_timeout', 'watch_fanout'])
def test_group_collectives(scenario):
    _run(scenario)


def test_session_failover_between_ranks():
    _run('session_failover')


def test_watch_kinds_cross_the_frame_fanout():
    _run('watch_kinds')


def test_watch_fanout_uses_one_server_watch():
    """Only the owner rank arms the ZooKeeper watch (R1: one server watch
    per path, the node fans the events out): checked in the fake server's
    log of the sessions that armed a data watch on the path."""
    zk = _run('watch_fanout')
    sids = zk.db.watch_log.get('/fan', set())
    assert len(sids) == 1, sids


@pytest.mark.parametrize('scenario', ['metrics', 'watch_fanout',
                                      'session_failover'])
def test_group_eight_ranks(scenario):
    """The node layer at world 8 (gloo): R4 metrics all-reduce, R1 watch
    fan-out from one owner rank to seven, R3 session credential broadcast
    and adoption."""
    _run(scenario, world=8)
