"""In-batch ordering of the GPU server (csrc/kernels/tree.hip tree_order_*,
zk_tree_serve_ordered) against the fake server applying the same requests
one by one.

ZooKeeper applies one session's requests in order (the reference pipelines
them over one connection and matches replies by xid,
lib/connection-fsm.js:384-408), so a batch holding create -> set -> get ->
delete -> create of one path must answer exactly as the sequential server
does.  The GPU server groups the batch by path and serves it in passes of
equal same-path rank; reads and sets that a later write of the batch would
overwrite reply from a snapshot.
"""

import random

import numpy as np
import pytest
import torch

from zkmi import jute
from zkmi.server.fakezk import ZKDatabase, ZKServerError  # noqa: F401


class _Loop(object):
    """Just enough of an event loop for ZKDatabase (no expiry ticks run)."""

    class _H(object):
        def cancel(self):
            pass

    def call_later(self, ms, fn):
        return self._H()

    def time_ms(self):
        return 0


def _dev_bytes(b, dev):
    a = np.frombuffer(bytes(b) if b else b'\0', np.uint8).copy()
    return torch.from_numpy(a).to(dev)


def _serve(srv, pk, dev, **kw):
    s = b''.join(jute.frame(jute.encode_request(p)) for p in pk)
    out, total, _, _ = srv.serve(_dev_bytes(s, dev), len(s), **kw)
    rx = bytes(out[:total.item()].cpu().numpy().tobytes())
    frames, _, bad = jute.scan_frames(rx)
    assert bad == -1 and len(frames) == len(pk)
    xmap = {p['xid']: p['opcode'] for p in pk}
    return [jute.decode_response(rx[o:o + ln], xmap) for o, ln in frames]


def _key(rep):
    """What must agree between the GPU and the sequential server: the error,
    and for a success the data / path / version / data length (creation
    zxids, times and the parent's counts differ between the two trees)."""
    k = [rep['xid'], rep['err']]
    if rep['err'] == 'OK':
        if 'data' in rep:
            k.append(bytes(rep['data'] or b''))
        if rep.get('path') is not None:
            k.append(rep['path'])
        st = rep.get('stat')
        if st is not None:
            k += [st.version, st.dataLength]
    return tuple(k)


def _mirror(tree, leaves):
    """A fake server database holding /bench/d000000 and the given existing
    leaves with the GPU tree's data and version."""
    db = ZKDatabase(_Loop())
    db.create('/bench', b'', [db._world()], [], None)
    db.create('/bench/d000000', b'', [db._world()], [], None)
    for p in leaves:
        data, st = tree.node_slot_host(tree.find_host(p))
        db.create(p, data, [db._world()], [], None)
        assert st.version == 0
    return db


def _sequential(db, pk):
    out = []
    for p in pk:
        rep = db.handle(dict(p), None)
        out.append(_key(rep))        # keys copy the live Stat's fields now
    return out


def _random_batch(rng, paths, n, xid0=0):
    pk = []
    for k in range(n):
        path = rng.choice(paths)
        op = rng.choice(['CREATE', 'SET_DATA', 'GET_DATA', 'EXISTS',
                         'DELETE', 'GET_DATA'])
        x = xid0 + k
        if op == 'CREATE':
            pk.append({'xid': x, 'opcode': op, 'path': path,
                       'data': bytes(rng.getrandbits(8)
                                     for _ in range(rng.randint(0, 100))),
                       'acl': jute.DEFAULT_ACL, 'flags': []})
        elif op == 'SET_DATA':
            pk.append({'xid': x, 'opcode': op, 'path': path,
                       'data': bytes(rng.getrandbits(8)
                                     for _ in range(rng.randint(0, 120))),
                       'version': rng.choice([-1, -1, 0, 1, 2])})
        elif op == 'DELETE':
            pk.append({'xid': x, 'opcode': op, 'path': path,
                       'version': rng.choice([-1, -1, 0, 1])})
        else:
            pk.append({'xid': x, 'opcode': op, 'path': path,
                       'watch': False})
    return pk


@pytest.mark.gpu
def test_ordered_batch_matches_sequential_server():
    from zkmi.bench.synthetic import GpuTree, GpuServer
    dev = torch.device('cuda', 0)
    tree = GpuTree(1000, 16, fanout=100, device=dev, spare=0.5,
                   scratch=1 << 20)
    srv = GpuServer(tree, 1024, 1 << 20)
    leaves = ['/bench/d000000/n%09d' % i for i in (3, 4)]
    paths = leaves + ['/bench/d000000/ord%d' % i for i in range(6)]
    db = _mirror(tree, leaves)
    rng = random.Random(7)
    xid = 0
    for rnd in range(4):
        pk = _random_batch(rng, paths, 240, xid)
        xid += len(pk)
        want = _sequential(db, pk)
        got = [_key(r) for r in _serve(srv, pk, dev, ordered=True,
                                       passes=80)]
        maxrank, used = srv.order_stats()
        assert maxrank < 80
        assert used > 0                      # snapshots were taken
        assert got == want, 'round %d: first mismatch at %d' % (
            rnd, next(i for i, (a, b) in enumerate(zip(got, want))
                      if a != b))
        # the tree the batch left matches too (plain, unordered reads)
        probe = [{'xid': 100000 + i, 'opcode': 'GET_DATA', 'path': p,
                  'watch': False} for i, p in enumerate(paths)]
        assert [_key(r) for r in _serve(srv, probe, dev)] == \
            _sequential(db, probe)


@pytest.mark.gpu
def test_ordered_create_set_delete_create_chain():
    """The canonical chain on one path, with reads between every step."""
    from zkmi.bench.synthetic import GpuTree, GpuServer
    dev = torch.device('cuda', 0)
    tree = GpuTree(1000, 16, fanout=100, device=dev, scratch=1 << 16)
    srv = GpuServer(tree, 64, 1 << 16)
    p = '/bench/d000000/chain'
    A = jute.DEFAULT_ACL
    pk = [
        {'xid': 0, 'opcode': 'GET_DATA', 'path': p, 'watch': False},
        {'xid': 1, 'opcode': 'CREATE', 'path': p, 'data': b'one', 'acl': A,
         'flags': []},
        {'xid': 2, 'opcode': 'GET_DATA', 'path': p, 'watch': False},
        {'xid': 3, 'opcode': 'SET_DATA', 'path': p, 'data': b'two',
         'version': 0},
        {'xid': 4, 'opcode': 'SET_DATA', 'path': p, 'data': b'three',
         'version': 0},                                   # BAD_VERSION now
        {'xid': 5, 'opcode': 'EXISTS', 'path': p, 'watch': False},
        {'xid': 6, 'opcode': 'GET_DATA', 'path': p, 'watch': False},
        {'xid': 7, 'opcode': 'DELETE', 'path': p, 'version': 1},
        {'xid': 8, 'opcode': 'GET_DATA', 'path': p, 'watch': False},
        {'xid': 9, 'opcode': 'CREATE', 'path': p, 'data': b'again',
         'acl': A, 'flags': []},
        {'xid': 10, 'opcode': 'GET_DATA', 'path': p, 'watch': False},
    ]
    reps = _serve(srv, pk, dev, ordered=True, passes=16)
    errs = [r['err'] for r in reps]
    assert errs == ['NO_NODE', 'OK', 'OK', 'OK', 'BAD_VERSION', 'OK', 'OK',
                    'OK', 'NO_NODE', 'OK', 'OK']
    assert reps[2]['data'] == b'one' and reps[2]['stat'].version == 0
    assert reps[3]['stat'].version == 1
    assert reps[5]['stat'].version == 1 and reps[5]['stat'].dataLength == 3
    assert reps[6]['data'] == b'two'
    assert reps[9]['path'] == p
    assert reps[10]['data'] == b'again' and reps[10]['stat'].version == 0
    # zxids: writes keep their batch position (xid order)
    zx = [r['zxid'] for r in reps]
    assert zx[1] < zx[3] < zx[7] < zx[9]


@pytest.mark.gpu
def test_ordered_excess_rank_is_refused():
    """More same-path requests than passes: the excess is answered
    SYSTEMERROR and order_stats reports the rank; nothing is misordered."""
    from zkmi.bench.synthetic import GpuTree, GpuServer
    dev = torch.device('cuda', 0)
    tree = GpuTree(1000, 16, fanout=100, device=dev, scratch=1 << 16)
    srv = GpuServer(tree, 64, 1 << 16)
    p = '/bench/d000000/n000000009'
    pk = [{'xid': k, 'opcode': 'SET_DATA', 'path': p,
           'data': b'v%d' % k, 'version': k} for k in range(10)]
    reps = _serve(srv, pk, dev, ordered=True, passes=4)
    assert [r['err'] for r in reps] == ['OK'] * 4 + ['SYSTEM_ERROR'] * 6
    assert [r['stat'].version for r in reps[:4]] == [1, 2, 3, 4]
    assert srv.order_stats()[0] == 9
    data, st = tree.node_slot_host(tree.find_host(p))
    assert data == b'v3' and st.version == 4


@pytest.mark.gpu
def test_ordered_read_only_and_unrelated_paths_single_rank():
    """Paths only read, and SEQUENTIAL creates, are never ranked: a GET
    batch is served in one effective pass and all succeed."""
    from zkmi.bench.synthetic import GpuTree, GpuServer
    dev = torch.device('cuda', 0)
    tree = GpuTree(1000, 16, fanout=100, device=dev)
    srv = GpuServer(tree, 256, 1 << 17)
    p = '/bench/d000000/n000000001'
    pk = [{'xid': k, 'opcode': 'GET_DATA', 'path': p, 'watch': False}
          for k in range(50)]
    pk += [{'xid': 50 + k, 'opcode': 'CREATE', 'path': '/bench/d000001/s-',
            'data': b'', 'acl': jute.DEFAULT_ACL, 'flags': ['SEQUENTIAL']}
           for k in range(50)]
    reps = _serve(srv, pk, dev, ordered=True, passes=2)
    assert all(r['err'] == 'OK' for r in reps)
    assert srv.order_stats() == (0, 0)
    assert len({r['path'] for r in reps[50:]}) == 50


@pytest.mark.gpu
def test_chain_pipeline_steps():
    """bench --workload chain: every path's create -> set -> get -> delete
    in one batch, checked on the device; the node count stays steady."""
    from zkmi.bench.synthetic import GpuTree, ChainPipeline
    from zkmi.ops import _lib
    dev = torch.device('cuda', 0)
    tree = GpuTree(20000, 37, fanout=100, device=dev, spare=1.0,
                   scratch=1 << 22)
    pipe = ChainPipeline(tree, 4 * 2048, data_bytes=100, ndirs=64)
    hw = None
    for s in range(5):
        ok = pipe.step()
        assert int(ok.item()) == pipe.n, pipe.diagnose()
        if s == 1:
            hw = int(tree.counters[_lib.TC_NODES].item())
    assert int(tree.counters[_lib.TC_NODES].item()) == hw
    assert pipe.drv.server.order_stats()[0] == 3


def _key_tree(rep):
    """_key plus the parent-visible Stat fields (children count and
    cversion): what a batch mixing a node's and its children's writes must
    get right."""
    k = list(_key(rep))
    st = rep.get('stat') if rep['err'] == 'OK' else None
    if st is not None:
        k += [st.numChildren, st.cversion]
    return tuple(k)


@pytest.mark.gpu
def test_ordered_parent_child_batch_matches_sequential_server():
    """createWithEmptyParents in ONE batch (lib/client.js:412-481,
    test/basic.test.js:317-611): depth-3 creates, the parents' Stat read
    between the children's writes, a child created before its parent, a
    parent delete refused while it has a child — every reply as the
    sequential server gives it (a create and its parent's create conflict;
    a parent's Stat read conflicts with its children's writes)."""
    from zkmi.bench.synthetic import GpuTree, GpuServer
    dev = torch.device('cuda', 0)
    tree = GpuTree(1000, 16, fanout=100, device=dev, spare=0.5,
                   scratch=1 << 20)
    srv = GpuServer(tree, 256, 1 << 18)
    db = _mirror(tree, [])
    A = jute.DEFAULT_ACL
    d = '/bench/d000000'
    x, y, z = d + '/x', d + '/x/y', d + '/x/y/z'

    def c(p, data=b'', flags=()):
        return {'opcode': 'CREATE', 'path': p, 'data': data, 'acl': A,
                'flags': list(flags)}

    def ex(p):
        return {'opcode': 'EXISTS', 'path': p, 'watch': False}

    def get(p):
        return {'opcode': 'GET_DATA', 'path': p, 'watch': False}

    def rm(p, v=-1):
        return {'opcode': 'DELETE', 'path': p, 'version': v}

    batches = [
        # child before its parent: NO_NODE, then the chain in order
        [c(y, b'early'), ex(x), c(x, b'null'), c(y, b'null'), c(z, b'leaf'),
         ex(x), get(y), ex(d + '/x/y/z'), c(z, b'again'), rm(y),
         c(x + '/s-', b'', ['SEQUENTIAL']), ex(x)],
        # tear down bottom-up with the parents' Stat read in between
        [ex(y), rm(z), ex(y), rm(y), ex(x), get(x), rm(x + '/s-0000000001'),
         rm(x), ex(x), get(y)],
        # the same path rebuilt and re-deleted in one batch
        [c(x, b'1'), c(y, b'2'), rm(y), ex(x), rm(x), c(x, b'3'), ex(x),
         get(x)],
    ]
    xid = 0
    for bno, pk in enumerate(batches):
        for p in pk:
            p['xid'] = xid
            xid += 1
        want = [_key_tree(db.handle(dict(p), None)) for p in pk]
        got = [_key_tree(r) for r in _serve(srv, pk, dev, ordered=True,
                                            passes=16)]
        assert srv.order_stats()[0] < 16
        assert got == want, 'batch %d: first mismatch at %d: %r vs %r' % (
            bno, *next((i, a, b) for i, (a, b) in enumerate(zip(got, want))
                       if a != b))


@pytest.mark.gpu
def test_nest_pipeline_steps():
    """bench --workload nest: depth-3 creates, the parent's EXISTS and the
    bottom-up deletes of every tree in one batch, checked on the device."""
    from zkmi.bench.synthetic import GpuTree, NestPipeline
    from zkmi.ops import _lib
    dev = torch.device('cuda', 0)
    tree = GpuTree(20000, 37, fanout=100, device=dev, spare=1.0,
                   scratch=1 << 22)
    pipe = NestPipeline(tree, 7 * 1024, ndirs=64)
    hw = top = None
    for s in range(12):
        ok = pipe.step()
        assert int(ok.item()) == pipe.n, pipe.diagnose()
        if s == 1:
            hw = int(tree.counters[_lib.TC_NODES].item())
            top = int(tree.counters[_lib.TC_PATH_TOP].item())
    assert int(tree.counters[_lib.TC_NODES].item()) == hw
    # recycled nodes reuse their path storage across the three path
    # lengths: the path arena does not grow step after step
    assert int(tree.counters[_lib.TC_PATH_TOP].item()) == top
    assert pipe.drv.server.order_stats()[0] == 5
