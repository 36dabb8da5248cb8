"""Bulk (pipelined, GPU-coded) requests on a live connection
(zkmi/models/bulk.py).  The CPU tests drive the host-codec path
(``device=False``); the GPU test drives K10 encode + K1/K2-K8 decode over the
same TCP connection and checks reply-for-reply parity with the interactive
API."""

import pytest

from zkmi.server import FakeZKServer

from zkhelpers import Box, client, wait_for


@pytest.fixture
def zk():
    s = FakeZKServer(tick_ms=250)
    yield s
    s.shutdown()


def _populate(c, n):
    c.call_sync('create', '/bulk', b'', {})
    for i in range(n):
        c.call_sync('create', '/bulk/n%04d' % i, b'v%d' % i, {})


def _run(c, fn, *a):
    b = Box()
    getattr(c, fn)(*a, b)
    return b.wait(20)


def _check_mixed(c):
    _populate(c, 20)
    paths = ['/bulk/n%04d' % i for i in range(20)] + ['/bulk/missing']
    err, res = _run(c, 'bulk_get', paths)
    assert err is None
    pk = res.packets()
    assert len(pk) == 21
    for i in range(20):
        assert pk[i]['err'] == 'OK'
        assert pk[i]['data'] == b'v%d' % i
        # identical to the interactive get
        d2, st2 = c.call_sync('get', paths[i])
        assert d2 == pk[i]['data']
        assert st2.as_tuple() == pk[i]['stat'].as_tuple()
    assert pk[20]['err'] == 'NO_NODE'
    assert res.errors()[20] == 'NO_NODE'
    assert res.ok_count() == 20
    # writes: create / set with CAS / delete / exists / list
    reqs = [
        {'opcode': 'CREATE', 'path': '/bulk/new', 'data': b'x'},
        {'opcode': 'SET_DATA', 'path': '/bulk/n0000', 'data': b'y',
         'version': 0},
        {'opcode': 'SET_DATA', 'path': '/bulk/n0001', 'data': b'z',
         'version': 5},
        {'opcode': 'DELETE', 'path': '/bulk/n0002', 'version': -1},
        {'opcode': 'EXISTS', 'path': '/bulk/n0002'},
        {'opcode': 'GET_CHILDREN2', 'path': '/bulk'},
        {'opcode': 'CREATE', 'path': '/bulk/seq-', 'data': b'',
         'flags': ['SEQUENTIAL']},
    ]
    err, res = _run(c, 'bulk', reqs)
    assert err is None
    pk = res.packets()
    assert [p['err'] for p in pk] == ['OK', 'OK', 'BAD_VERSION', 'OK',
                                      'NO_NODE', 'OK', 'OK']
    assert pk[0]['path'] == '/bulk/new'
    assert pk[1]['stat'].version == 1
    assert 'n0002' not in pk[5]['children'] and 'new' in pk[5]['children']
    assert pk[6]['path'].startswith('/bulk/seq-') and len(pk[6]['path']) == 20
    assert c.call_sync('get', '/bulk/n0000')[0] == b'y'


def test_bulk_host_codec(zk):
    c = client(zk.servers(), device=False)
    c.wait_connected(10)
    try:
        _check_mixed(c)
    finally:
        c.close_sync(10)


def test_bulk_interleaves_with_interactive_requests(zk):
    """Bulk replies are routed by xid range; ordinary requests and pings
    sent meanwhile keep their own replies."""
    c = client(zk.servers(), device=False)
    c.wait_connected(10)
    try:
        _populate(c, 50)
        boxes = []
        bb = Box()
        c.bulk_get(['/bulk/n%04d' % i for i in range(50)], bb)
        for i in range(10):
            b = Box()
            c.get('/bulk/n%04d' % i, b)
            boxes.append(b)
        pinged = Box()
        c.ping(pinged)
        err, res = bb.wait(20)
        assert err is None and res.ok_count() == 50
        for i, b in enumerate(boxes):
            e, data, st = b.wait(10)
            assert e is None and data == b'v%d' % i
        assert pinged.wait(10) == (None,)
    finally:
        c.close_sync(10)


def test_bulk_not_connected_and_bad_args(zk):
    c = client(zk.servers(), device=False)
    with pytest.raises(ValueError):
        c.bulk([{'opcode': 'PING'}], lambda *a: None)
    with pytest.raises(ValueError):
        c.bulk([{'opcode': 'GET_DATA', 'path': '/a', 'watch': True}],
               lambda *a: None)
    with pytest.raises(TypeError):
        c.bulk_get('/a', lambda *a: None)
    import torch
    with pytest.raises(ValueError):       # device paths on the host codec
        c.bulk_get((torch.zeros(2, dtype=torch.uint8),
                    torch.zeros(1, dtype=torch.int64),
                    torch.ones(1, dtype=torch.int32)), lambda *a: None)
    c.wait_connected(10)
    c.close_sync(10)
    b = Box()
    c.bulk_get(['/a'], b)
    err = b.wait(10)[0]
    assert err is not None and err.code == 'CONNECTION_LOSS'


def test_bulk_fails_on_connection_loss(zk):
    c = client(zk.servers(), device=False)
    c.wait_connected(10)
    try:
        _populate(c, 5)
        zk.set_mode('hang')
        # the server stops reading first, so the batch is still in flight
        # when the connection drops (else it could be answered in time)
        zk.pause_reads()
        b = Box()
        c.bulk_get(['/bulk/n%04d' % i for i in range(5)], b)
        zk.drop_connections()
        err = b.wait(20)[0]
        assert err is not None
    finally:
        zk.resume_reads()
        zk.set_mode('normal')
        wait_for(lambda: c.isConnected(), 10)
        c.close_sync(10)


@pytest.mark.gpu
def test_bulk_gpu_codec(zk, gpu):
    from zkmi.ops import _lib
    assert _lib.available(), 'HIP library must be built on a GPU box'
    c = client(zk.servers(), device=gpu)
    c.wait_connected(10)
    try:
        _check_mixed(c)
        # a larger pipelined batch, decoded on the GPU
        err, res = _run(c, 'bulk_get', ['/bulk/n%04d' % (i % 20)
                                         for i in range(2000)])
        assert err is None and res.replies is not None
        assert res.ok_count() == 2000 - 2000 // 20     # n0002 was deleted
    finally:
        c.close_sync(10)


def test_bulk_empty_batch(zk):
    """An empty bulk completes with an empty result and reserves no xids
    (it used to fail on a missing attribute)."""
    c = client(zk.servers())
    c.wait_connected(10)
    err, res = _run(c, 'bulk', [])
    assert err is None
    assert res.n == 0 and res.packets() == []
    # the connection keeps working afterwards
    c.call_sync('create', '/after', b'ok', {})
    assert c.call_sync('get', '/after')[0] == b'ok'
    c.close_sync(10)


@pytest.mark.gpu
def test_bulk_gpu_capture_native_server(gpu):
    """The GPU bulk path on the live connection against the native server:
    K10 into a pinned TX buffer, replies captured by the native loop into a
    pinned RX buffer (no reply frame routed through Python), K1 + K2-K8 on
    the GPU; device-tensor paths; a second batch with replies bigger than
    the RX reservation falls back to per-frame collection and stays exact."""
    import torch
    from zkmi.server import fast
    from zkmi.runtime import nloop
    if not (fast.available() and nloop.available()):
        pytest.skip('native server / loop not built')
    srv = fast.FastZKServer(preload=20000, data_bytes=100)
    try:
        c = client(srv.servers(), device=gpu)
        c.wait_connected(10)
        n = 20000
        paths = ['/bench/d%06d/n%09d' % (i // 1000, i) for i in range(n)]
        blob = ''.join(paths).encode()
        arena = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(gpu)
        idx = torch.randperm(n, device=gpu)
        off = idx * 25
        ln = torch.full((n,), 25, dtype=torch.int32, device=gpu)
        err, res = _run(c, 'bulk_get', (arena, off, ln))
        assert err is None and res.replies is not None
        assert res.ok_count() == n
        conn = c.loop.run(lambda: c.getSession().getConnection())
        assert conn.bulk_frames_py == 0
        # the replies are the requested nodes: czxid order follows the
        # preload order (node i was created after i + dirs + 3 nodes)
        r = res.replies
        czx = r.stat64[0, :n]
        assert bool((czx - czx.min() == idx - idx.min()).all())
        assert bool((r.pay_len[:n] == 100).all())
        # big values: the RX reservation overflows, per-frame fallback
        c.call_sync('create', '/big', b'x' * 5000, {})
        err, res = _run(c, 'bulk_get', ['/big'] * 300)
        assert err is None and res.ok_count() == 300
        assert conn.bulk_frames_py > 0
        pk = res.packets()
        assert pk[7]['data'] == b'x' * 5000
        c.close_sync(10)
    finally:
        srv.shutdown()
