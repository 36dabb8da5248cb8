"""The native completion path of the interactive API (CPU): the native
loop's reply router (``Transport.route``, csrc/host/zk_loop.cpp) settles
replies to outstanding requests without Python framing/decoding, and
``Transport.request`` encodes requests straight into the write buffer.

Parity targets: the reply routing of ``lib/connection-fsm.js:213-229`` and
``:384-408`` (every reply settles its request, in stream order with the
notifications around it), ``lib/zk-session.js:227-238`` (every packet
advances lastZxid and the expiry timer)."""

import threading

import pytest

from zkmi.errors import ZKError
from zkmi.server import FakeZKServer
from zkmi.runtime import nloop

from zkhelpers import Box, client, wait_for

pytestmark = pytest.mark.skipif(not nloop.available(),
                                reason='native loop not built')


@pytest.fixture
def zk():
    s = FakeZKServer(tick_ms=250)
    yield s
    s.shutdown()


@pytest.fixture
def zkc(zk):
    c = client(zk.servers())
    c.wait_connected(10)
    yield c
    c.close_sync(10)


def _conn(c):
    return c.loop.run(lambda: c.getSession().getConnection())


def _routed(c):
    conn = _conn(c)
    return c.loop.run(lambda: conn.socket.transport.route_state()[2])


def test_router_settles_replies(zkc):
    conn = _conn(zkc)
    assert conn.routing
    before = _routed(zkc)
    assert zkc.call_sync('create', '/r', b'abc', {}) == '/r'
    data, stat = zkc.call_sync('get', '/r')
    assert data == b'abc' and stat.dataLength == 3
    assert _routed(zkc) >= before + 2
    # nothing left behind in the connection's tables
    assert zkc.loop.run(lambda: (len(conn.reqs), len(conn.xid_map))) == (0, 0)


def test_error_replies_and_pipelined_mix(zkc):
    zkc.call_sync('create', '/m', b'', {})
    for i in range(0, 200, 2):
        zkc.call_sync('create', '/m/n%d' % i, b'%d' % i, {})
    n = 200
    got = {}
    done = threading.Event()

    def issue():
        for i in range(n):
            def cb(err, data=None, stat=None, i=i):
                got[i] = (err, data)
                if len(got) == n:
                    done.set()
            zkc.get('/m/n%d' % i, cb)
    zkc.loop.call_soon(issue)
    assert done.wait(20)
    for i in range(n):
        err, data = got[i]
        if i % 2 == 0:
            assert err is None and data == b'%d' % i
        else:
            assert isinstance(err, ZKError) and err.code == 'NO_NODE'


def test_last_zxid_and_liveness_follow_routed_replies(zkc):
    sess = zkc.loop.run(zkc.getSession)
    z0 = zkc.loop.run(lambda: sess.last_zxid)
    zkc.call_sync('create', '/z', b'', {})
    zkc.call_sync('set', '/z', b'x', -1)
    st = zkc.call_sync('stat', '/z')
    z1 = zkc.loop.run(lambda: sess.last_zxid)
    assert z1 >= st.mzxid > z0
    assert zkc.loop.run(lambda: sess.credentials()['lastZxid']) == z1

    # the routed replies alone keep the session alive: forget the Python
    # side's last packet and ask again
    def probe():
        sess.last_pkt = None
        return sess.isAlive()
    assert zkc.loop.run(probe)


def test_notification_order_around_routed_replies(zk, zkc):
    """A watch event and the replies around it reach the client in stream
    order: the notification goes through Python's path, the replies through
    the router, and neither overtakes the other."""
    zkc.call_sync('create', '/w', b'0', {})
    order = []
    fired = Box()

    w = zkc.watcher('/w')
    w.on('dataChanged', lambda d, s: (order.append(('data', d)), fired(d)))
    assert wait_for(lambda: ('data', b'0') in order, 10)
    done = threading.Event()

    def go():
        zkc.set('/w', b'1', -1, lambda err, *a: order.append(('set', err)))
        zkc.get('/w', lambda err, d=None, s=None: (order.append(('get', d)),
                                                     done.set()))
    conn = _conn(zkc)
    framed0 = zkc.loop.run(lambda: conn.decoder.frames_in)
    zkc.loop.call_soon(go)
    assert done.wait(10)
    assert wait_for(lambda: ('data', b'1') in order, 10)
    i_set = order.index(('set', None))
    i_get = order.index(('get', b'1'))
    assert i_set < i_get
    # the notification and the replies (the watcher's re-arm included,
    # four frames at least) were framed and decoded natively: Python's
    # framer saw at most a ping reply (xid -2) that landed in between
    assert zkc.loop.run(lambda: conn.decoder.frames_in) - framed0 <= 1


def test_large_reply_split_across_reads(zkc):
    blob = bytes(range(256)) * 4096           # 1 MiB: many recv() calls
    zkc.call_sync('create', '/big', blob, {})
    before = _routed(zkc)
    data, stat = zkc.call_sync('get', '/big')
    assert data == blob and stat.dataLength == len(blob)
    assert _routed(zkc) == before + 1


def test_router_off_while_paused_falls_back(zkc):
    """pause_reading holds the stream: the router steps aside, requests go
    the Python way and settle when reading resumes."""
    conn = _conn(zkc)
    sock = conn.socket
    res = Box()

    def go():
        sock.pause_reading()
        zkc.create('/p', b'x', {}, lambda err, *a: res(err, *a))
    zkc.loop.run(go)
    assert not res.ev.wait(0.5)
    zkc.loop.run(sock.resume_reading)
    err, path = res.wait(10)
    assert err is None and path == '/p'
    assert zkc.call_sync('get', '/p')[0] == b'x'


def test_close_with_routed_requests_in_flight(zk):
    c = client(zk.servers())
    c.wait_connected(10)
    n = 100
    got = []
    done = threading.Event()

    def go():
        for i in range(n):
            c.stat('/nope%d' % i, lambda err, *a: (got.append(err),
                                                       len(got) == n and
                                                       done.set()))
        c.close()
    c.loop.call_soon(go)
    assert done.wait(20)
    # every request settles exactly once: a reply (NO_NODE) or a
    # connection error, never both and never neither
    assert len(got) == n
    assert all(e is not None for e in got)


def test_direct_requests_from_many_threads(zkc):
    """call_sync from several threads at once sends from each caller's
    thread (request_direct) while the loop thread issues its own requests:
    every xid stays unique and every reply reaches its caller."""
    conn = _conn(zkc)
    zkc.call_sync('create', '/t', b'', {})
    for k in range(8):
        zkc.call_sync('create', '/t/%d' % k, b'v%d' % k, {})
    errors = []
    loop_done = threading.Event()
    got = []

    def loop_side():
        def cb(err, data=None, stat=None):
            got.append((err, data))
            if len(got) == 400:
                loop_done.set()
        for i in range(400):
            zkc.get('/t/%d' % (i % 8), cb)

    def worker(k):
        try:
            for i in range(200):
                data, stat = zkc.call_sync('get', '/t/%d' % k)
                assert data == b'v%d' % k
            try:
                zkc.call_sync('get', '/t/missing%d' % k)
                errors.append('no error for a missing node')
            except ZKError as e:
                assert e.code == 'NO_NODE'
        except Exception as e:          # reported below
            errors.append(repr(e))
    ths = [threading.Thread(target=worker, args=(k,)) for k in range(8)]
    zkc.loop.call_soon(loop_side)
    for t in ths:
        t.start()
    for t in ths:
        t.join(60)
    assert loop_done.wait(20)
    assert not errors, errors
    assert all(e is None and d is not None and d.startswith(b'v')
               for e, d in got)
    assert zkc.loop.run(lambda: (len(conn.reqs), len(conn.xid_map))) == (0, 0)


def test_direct_falls_back_when_router_off(zkc):
    """With the router off (a paused socket) a blocking call hops to the
    loop thread as before and still completes once reading resumes."""
    conn = _conn(zkc)
    sock = conn.socket
    zkc.loop.run(sock.pause_reading)
    res = Box()

    def call():
        try:
            res(zkc.call_sync('create', '/fb', b'x', {}, timeout=10))
        except Exception as e:          # reported by the assert below
            res(e)
    th = threading.Thread(target=call)
    th.start()
    assert not res.ev.wait(0.3)
    zkc.loop.run(sock.resume_reading)
    th.join(10)
    assert res.wait(10)[0] == '/fb'


@pytest.fixture
def pzkc(zk):
    """A client on a loop of its own: holding its loop thread (the tests
    below do, to order events) leaves the fake server's loop running."""
    from zkmi.runtime import loop as L
    lp = L.new_loop('completion-private')
    c = client(zk.servers(), loop=lp)
    c.wait_connected(10)
    yield c
    try:
        c.close_sync(10)
    finally:
        lp.stop()


def test_failed_direct_send_settles_once(pzkc):
    """A direct send that fails (the socket is already shut for writing)
    settles its request exactly once: the transport unregisters it, so the
    connection's later failure does not fail it a second time (ADVICE r3:
    a second callback released call_sync's lock twice and aborted the
    connection's cleanup)."""
    import os
    import socket
    conn = _conn(pzkc)
    fd = pzkc.loop.run(lambda: conn.socket.transport.get_extra_info('fd'))
    gate = threading.Event()
    pzkc.loop.call_soon(gate.wait, 10)          # hold the loop thread
    s = socket.socket(fileno=os.dup(fd))    # closing the dup leaves fd
    try:
        s.shutdown(socket.SHUT_WR)
    finally:
        s.close()
    calls = []
    pzkc.get('/nope', lambda err, *a: calls.append(err))   # sent directly
    gate.set()
    assert wait_for(lambda: len(calls) >= 1, 10)
    import time
    time.sleep(0.5)             # the connection's failure has run by now
    assert len(calls) == 1, calls
    assert calls[0] is not None and calls[0].code == 'CONNECTION_LOSS'


def test_direct_send_keeps_fifo_behind_queued_submissions(pzkc):
    """A request sent from a thread must not overtake that thread's earlier
    submissions still queued for the loop: a bulk_set queued
    while the loop is busy, then a blocking get from the same thread, must
    read the value the bulk_set wrote."""
    pzkc.call_sync('create', '/fifo', b'old', {})
    # a first bulk batch pays the bulk path's imports and setup (seconds
    # under the sanitizers) before the loop is held
    pzkc.call_sync('bulk_set', ['/fifo'], b'old')
    gate = threading.Event()
    pzkc.loop.call_soon(gate.wait, 10)          # the loop is busy
    res = Box()
    pzkc.bulk_set(['/fifo'], b'new', lambda err, r=None: res(err))
    assert pzkc._hops >= 1
    got = Box()

    def reader():
        got(pzkc.call_sync('get', '/fifo')[0])
    th = threading.Thread(target=reader)
    th.start()
    import time
    time.sleep(0.2)
    gate.set()
    th.join(10)
    assert res.wait(10)[0] is None
    assert got.wait(10)[0] == b'new'
