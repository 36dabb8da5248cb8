"""The native epoll loop (csrc/host/zk_loop.cpp via zkmi/runtime/nloop.py):
scheduling, timers, exception capture, TCP transports (connect, refuse,
half-close, abort, pause, bulk writes) and the client/fake-server stack on
both loop implementations.  CPU only."""

import os
import threading
import time

import pytest

from zkmi.runtime import nloop
from zkmi.runtime.loop import Loop, wait_for
from zkmi.server import FakeZKServer

from zkhelpers import client

pytestmark = pytest.mark.skipif(not nloop.available(),
                                reason='native loop not built')


@pytest.fixture
def nl():
    lp = nloop.NativeLoop('test-native')
    yield lp
    lp.stop()


def test_call_soon_order_and_threads(nl):
    seen = []
    done = threading.Event()
    nl.call_soon(seen.append, 1)
    nl.call_soon(seen.append, 2)
    h = nl.call_soon(seen.append, 'cancelled')
    h.cancel()
    nl.call_soon(lambda: (seen.append(nl.in_loop()), done.set()))
    assert done.wait(5)
    assert seen == [1, 2, True]
    assert not nl.in_loop()
    assert nl.run(lambda: 41 + 1) == 42
    with pytest.raises(KeyError):
        nl.run(lambda: {}['x'])


def test_waiter_set_on_loop_and_off_loop(nl):
    """Waiter (Client.call_sync's completion flag): set on the loop thread
    it flips once the loop lets go of the GIL for its next wait; set from
    another thread it flips at once; wait() times out unset."""
    w = nl.waiter()
    assert not w.is_set
    t0 = time.perf_counter()
    assert not w.wait(0.0, 0.02)
    assert time.perf_counter() - t0 >= 0.015
    seen = []

    def on_loop():
        w.set()
        seen.append(w.is_set)          # deferred: not yet, same turn
    nl.call_soon(on_loop)
    assert w.wait(0.0, 5.0) and w.is_set
    assert seen == [False]
    w2 = nl.waiter()
    threading.Timer(0.01, w2.set).start()
    assert w2.wait(0.001, 5.0)
    # a spin-only wait that the loop settles
    w3 = nl.waiter()
    nl.call_soon(w3.set)
    assert w3.wait(1.0, 5.0)


def test_waiter_flipped_when_the_loop_stops():
    lp = nloop.NativeLoop('t-stop')
    w = lp.waiter()

    def last():
        w.set()
        lp.stop()
    lp.call_soon(last)
    assert w.wait(0.0, 5.0)


def test_timers_fire_in_deadline_order(nl):
    seen = []
    t0 = nl.time_ms()
    nl.call_later(60, seen.append, 'c')
    nl.call_later(20, seen.append, 'a')
    nl.call_later(40, seen.append, 'b')
    x = nl.call_later(30, seen.append, 'never')
    x.cancel()
    assert x.cancelled
    assert wait_for(lambda: len(seen) == 3, 5)
    assert seen == ['a', 'b', 'c']
    assert nl.time_ms() - t0 >= 60
    # a timer armed from the loop thread, chained
    box = []

    def chain(k):
        box.append(k)
        if k < 5:
            nl.call_later(1, chain, k + 1)
    nl.call_soon(chain, 0)
    assert wait_for(lambda: len(box) == 6, 5)
    assert nl.stats()['timers'] == 0


def test_callback_exceptions_are_recorded(nl):
    nl.call_soon(lambda: 1 / 0)
    nl.call_soon(lambda: None)
    assert wait_for(lambda: len(nl.errors) == 1, 5)
    assert isinstance(nl.errors[0], ZeroDivisionError)
    assert nl.run(lambda: 'alive') == 'alive'


class Proto(object):
    def __init__(self):
        self.events = []
        self.data = bytearray()
        self.tr = None

    def connection_made(self, tr):
        self.tr = tr
        self.events.append('made')

    def data_received(self, b):
        self.data += b

    def eof_received(self):
        self.events.append('eof')
        return True

    def connection_lost(self, exc):
        self.events.append(('lost', exc))


def _pair(lp):
    srv_protos = []

    def factory():
        p = Proto()
        srv_protos.append(p)
        return p
    srv = lp.start_server(factory, '127.0.0.1', 0)
    cp = Proto()
    fails = []
    lp.run(lambda: lp.open_connection(cp, '127.0.0.1', srv.port,
                                      fails.append))
    assert wait_for(lambda: cp.tr is not None and srv_protos, 5), fails
    assert wait_for(lambda: srv_protos[0].tr is not None, 5)
    return srv, cp, srv_protos[0]


@pytest.mark.parametrize('kind', ['native', 'asyncio'])
def test_tcp_roundtrip_halfclose_and_bulk(kind):
    lp = nloop.NativeLoop('t') if kind == 'native' else Loop('t')
    try:
        srv, cp, sp = _pair(lp)
        big = os.urandom(3 << 20)                 # forces EPOLLOUT flushing
        lp.run(lambda: cp.tr.write(b'hello ' + big))
        assert wait_for(lambda: len(sp.data) == 6 + len(big), 10)
        assert bytes(sp.data) == b'hello ' + big
        # half-close: the peer sees EOF and can still answer
        lp.run(cp.tr.write_eof)
        assert wait_for(lambda: 'eof' in sp.events, 5)
        lp.run(lambda: sp.tr.write(b'bye'))
        assert wait_for(lambda: bytes(cp.data) == b'bye', 5)
        lp.run(sp.tr.abort)
        assert wait_for(lambda: 'eof' in cp.events, 5)
        if kind == 'native':
            # both directions are down: the native loop closes the socket
            # and reports a clean loss (asyncio keeps it half-open)
            assert wait_for(lambda: ('lost', None) in cp.events, 5)
        lp.run(srv.close)
    finally:
        lp.stop()


def test_connect_refused_reports_on_loop(nl):
    import socket
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()                                   # nothing listens there
    fails = []
    p = Proto()
    nl.run(lambda: nl.open_connection(p, '127.0.0.1', port,
                                      lambda e: fails.append(
                                          (e, nl.in_loop()))))
    assert wait_for(lambda: fails, 5)
    exc, on_loop = fails[0]
    assert isinstance(exc, ConnectionRefusedError) and on_loop
    assert p.events == []


def test_pause_resume_and_cancelled_connect(nl):
    srv, cp, sp = _pair(nl)
    nl.run(sp.tr.pause_reading)
    nl.run(lambda: cp.tr.write(b'x' * 1000))
    time.sleep(0.1)
    assert len(sp.data) == 0
    nl.run(sp.tr.resume_reading)
    assert wait_for(lambda: len(sp.data) == 1000, 5)
    # an abandoned connect reports nothing
    p = Proto()
    fails = []
    nl.run(lambda: nl.open_connection(p, '127.0.0.1', srv.port,
                                      fails.append).cancel())
    time.sleep(0.1)
    assert p.events == [] and fails == []
    nl.run(srv.close)


@pytest.mark.parametrize('kind', ['native', 'asyncio'])
def test_client_stack_on_both_loops(kind):
    lp = nloop.NativeLoop('c') if kind == 'native' else Loop('c')
    slp = nloop.NativeLoop('s') if kind == 'native' else Loop('s')
    srv = FakeZKServer(loop=slp)
    try:
        c = client(srv.servers(), loop=lp)
        c.wait_connected(10)
        c.call_sync('create', '/loopkind', kind.encode(), {})
        data, stat = c.call_sync('get', '/loopkind')
        assert data == kind.encode() and stat.version == 0
        got = []
        c.watcher('/loopkind').on('dataChanged', lambda d, s: got.append(d))
        assert wait_for(lambda: got == [kind.encode()], 5)
        c.call_sync('set', '/loopkind', b'v2', -1)
        assert wait_for(lambda: got[-1:] == [b'v2'], 5)
        c.close_sync(10)
        assert c._test_recorder.events == ['session', 'connect', 'close']
        assert lp.errors == [] and slp.errors == []
    finally:
        srv.stop()
        lp.stop()
        slp.stop()


def test_transport_capture_routes_xid_range(nl):
    """Transport.capture: the reply frames of an xid range land in a raw
    buffer (length prefix included, in order) inside the loop's read path;
    other frames (a ping in the middle) still reach Python; a too-small
    buffer ends the capture with status 1 and the rest flows to Python."""
    import ctypes
    from zkmi import jute
    from zkmi.runtime.tcp import TcpSocket
    from zkmi.streams import ZKDecoder
    srv = FakeZKServer()
    for k in range(500):
        srv.cli_create('/c%03d' % k, b'v' * (k % 40))
    try:
        sock = TcpSocket(nl)
        dec = ZKDecoder()
        got = []
        sock.on('data', lambda d: got.extend(dec.feed(d)[0]))
        up = threading.Event()
        sock.on('connect', up.set)
        nl.run(lambda: sock.connect('127.0.0.1', srv.port))
        assert up.wait(5)
        nl.run(lambda: sock.write(jute.frame(jute.encode_connect_request({
            'protocolVersion': 0, 'lastZxidSeen': 0, 'timeOut': 30000,
            'sessionId': 0, 'passwd': b'\0' * 8}))))
        assert wait_for(lambda: len(got) == 1, 5)

        def gets(x0, n, ping_at):
            out = []
            for k in range(n):
                if k == ping_at:
                    out.append(jute.frame(jute.encode_request(
                        {'xid': -2, 'opcode': 'PING'})))
                out.append(jute.frame(jute.encode_request({
                    'xid': x0 + k, 'opcode': 'GET_DATA', 'watch': False,
                    'path': '/c%03d' % k})))
            return b''.join(out)
        # reference bytes: the same requests without capture
        got.clear()
        nl.run(lambda: sock.write(gets(100, 500, 250)))
        assert wait_for(lambda: len(got) == 501, 10)
        want = b''.join(jute.frame(b) for b in got
                        if b[:4] != b'\xff\xff\xff\xfe')
        # captured run
        for size, status_want in ((1 << 20, 0), (30000, 1)):
            got.clear()
            done = []
            buf = ctypes.create_string_buffer(size)
            nl.run(lambda: sock.capture(
                100, 500, ctypes.addressof(buf), size, 1 << 24,
                lambda *a: done.append(a), b''))
            nl.run(lambda: sock.write(gets(100, 500, 250)))
            assert wait_for(lambda: done, 10)
            st, nbytes, nframes, last = done[0]
            assert st == status_want
            assert buf.raw[:nbytes] == want[:nbytes]
            if st == 0:
                assert nframes == 500 and nbytes == len(want)
                assert wait_for(lambda: len(got) == 1, 5)   # the ping only
                assert got[0][:4] == b'\xff\xff\xff\xfe'
                assert buf.raw[last:last + 4] == want[last:last + 4]
            else:
                # the frames past the buffer arrive through 'data'
                assert wait_for(lambda: len(got) == 501 - nframes, 10)
        nl.run(sock.destroy)
    finally:
        srv.shutdown()


def test_chained_capture_takes_leftover_bytes(nl):
    """A capture whose done callback starts the next capture (a bulk
    callback chaining the next batch) hands the bytes after its last frame
    to that capture: with both batches' replies in one read, the second
    capture still gets all of its frames and Python none."""
    import ctypes
    from zkmi import jute
    from zkmi.runtime.tcp import TcpSocket
    from zkmi.streams import ZKDecoder
    srv = FakeZKServer()
    for k in range(100):
        srv.cli_create('/q%03d' % k, b'w' * (k % 50))
    try:
        sock = TcpSocket(nl)
        dec = ZKDecoder()
        got = []
        sock.on('data', lambda d: got.extend(dec.feed(d)[0]))
        up = threading.Event()
        sock.on('connect', up.set)
        nl.run(lambda: sock.connect('127.0.0.1', srv.port))
        assert up.wait(5)
        nl.run(lambda: sock.write(jute.frame(jute.encode_connect_request({
            'protocolVersion': 0, 'lastZxidSeen': 0, 'timeOut': 30000,
            'sessionId': 0, 'passwd': b'\0' * 8}))))
        assert wait_for(lambda: len(got) == 1, 5)
        got.clear()
        bufs = [ctypes.create_string_buffer(1 << 16) for _ in range(2)]
        done = []

        def second(*a):
            done.append(('b',) + a)

        def first(*a):
            done.append(('a',) + a)
            sock.capture(300, 50, ctypes.addressof(bufs[1]), 1 << 16,
                         1 << 24, second, b'')

        nl.run(lambda: sock.capture(200, 50, ctypes.addressof(bufs[0]),
                                    1 << 16, 1 << 24, first, b''))
        reqs = b''.join(jute.frame(jute.encode_request({
            'xid': x0 + k, 'opcode': 'GET_DATA', 'watch': False,
            'path': '/q%03d' % (k + (50 if x0 == 300 else 0))}))
            for x0 in (200, 300) for k in range(50))
        nl.run(lambda: sock.write(reqs))
        assert wait_for(lambda: len(done) == 2, 10), done
        assert [d[:2] for d in done] == [('a', 0), ('b', 0)]
        assert done[0][3] == 50 and done[1][3] == 50
        assert got == []
        nl.run(sock.destroy)
    finally:
        srv.shutdown()


def test_busy_poll_does_not_spin_between_timers():
    """With the busy-poll window on, a loop whose only events are timers
    blocks between them (the window follows socket activity only)."""
    import subprocess
    import sys
    if 'san' in os.environ.get('LD_PRELOAD', ''):
        pytest.skip('CPU-time check; meaningless under a sanitizer runtime')
    code = r'''
import resource, time
from zkmi.runtime import nloop
lp = nloop.NativeLoop('spin-check')
for k in range(1, 5):
    lp.call_later(200 * k, lambda: None)
time.sleep(0.1)
r0 = resource.getrusage(resource.RUSAGE_SELF)
time.sleep(0.9)
r1 = resource.getrusage(resource.RUSAGE_SELF)
lp.stop()
print((r1.ru_utime + r1.ru_stime) - (r0.ru_utime + r0.ru_stime))
'''
    env = dict(os.environ, ZKMI_LOOP_SPIN_US='50')
    env.pop('ZKMI_NATIVE_LOOP_PATH', None)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, '-c', code], cwd=root, env=env,
                         stdout=subprocess.PIPE, text=True, timeout=60)
    cpu = float(out.stdout.strip().splitlines()[-1])
    assert cpu < 0.15, 'loop burnt %.2f s of CPU in 0.9 s of timers' % cpu
