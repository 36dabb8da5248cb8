"""The native watch-event engine (csrc/host/zk_watch.cpp): every watch of a
session in one native table instead of one ZKWatchEvent state machine per
(path, event).  The same scenarios run against the engine and against the
Python FSMs (``ClientConfig(native_watch=False)``) and must give the same
event sequences; at scale the engine holds thousands of watches with no
Python state machine behind them.

Reference: lib/zk-session.js:527-614 (ZKWatcher), :616-1005
(ZKWatchEvent), :421-471 (SET_WATCHES resume)."""

import threading

import pytest

from zkmi.server import fast
from zkmi.server.fakezk import FakeZKServer

from zkhelpers import client, fast_config, wait_for

try:
    from zkmi import _zkwatch
except ImportError:
    _zkwatch = None

pytestmark = pytest.mark.skipif(_zkwatch is None,
                                reason='watch engine not built')


def _scenario(native):
    """Data, children and existence watches through changes, a deletion
    and a forced reconnect (the watches resume with SET_WATCHES); returns
    the events every listener saw, in order."""
    zk = FakeZKServer(tick_ms=250)
    got = []
    lock = threading.Lock()

    def rec(*ev):
        with lock:
            got.append(ev)
    try:
        cfg = fast_config(native_watch=native)
        c = client(zk.servers(), config=cfg)
        w = client(zk.servers())
        c.wait_connected(10)
        w.wait_connected(10)
        w.call_sync('create', '/a', b'1', {})
        c.watcher('/a').on('dataChanged',
                           lambda d, s: rec('a.data', d, s.version))
        c.watcher('/a').on('deleted', lambda: rec('a.deleted'))
        c.watcher('/kids').on('childrenChanged',
                              lambda k, s: rec('kids', sorted(k)))
        c.watcher('/later').on('created', lambda s: rec('later.created'))
        assert wait_for(lambda: ('a.data', b'1', 0) in got, 5)
        w.call_sync('set', '/a', b'2', -1)
        assert wait_for(lambda: ('a.data', b'2', 1) in got, 5)
        w.call_sync('create', '/kids', b'', {})
        assert wait_for(lambda: ('kids', []) in got, 5)
        w.call_sync('create', '/kids/x', b'', {})
        assert wait_for(lambda: ('kids', ['x']) in got, 5)
        # a forced reconnect: the watches resume (SET_WATCHES) and a change
        # made while disconnected is caught up
        conn = c.getSession().getConnection()
        reconnected = threading.Event()
        c.once('connect', lambda: reconnected.set())
        c.loop.run(lambda: conn.zcf_socket.destroy())
        w.call_sync('set', '/a', b'3', -1)
        assert reconnected.wait(10)
        assert wait_for(lambda: ('a.data', b'3', 2) in got, 5)
        w.call_sync('create', '/later', b'', {})
        assert wait_for(lambda: ('later.created',) in got, 5)
        w.call_sync('delete', '/a', -1)
        assert wait_for(lambda: ('a.deleted',) in got, 5)
        sess = c.getSession()
        kinds = sorted(type(ev).__name__ for ev in
                       c.loop.run(lambda: [e for p in ('/a', '/kids')
                                           for e in sess.watchers[p]
                                           .events()]))
        c.close_sync(10)
        w.close_sync(10)
        return got, kinds
    finally:
        zk.shutdown()


def test_engine_matches_python_fsms():
    got_native, kinds_native = _scenario(True)
    got_py, kinds_py = _scenario(False)
    assert got_native == got_py
    assert set(kinds_native) == {'_NativeWatchEvent'}
    assert set(kinds_py) == {'ZKWatchEvent'}


@pytest.mark.skipif(not fast.available(), reason='zk_fastserver not built')
def test_engine_thousands_of_watchers():
    """2000 paths watched the reference way (watcher(p).on('dataChanged')),
    every one fired by a bulk write and re-armed: one native table entry
    each, no Python state machine."""
    srv = fast.FastZKServer(preload=2000, data_bytes=8, fanout=100)
    try:
        c = client([srv.address])
        w = client([srv.address])
        c.wait_connected(10)
        w.wait_connected(10)
        paths = ['/bench/d%06d/n%09d' % (i // 100, i) for i in range(2000)]
        seen = {}
        lock = threading.Lock()

        def on(p):
            def f(data, stat):
                with lock:
                    seen.setdefault(p, []).append(stat.version)
            return f
        for p in paths:
            c.watcher(p).on('dataChanged', on(p))
        assert wait_for(lambda: len(seen) == 2000, 20)
        wt = c.getSession().wt
        assert c.loop.run(wt.counts)['armed'] == 2000
        res = w.call_sync('bulk_set', paths, b'new')
        assert res.errors() == ['OK'] * 2000
        assert wait_for(lambda: all(seen[p] == [0, 1] for p in paths), 20)
        assert wait_for(lambda: c.loop.run(wt.counts)['armed'] == 2000, 10)
        st = c.loop.run(lambda: wt.state(paths[7], 'dataChanged'))
        assert st == 'armed'
        hist = c.loop.run(lambda: wt.history(paths[7], 'dataChanged'))
        assert hist[:4] == ['wait_session', 'arming', 'armed', 'wait_session']
        c.close_sync(10)
        w.close_sync(10)
    finally:
        srv.shutdown()


def _raising_created(native):
    """A data watch on a missing node waits for it (wait_node) behind the
    implicit existence watch; a user 'created' listener that raises must
    not leave the data watch stuck, and its exception reaches the loop's
    errors (the Python FSMs pass it on the same way)."""
    zk = FakeZKServer(tick_ms=250)
    got = []
    try:
        c = client(zk.servers(), config=fast_config(native_watch=native))
        w = client(zk.servers())
        c.wait_connected(10)
        w.wait_connected(10)
        errs0 = len(c.loop.errors)

        def boom(stat):
            got.append('created')
            raise RuntimeError('listener failed')
        c.watcher('/n').on('dataChanged', lambda d, s: got.append(d))
        c.watcher('/n').on('created', boom)
        assert wait_for(lambda: c.loop.run(
            lambda: c.getSession().wt.state('/n', 'dataChanged')
            if native else 'wait_node') == 'wait_node', 5)
        w.call_sync('create', '/n', b'x', {})
        assert wait_for(lambda: b'x' in got, 5), got
        errs = c.loop.run(lambda: c.loop.errors[errs0:])
        c.loop.run(lambda: c.loop.errors.__delitem__(
            slice(errs0, len(c.loop.errors))))
        c.close_sync(10)
        w.close_sync(10)
        return got, [type(e).__name__ for e in errs]
    finally:
        zk.shutdown()


def test_raising_listener_does_not_strand_wait_node():
    """(The reference's EventEmitter would crash the process on the throw;
    the Python FSMs leave the data watch in wait_node.  The engine keeps
    going and hands the error to the loop.)"""
    got, errs = _raising_created(True)
    assert got == ['created', b'x']
    assert errs == ['RuntimeError']


def test_closed_session_is_collected():
    """The table refers to the session (its emit) and the session to the
    table: a GC type pair, so a closed client's session and its watch
    engine are collected, and close() stops the doublecheck timer."""
    import gc
    import weakref
    zk = FakeZKServer(tick_ms=250)
    try:
        c = client(zk.servers())
        c.wait_connected(10)
        c.call_sync('create', '/g', b'1', {})
        seen = []
        c.watcher('/g').on('dataChanged', lambda d, s: seen.append(d))
        assert wait_for(lambda: seen == [b'1'], 5)
        sess = c.getSession()
        ref = weakref.ref(sess)
        wt = sess.wt
        assert c.loop.run(wt.counts)['armed'] == 1
        c.close_sync(10)
        assert c.loop.run(wt.counts)['armed'] == 0
        del sess, wt
        loop = c.loop
        c = None
        for _ in range(3):
            loop.run(lambda: None)
            gc.collect()
        assert ref() is None, gc.get_referrers(ref())
    finally:
        zk.shutdown()
