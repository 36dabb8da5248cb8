"""FSM runtime (the re-provided mooremachine contract), event emitter,
watcher double-check, tracing, metrics and logging."""

import threading
import time

import pytest

from zkmi.runtime.emitter import EventEmitter
from zkmi.runtime.fsm import FSM
from zkmi.runtime.loop import default_loop, wait_for
from zkmi.server import FakeZKServer
from zkmi.utils.log import create_logger
from zkmi.utils.metrics import create_collector
from zkmi.utils.trace import RequestTracer

from zkhelpers import client, fast_config


class Toy(FSM):
    def __init__(self, loop, log):
        self.log = log
        self.ext = EventEmitter()
        FSM.__init__(self, 'a', loop)

    def state_a(self, S):
        self.log.append('enter a')
        S.on(self.ext, 'go', lambda: S.gotoState('b'))
        S.on(self.ext, 'sub', lambda: S.gotoState('a.sub'))

    def state_a__sub(self, S):
        self.log.append('enter a.sub')
        S.on(self.ext, 'up', lambda: S.gotoState('a'))

    def state_b(self, S):
        self.log.append('enter b')
        S.gotoState('c')           # synchronous transition in an entry
        self.log.append('after goto in b')

    def state_c(self, S):
        self.log.append('enter c')
        self.cb = S.callback(lambda: self.log.append('cb ran'))
        S.timeout(30, lambda: self.log.append('timeout fired'))
        S.on(self.ext, 'back', lambda: S.gotoState('a'))


@pytest.fixture(params=['native', 'python'])
def fsm_runtime(request, monkeypatch):
    """Both FSM runtimes: the native one (csrc/host/zk_fsm.cpp) and the
    Python oracle (ZKMI_PY_FSM=1)."""
    from zkmi.runtime import fsm
    if request.param == 'native':
        if fsm._zkfsm is None:
            pytest.skip('native FSM runtime not built')
        monkeypatch.delenv('ZKMI_PY_FSM', raising=False)
    else:
        monkeypatch.setenv('ZKMI_PY_FSM', '1')
    return request.param


def test_fsm_semantics(fsm_runtime):
    loop = default_loop()
    log = []
    changes = []

    def build():
        t = Toy(loop, log)
        t.on('stateChanged', changes.append)
        return t
    t = loop.run(build)
    assert t.isInState('a')
    loop.run(lambda: t.ext.emit('sub'))
    assert t.getState() == 'a.sub' and t.isInState('a')
    # parent handlers stay live in the sub-state
    assert t.ext.listenerCount('go') == 1
    loop.run(lambda: t.ext.emit('go'))
    # queued synchronous transition: b's entry completes before c enters,
    # and stateChanged follows entry order
    assert log[-4:] == ['enter b', 'after goto in b', 'enter c'][-3:] or \
        log[-3:] == ['enter b', 'after goto in b', 'enter c']
    assert changes[-2:] == ['b', 'c']
    # leaving a state disposes its listeners / timers / callbacks
    assert t.ext.listenerCount('go') == 0
    cb = t.cb
    loop.run(lambda: t.ext.emit('back'))
    time.sleep(0.08)
    loop.run(cb)
    assert 'timeout fired' not in log and 'cb ran' not in log
    assert t.getState() == 'a'


def test_fsm_stale_handle_raises(fsm_runtime):
    loop = default_loop()

    class T(FSM):
        def state_x(self, S):
            self.S = S

        def state_y(self, S):
            pass
    t = loop.run(lambda: T('x', loop))
    S = t.S
    loop.run(lambda: S.gotoState('y'))
    with pytest.raises(AssertionError):
        loop.run(lambda: S.gotoState('x'))


def test_fsm_runtime_kind(fsm_runtime):
    """The machine runs on the runtime asked for; the native core's
    interval re-arms and its disposal cancels it."""
    from zkmi.runtime import fsm
    loop = default_loop()
    ticks = []

    class T(FSM):
        def state_x(self, S):
            S.interval(10, lambda: ticks.append(1))
            S.on(self, 'stop', lambda: S.gotoState('y'))

        def state_y(self, S):
            pass
    t = loop.run(lambda: T('x', loop))
    kind = type(t._fsm_core).__name__
    assert kind == ('Core' if fsm_runtime == 'native' else 'PyCore')
    assert wait_for(lambda: len(ticks) >= 3, 5)
    loop.run(lambda: t.emit('stop'))
    n = len(ticks)
    time.sleep(0.08)
    assert len(ticks) == n and t.fsm_history == ['x', 'y']


def test_emitter_semantics():
    e = EventEmitter()
    got = []
    f = lambda *a: got.append(('f', a))   # noqa: E731
    e.on('x', f)
    e.once('x', lambda *a: got.append(('once', a)))
    e.emit('x', 1)
    e.emit('x', 2)
    assert got == [('f', (1,)), ('once', (1,)), ('f', (2,))]
    e.removeListener('x', f)
    assert not e.emit('x', 3)
    with pytest.raises(ValueError):
        e.emit('error', ValueError('boom'))


def test_watch_double_check_ok_and_miss():
    """armed -> armed.doublecheck (4h + U(0,8h) in production, ms here):
    the re-read zxid must match, else the missed wakeup is fatal
    (zk-session.js:923-970)."""
    zk = FakeZKServer(tick_ms=250)
    loop = default_loop()
    try:
        cfg = fast_config(doublecheck_ms=150, doublecheck_rand_ms=0)
        c = client(zk.servers(), config=cfg)
        c.wait_connected(10)
        zk.cli_create('/dc', b'1')
        seen = []
        c.watcher('/dc').on('dataChanged', lambda d, s: seen.append(d))
        assert wait_for(lambda: seen == [b'1'], 5)
        ev = c.watcher('/dc').evts['dataChanged']
        assert wait_for(lambda: 'armed.doublecheck' in ev.fsm_history, 5)
        assert wait_for(lambda: ev.getState() == 'armed', 5)
        # now change the node WITHOUT notifying the client (a lost wakeup)
        before = len(loop.errors)

        def sneaky():
            n = zk.db.nodes['/dc']
            zk.db.zxid += 1
            n.data = b'2'
            n.stat.mzxid = zk.db.zxid
            zk.db.data_watches.pop('/dc', None)
        zk.run(sneaky)
        assert wait_for(lambda: len(loop.errors) > before, 5)
        err = loop.errors.pop()
        assert 'double-check failed' in str(err)
        c.close_sync(10)
    finally:
        zk.shutdown()


def test_request_tracer_and_metrics():
    zk = FakeZKServer(tick_ms=250)
    try:
        tr = RequestTracer()
        col = create_collector()
        c = client(zk.servers(), tracer=tr, collector=col)
        c.wait_connected(10)
        for _ in range(20):
            c.call_sync('ping')
        c.call_sync('create', '/t', b'x', {})
        for _ in range(30):
            c.call_sync('get', '/t')
        s = tr.summary()
        assert s['GET_DATA']['n'] == 30 and s['PING']['n'] >= 20
        assert s['GET_DATA']['p99_us'] >= s['GET_DATA']['p50_us'] > 0
        assert col.getCollector('zookeeper_events').get(
            {'evtype': 'connect'}) == 1
        c.close_sync(10)
    finally:
        zk.shutdown()


def test_structured_logger_children():
    import io
    buf = io.StringIO()
    log = create_logger('t', level='trace', stream=buf, a=1)
    recs = log.capture()
    ch = log.child(component='X', b=2)
    ch.info({'k': 'v'}, 'hello %s', 'world')
    ch.trace('t')
    assert recs[0]['msg'] == 'hello world' and recs[0]['a'] == 1
    assert recs[0]['component'] == 'X' and recs[0]['k'] == 'v'
    assert recs[1]['level'] == 10
    assert '"msg": "hello world"' in buf.getvalue()


def test_loop_run_from_threads():
    loop = default_loop()
    out = []

    def worker(i):
        out.append(loop.run(lambda: (loop.in_loop(), i)))
    ts = [threading.Thread(target=worker, args=(i,)) for i in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert sorted(out) == [(True, i) for i in range(8)]


class _ManualLoop(object):
    """A loop whose clock only moves when the test advances it."""

    def __init__(self):
        self.now = 0.0
        self.timers = []

    def time_ms(self):
        return self.now

    def call_later(self, ms, fn):
        loop = self

        class _H(object):
            cancelled = False

            def cancel(self):
                self.cancelled = True
                loop.timers.remove(entry)
        entry = [self.now + ms, fn, _H()]
        self.timers.append(entry)
        return entry[2]

    def advance(self, ms):
        end = self.now + ms
        while True:
            due = [t for t in self.timers if t[0] <= end]
            if not due:
                break
            t = min(due, key=lambda e: e[0])
            self.timers.remove(t)
            self.now = t[0]
            t[1]()
        self.now = end


def test_expiry_timer_rearms_on_shorter_timeout():
    """A reattach that negotiates a shorter session timeout must move the
    expiry earlier (lib/zk-session.js:99-108 clears and re-sets the timer on
    every reset); a reset with the same timeout pushes the deadline out."""
    from zkmi.models.session import ExpiryTimer
    loop = _ManualLoop()
    fired = []
    t = ExpiryTimer(loop)
    t.on('timeout', lambda: fired.append(loop.time_ms()))
    t.reset(30000)
    loop.advance(1000)
    t.reset(4000)              # deadline 5000, not the old 30000
    loop.advance(10000)
    assert fired == [5000]
    t.reset(4000)              # at 11000: deadline 15000
    loop.advance(2000)
    t.reset(4000)              # at 13000: deadline pushed to 17000
    loop.advance(3000)
    assert fired == [5000]
    loop.advance(1000)
    assert fired == [5000, 17000]
