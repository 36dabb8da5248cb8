"""Shared helpers for the client integration suites (the role of the
reference's test/zkserver.js + test/utils.js)."""

import threading
import time

from zkmi import Client
from zkmi.config import ClientConfig, RecoveryPolicy
from zkmi.runtime.loop import wait_for  # noqa: F401


def fast_config(**kw):
    """Reference semantics with the time constants shrunk so failure /
    expiry scenarios finish in seconds."""
    cfg = ClientConfig(
        ping_floor_ms=kw.pop('ping_floor_ms', 200),
        ping_timeout_floor_ms=kw.pop('ping_timeout_floor_ms', 200),
        connect_policy=kw.pop('connect_policy',
                              RecoveryPolicy(1000, 3, 50, 400)),
        default_policy=kw.pop('default_policy',
                              RecoveryPolicy(1000, 3, 100, 800)),
        **kw)
    return cfg


def client(servers, session_timeout=None, config=None, **kw):
    o = {'servers': servers, 'config': config or fast_config()}
    if session_timeout is not None:
        o['sessionTimeout'] = session_timeout
    o.update(kw)
    rec = Recorder(None)
    o['listeners'] = rec.listeners() + list(o.get('listeners') or ())
    c = Client(o)
    c._test_recorder = rec
    return c


class Recorder(object):
    """Collects client events in order (the reference tests push event
    names into an array, test/basic.test.js:1001-1004).  ``client()``
    attaches one before the client starts; ``Recorder(c)`` returns it, so
    no early 'session'/'connect' is lost to the loop thread."""

    EVENTS = ('session', 'connect', 'disconnect', 'expire', 'failed', 'close')

    def __new__(cls, c, events=EVENTS):
        pre = getattr(c, '_test_recorder', None)
        if pre is not None:
            return pre
        return object.__new__(cls)

    def __init__(self, c, events=EVENTS):
        if getattr(self, 'events', None) is not None:
            return
        self.events = []
        self.lock = threading.Lock()
        self._names = events
        if c is not None:
            for e in events:
                c.on(e, self._mk(e))

    def listeners(self):
        return [(e, self._mk(e)) for e in self._names]

    def _mk(self, e):
        def f(*a):
            with self.lock:
                self.events.append(e)
        return f

    def count(self, e):
        with self.lock:
            return self.events.count(e)

    def wait(self, e, n=1, timeout=10.0):
        ok = wait_for(lambda: self.count(e) >= n, timeout)
        assert ok, 'timed out waiting for %d x %r (have %r)' % (
            n, e, self.events)


class Box(object):
    """Thread-safe result box for callbacks."""

    def __init__(self):
        self.ev = threading.Event()
        self.val = None

    def __call__(self, *a):
        self.val = a
        self.ev.set()

    def wait(self, timeout=10.0):
        assert self.ev.wait(timeout), 'callback not called'
        return self.val


def sleep(s):
    time.sleep(s)
