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
    return Client(o)


class Recorder(object):
    """Collects client events in order (the reference tests push event
    names into an array, test/basic.test.js:1001-1004)."""

    def __init__(self, c, events=('session', 'connect', 'disconnect',
                                  'expire', 'failed', 'close')):
        self.events = []
        self.lock = threading.Lock()
        for e in events:
            c.on(e, self._mk(e))

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
