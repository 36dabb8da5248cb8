"""Event-loop runtime: one loop on a dedicated thread.

Two implementations with one surface: the native epoll loop
(:mod:`zkmi.runtime.nloop`, ``csrc/host/zk_loop.cpp``; the default when
built) and the asyncio loop below (``ZKMI_LOOP=asyncio``, and the fallback).

The reference is single-threaded on the Node event loop; every FSM, timer and
socket callback runs there.  We keep that model exactly — all
FSM code runs on the loop thread, so the state machines need no locks — and
add thread-safe entry points so ordinary (blocking) Python code can drive a
client from any thread.

``setImmediate`` -> :meth:`Loop.call_soon`; ``setTimeout`` ->
:meth:`Loop.call_later` (milliseconds); socket I/O uses asyncio transports.
Exceptions escaping a callback are recorded in :attr:`Loop.errors` (the Node
reference would crash the process — e.g. the watcher double-check,
``lib/zk-session.js:923-970``); the test-suite asserts the list stays empty.
"""

import asyncio
import logging
import threading
import time

_log = logging.getLogger('zkmi.loop')


class TimerHandle(object):
    """Timer wrapper with the Node-ish ``unref`` / ``cancel`` surface."""

    __slots__ = ('_h', 'cancelled')

    def __init__(self, h):
        self._h = h
        self.cancelled = False

    def cancel(self):
        if not self.cancelled:
            self.cancelled = True
            self._h.cancel()

    clear = cancel

    def unref(self):
        # asyncio timers never keep a daemon loop thread alive; kept for
        # parity with Node's timer.unref() used by the reference.
        return self


class Loop(object):

    def __init__(self, name='zkmi-loop'):
        self._loop = asyncio.new_event_loop()
        self._loop.set_exception_handler(self._on_exception)
        self.errors = []
        self._started = threading.Event()
        self._thread = threading.Thread(target=self._run, name=name,
                                        daemon=True)
        self._thread.start()
        self._started.wait()

    def _run(self):
        asyncio.set_event_loop(self._loop)
        self._loop.call_soon(self._started.set)
        self._loop.run_forever()

    def _on_exception(self, loop, ctx):
        exc = ctx.get('exception')
        msg = ctx.get('message')
        if exc is None:
            # asyncio housekeeping chatter (e.g. unclosed transports at
            # shutdown) is not a callback failure.
            _log.debug('loop: %s', msg)
            return
        self.errors.append(exc)
        _log.error('exception in loop callback: %s', msg, exc_info=exc)

    # -- scheduling ---------------------------------------------------------

    @property
    def aio(self):
        return self._loop

    def in_loop(self):
        return threading.current_thread() is self._thread

    def time_ms(self):
        return self._loop.time() * 1000.0

    def call_soon(self, fn, *args):
        if self.in_loop():
            return TimerHandle(self._loop.call_soon(fn, *args))
        return TimerHandle(self._loop.call_soon_threadsafe(fn, *args))

    def call_later(self, ms, fn, *args):
        if not self.in_loop():
            fut = self.run(lambda: self.call_later(ms, fn, *args))
            return fut
        return TimerHandle(self._loop.call_later(max(ms, 0) / 1000.0, fn,
                                                 *args))

    def run(self, fn, timeout=None):
        """Run ``fn()`` on the loop thread and return its result.

        Called from the loop thread it simply calls ``fn``."""
        if self.in_loop():
            return fn()
        done = threading.Event()
        box = {}

        def _call():
            try:
                box['r'] = fn()
            except BaseException as e:  # propagate to the caller
                box['e'] = e
            finally:
                done.set()
        self._loop.call_soon_threadsafe(_call)
        if not done.wait(timeout):
            raise TimeoutError('loop call timed out')
        if 'e' in box:
            raise box['e']
        return box.get('r')

    # -- sockets (same surface as the native loop) ---------------------------

    def open_connection(self, protocol, host, port, on_fail):
        """Start a TCP connect (any thread).  ``protocol`` gets the asyncio
        callbacks; ``on_fail(OSError)`` runs on the loop if the connect
        fails.  Returns a handle whose ``cancel()`` abandons the attempt."""
        async def go():
            try:
                await self._loop.create_connection(lambda: protocol, host,
                                                   port)
            except asyncio.CancelledError:
                return
            except OSError as e:
                on_fail(e)
        if self.in_loop():
            return self._loop.create_task(go())
        return asyncio.run_coroutine_threadsafe(go(), self._loop)

    def start_server(self, factory, host, port):
        """Listen on ``host:port`` (0 = any free port); call from a thread
        other than the loop's.  Returns an object with ``port`` and
        ``close()`` (close on the loop thread)."""
        async def go():
            return await self._loop.create_server(factory, host, port,
                                                  reuse_address=True)
        srv = asyncio.run_coroutine_threadsafe(go(), self._loop).result(10)
        return _AioServer(srv)

    def spawn(self, coro):
        """Schedule a coroutine on the loop (thread-safe)."""
        if self.in_loop():
            return self._loop.create_task(coro)
        return asyncio.run_coroutine_threadsafe(coro, self._loop)

    def stop(self):
        if self._loop.is_closed():
            return
        self._loop.call_soon_threadsafe(self._loop.stop)
        self._thread.join(timeout=5)


class _AioServer(object):
    __slots__ = ('_srv', 'port')

    def __init__(self, srv):
        self._srv = srv
        self.port = srv.sockets[0].getsockname()[1]

    def close(self):
        self._srv.close()


def new_loop(name='zkmi-loop'):
    """A new loop thread: native (epoll, csrc/host/zk_loop.cpp) when the
    extension is built, unless ``ZKMI_LOOP=asyncio``."""
    import os
    from . import nloop
    if os.environ.get('ZKMI_LOOP', 'native') != 'asyncio' and \
            nloop.available():
        return nloop.NativeLoop(name)
    return Loop(name)


_default = None
_default_lock = threading.Lock()


def default_loop():
    """The process-wide loop shared by clients that do not pass one (the
    Node reference shares one event loop between every client)."""
    global _default
    with _default_lock:
        if _default is None:
            _default = new_loop()
        return _default


def wait_for(cond, timeout=10.0, interval=0.01):
    """Poll ``cond()`` until true or ``timeout`` seconds pass
    (``test/utils.js:15-38``).  Returns the final value of ``cond()``."""
    deadline = time.monotonic() + timeout
    while True:
        v = cond()
        if v or time.monotonic() >= deadline:
            return v
        time.sleep(interval)
