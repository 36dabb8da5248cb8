"""Native event loop: ``csrc/host/zk_loop.cpp`` (epoll + eventfd + timer
heap + non-blocking TCP) on a dedicated thread.

The reference's runtime is Node's native event loop (libuv); this is
zkmi's.  Same surface as the asyncio :class:`~zkmi.runtime.loop.Loop`
(``call_soon``, ``call_later``, ``run``, ``in_loop``, ``time_ms``,
``open_connection``, ``start_server``, ``errors``, ``stop``), so every FSM,
the TCP socket wrapper and the fake server run unchanged on either.
:func:`zkmi.runtime.loop.default_loop` picks this one when the extension is
built (``ZKMI_LOOP=asyncio`` selects the asyncio loop).
"""

import logging
import threading

_log = logging.getLogger('zkmi.loop')

def _load():
    """The in-tree extension, or the one at ``ZKMI_NATIVE_LOOP_PATH`` (the
    sanitizer build, tools/sanitize_host.sh)."""
    import os
    path = os.environ.get('ZKMI_NATIVE_LOOP_PATH')
    if path:
        import importlib.util
        spec = importlib.util.spec_from_file_location('_zkloop', path)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        return mod
    try:
        from .. import _zkloop as mod
    except ImportError:     # not built (tools/build_native.py builds it)
        return None
    return mod


_zkloop = _load()


def available():
    return _zkloop is not None


class _ServerHandle(object):
    __slots__ = ('_s',)

    def __init__(self, s):
        self._s = s

    @property
    def port(self):
        return self._s.port

    def close(self):
        self._s.close()


class NativeLoop(object):

    native = True

    def __init__(self, name='zkmi-loop'):
        if _zkloop is None:
            raise RuntimeError('zkmi native loop not built: run '
                               '`python tools/build_native.py`')
        self.errors = []
        self._n = _zkloop.Loop(self._on_exception)
        # (the C method itself: asked on every data-API request)
        self.in_loop = self._n.in_loop
        self._thread = threading.Thread(target=self._main, name=name,
                                        daemon=True)
        started = threading.Event()
        self._n.call_soon(started.set)
        self._thread.start()
        started.wait()

    def _main(self):
        try:
            self._n.run()
        except BaseException as e:      # the loop itself failed
            self.errors.append(e)
            _log.error('native loop died: %s', e)

    def _on_exception(self, exc):
        self.errors.append(exc)
        _log.error('exception in loop callback: %r', exc, exc_info=exc)

    # -- scheduling ---------------------------------------------------------

    def waiter(self):
        """A completion flag a blocking caller waits on with the GIL
        released; ``set()`` from the loop thread takes effect when the loop
        next releases the GIL (csrc/host/zk_loop.cpp Waiter)."""
        return _zkloop.Waiter(self._n)

    def in_loop(self):
        return self._n.in_loop()

    def time_ms(self):
        return self._n.time_ms()

    def call_soon(self, fn, *args):
        return self._n.call_soon(fn, args)

    def call_later(self, ms, fn, *args):
        return self._n.call_later(max(ms, 0), fn, args)

    def run(self, fn, timeout=None):
        """Run ``fn()`` on the loop thread and return its result (called
        from the loop thread it simply calls ``fn``)."""
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
        self._n.call_soon(_call)
        if not done.wait(timeout):
            raise TimeoutError('loop call timed out')
        if 'e' in box:
            raise box['e']
        return box.get('r')

    # -- sockets ----------------------------------------------------------

    def open_connection(self, protocol, host, port, on_fail):
        """Start a TCP connect.  ``protocol`` gets asyncio-style callbacks;
        ``on_fail(OSError)`` runs on the loop if the connect fails.  Returns
        a handle whose ``cancel()`` abandons the attempt."""
        return self._n.connect(host, int(port), protocol, on_fail)

    def start_server(self, factory, host, port):
        """Listen on ``host:port`` (0 = any free port); ``factory()`` makes
        the protocol of each accepted connection.  Returns an object with
        ``port`` and ``close()``."""
        return _ServerHandle(self._n.listen(host, int(port), factory))

    def stats(self):
        return self._n.stats()

    def stop(self):
        if not self._thread.is_alive():
            return
        self._n.stop()
        if not self.in_loop():
            self._thread.join(timeout=5)
