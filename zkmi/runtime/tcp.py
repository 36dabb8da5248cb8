"""TCP socket with Node ``net.Socket``-like events, on the zkmi loop.

Events: ``connect``, ``data(bytes)``, ``end`` (peer half-closed; the socket
stays writable — the reference connects with ``allowHalfOpen: true``,
``lib/connection-fsm.js:99-103``), ``error(exc)``, ``close``.

Test hooks replace the reference tests' direct pokes at the socket
(``sock.emit('error')``, ``sock.destroy()``, ``sock.unpipe()``;
``test/basic.test.js:1059-1062``, ``:1260``, ``:1374``):
:meth:`inject_error`, :meth:`destroy`, :meth:`pause_reading`.
"""

import asyncio
import socket as _socket

from .emitter import EventEmitter


class _Proto(asyncio.Protocol):

    def __init__(self, sock):
        self.sock = sock

    def connection_made(self, transport):
        self.sock._on_made(transport)

    def data_received(self, data):
        self.sock._on_data(data)

    def eof_received(self):
        self.sock._on_eof()
        return True

    def connection_lost(self, exc):
        self.sock._on_lost(exc)


class TcpSocket(EventEmitter):

    def __init__(self, loop):
        EventEmitter.__init__(self)
        self.loop = loop
        self.transport = None
        self.closed = False
        self.ended = False
        self.connecting = False
        self._task = None
        self._paused = False
        self._held = []
        self.remote = None
        self.bytes_in = 0
        self.bytes_out = 0

    # -- client side ----------------------------------------------------------

    def connect(self, host, port):
        self.connecting = True
        self.remote = (host, port)
        self._task = self.loop.open_connection(_Proto(self), host, port,
                                               self._connect_failed)
        return self

    def _connect_failed(self, e):
        self.connecting = False
        if not self.closed:
            self._fail(e)

    # -- server side ----------------------------------------------------------

    @classmethod
    def protocol_for(cls, loop, on_accept):
        """Protocol factory for ``loop.start_server``: ``on_accept(sock)``
        is called with a connected :class:`TcpSocket`."""
        def factory():
            s = cls(loop)
            s._on_accept = on_accept
            return _Proto(s)
        return factory

    # -- transport callbacks --------------------------------------------------

    def _on_made(self, transport):
        self.transport = transport
        self.connecting = False
        sk = transport.get_extra_info('socket')
        if sk is not None:
            try:
                sk.setsockopt(_socket.IPPROTO_TCP, _socket.TCP_NODELAY, 1)
            except OSError:
                pass
        if self.closed:
            transport.abort()
            return
        acc = getattr(self, '_on_accept', None)
        if acc is not None:
            acc(self)
        else:
            self.emit('connect')

    def _on_data(self, data):
        if self.closed:
            return
        self.bytes_in += len(data)
        if self._paused:
            self._held.append(data)
            return
        self.emit('data', data)

    def _on_eof(self):
        if not self.closed:
            self.emit('end')

    def _on_lost(self, exc):
        if self.closed:
            return
        if exc is not None:
            self._fail(exc)
        else:
            self.closed = True
            self.emit('close')

    def _fail(self, exc):
        self.closed = True
        if self.transport is not None:
            self.transport.abort()
        self.emit('error', exc)
        self.emit('close')

    # -- API -----------------------------------------------------------------

    def write(self, data):
        """Queue ``data``; never raises (a write on a half-closed or dying
        socket is dropped, as Node drops writes after ``end()``).  An
        exception here would otherwise surface in whatever transport
        callback triggered the write and kill *that* connection."""
        if self.closed or self.ended or self.transport is None or \
                self.transport.is_closing():
            return False
        self.bytes_out += len(data)
        try:
            self.transport.write(data)
        except (OSError, RuntimeError):
            return False
        return True

    # -- GPU bulk path (native loop only) -------------------------------------

    def can_capture(self):
        """True when the transport can route a reply xid range into a
        buffer itself (the native loop's Transport.capture)."""
        return (self.transport is not None and not self.closed and
                not self._paused and hasattr(self.transport, 'capture'))

    def capture(self, x0, n, addr, size, max_packet, done, prefix=b''):
        """Copy the reply frames with xid in [x0, x0+n) into ``size``
        bytes at ``addr`` (a pinned host buffer) inside the loop's read
        path; ``done(status, nbytes, nframes, last_off)`` ends it (0 all
        frames, 1 buffer full, 2 bad frame length, 3 cancelled; the frames
        not captured go to 'data' as usual)."""
        self.transport.capture(x0, n, addr, size, max_packet, done, prefix)

    def can_route(self):
        """True when the transport can settle replies itself (the native
        loop's Transport.route)."""
        return (self.transport is not None and not self.closed and
                not self._paused and hasattr(self.transport, 'route'))

    def can_sink_notes(self):
        """True when the transport can keep NOTIFICATION frames itself (the
        native loop's Transport.note_sink)."""
        return (self.transport is not None and not self.closed and
                hasattr(self.transport, 'note_sink'))

    def note_sink(self, on, max_packet, prefix=b'', watchers=None,
                  bulk=None):
        """Keep (``on``) every NOTIFICATION frame in the transport instead of
        emitting it; :meth:`take_notes` drains them.  An event on a path of
        ``watchers`` (the session's path -> ZKWatcher dict) is emitted too,
        and kept only when its path is in ``bulk``."""
        self.transport.note_sink(on, max_packet, prefix, watchers, bulk)

    def take_notes(self):
        """(bytes, frames): the NOTIFICATION frames kept since the last
        call, length prefixes included."""
        t = self.transport
        if t is None or not hasattr(t, 'take_notes'):
            return b'', 0
        return t.take_notes()

    def capture_cancel(self):
        if self.transport is not None and hasattr(self.transport,
                                                  'capture_cancel'):
            self.transport.capture_cancel()

    def write_from(self, addr, n):
        """Queue ``n`` bytes at ``addr`` (raw memory, e.g. a pinned host
        buffer the GPU encoder filled) without a bytes object."""
        if self.closed or self.ended or self.transport is None or \
                self.transport.is_closing():
            return False
        f = getattr(self.transport, 'write_from', None)
        if f is None:
            import ctypes
            return self.write(ctypes.string_at(addr, n))
        self.bytes_out += n
        try:
            return f(addr, n)
        except (OSError, RuntimeError):
            return False

    def end(self, data=None):
        """Half-close after writing ``data`` (Node ``socket.end``)."""
        if data:
            self.write(data)
        if self.transport is not None and not self.closed and \
                not self.ended:
            self.ended = True
            try:
                if self.transport.can_write_eof():
                    self.transport.write_eof()
            except (OSError, RuntimeError):
                pass

    def destroy(self):
        if self.closed:
            return
        self.closed = True
        if self._task is not None and self.connecting:
            self._task.cancel()
        if self.transport is not None:
            self.transport.abort()
        self.loop.call_soon(self.emit, 'close')

    def pause_reading(self):
        """Stop delivering ``data`` events (the reference test #46 unpipes
        the socket, ``test/basic.test.js:1374``)."""
        self._paused = True
        t = self.transport
        if t is not None and hasattr(t, 'route'):
            # held means held: the native reply router stops settling (its
            # partial frame comes back through data_received, held here)
            t.route(False, None, None, None, None, 0, b'')

    def resume_reading(self):
        self._paused = False
        held, self._held = self._held, []
        for d in held:
            self.emit('data', d)

    def inject_error(self, err):
        """Emit ``error`` then close, as a real socket failure would."""
        if self.closed:
            return
        self._fail(err)
