"""L4 — one TCP connection to one ZooKeeper server.

Parity: ``ZKConnectionFSM`` (``lib/connection-fsm.js:27-351``), ``ZKRequest``
and reply routing (``:353-413``), ping / liveness (``:201-207``,
``:415-463``), ``setWatches`` (``:465-499``).

State graph (same as the reference)::

    init -> connecting -> handshaking -> connected -> closing -> closed
                 \\             \\             \\__________> error -> closed
                  \\_____________\\__________________________^

Per-connection state: the xid counter (starts at 0), the outstanding request
table keyed by xid, and the xid->opcode map the reply decoder needs because
ZooKeeper replies are not self-describing (SURVEY §7.4 hard part 1).
"""

import operator
import threading
import time

from .. import consts
from .. import codec
from ..errors import ZKError, ZKProtocolError, ZKPingTimeoutError, \
    ZKDecodeError
from ..runtime.emitter import EventEmitter
from ..runtime.fsm import FSM
from ..runtime.tcp import TcpSocket
from ..streams import ZKDecoder, ZKEncoder
from . import gpucodec
from .session import _zkmach, native_machines



class ZKRequest(EventEmitter):
    """An outstanding request; emits ``reply(pkt)`` or ``error(err, pkt)``
    (``lib/connection-fsm.js:378-382``).

    :meth:`then` registers a (reply, error) pair called directly, without
    listener bookkeeping — the client data API's per-request path."""

    __slots__ = ('packet', 't_submit', 'fast')

    def __init__(self, packet):
        self._listeners = {}
        self.packet = packet
        self.t_submit = 0.0             # set when a tracer records it
        self.fast = None

    def then(self, on_reply, on_error):
        self.fast = (on_reply, on_error)
        return self

    def settle(self, evt, *args):
        f = self.fast
        if f is None:
            self.emit(evt, *args)
            return
        f[0 if evt == 'reply' else 1](*args)
        if self._listeners.get(evt):
            self.emit(evt, *args)


def ZKConnectionFSM(client, backend, log, loop, config, tracer=None):
    """A connection: the native machine, or the Python oracle."""
    cls = NativeZKConnectionFSM if native_machines() else PyZKConnectionFSM
    return cls(client, backend, log, loop, config, tracer=tracer)


class _ConnBase(object):
    """The connection's transport plumbing (framing, request table, the
    native reply router, bulk batches, bulk notification capture) — what it
    is besides its state graph."""

    def __init__(self, client, backend, log, loop, config, tracer=None):
        self.client = client
        self.server = backend                 # {'address':..., 'port':...}
        self.log = log.child(component='ZKConnectionFSM')
        self.config = config
        self.tracer = tracer
        self.decoder = None
        self.encoder = None
        self.gpu = None
        self.xid_map = {}
        self.xid = 0
        # xids are also taken off the loop thread (request_direct)
        self.xid_lock = threading.Lock()
        self.bulks = []                 # in-flight BulkBatch (models/bulk.py)
        # bulk watch notifications (Client.watch_bulk): kept by the native
        # transport (note sink), or here on the asyncio loop
        self.note_native = False
        self.notes = None
        self.notes_left = (b'', 0)
        self.note_sess = None       # whose watchers the note sink spares
        self.bulk_frames_py = 0         # bulk replies routed one by one
        self.routing = False            # native reply router on (_route)
        self.reqs = {}
        self.socket = None
        self.session = None
        self.wanted = True
        self.last_error = None

    def nextXid(self):
        with self.xid_lock:
            x = self.xid
            self.xid = (x + 1) & 0x7fffffff
        return x

    # -- inbound plumbing -----------------------------------------------------

    def _on_data(self, chunk):
        dec = self.decoder
        if dec is None:
            return
        bodies, err = dec.feed(chunk)
        n = len(bodies)
        for i, body in enumerate(bodies):
            if self.decoder is not dec:
                return              # torn down mid-chunk
            self._in_rx(body, n - i - 1)
        if err is not None and self.decoder is dec:
            self._in_rxerr(err)

    def _decode_reply(self, body):
        try:
            pkt = codec.decode_response(body, self.xid_map)
        except (ZKDecodeError, ValueError, KeyError, UnicodeDecodeError) as e:
            raise ZKProtocolError('BAD_DECODE', 'Failed to decode Response: '
                                  '%s: %s' % (type(e).__name__, e))
        xid = pkt['xid']
        if xid >= 0:
            self.xid_map.pop(xid, None)
        return pkt

    # -- native completion path ----------------------------------------------

    def _route(self, on):
        """Settle replies to outstanding requests in the native transport
        (``Transport.route``, csrc/host/zk_loop.cpp): it frames the stream,
        decodes each reply whose xid is in :attr:`reqs` with the host codec,
        unlinks it from :attr:`reqs` and :attr:`xid_map` and calls the
        request's ``then`` pair — the per-reply work of ``on_rx`` /
        ``_decode_reply`` / ``processReply`` without a Python frame in
        between (``lib/connection-fsm.js:213-229``, ``:384-408``).  Every
        other frame still comes through ``on_rx`` in stream order.  Off while
        a tracer or trace logging wants each reply, on the asyncio loop and
        outside ``connected``."""
        sock = self.socket
        if not on:
            if self.routing:
                self.routing = False
                if sock is not None and sock.transport is not None:
                    z, rx, _ = sock.transport.route_state()
                    sock.transport.route(False, None, None, None, None, 0,
                                         b'')
                    if self.session is not None:
                        self.session.fold_routed(z, rx)
            return
        if self.routing or not self.config.native_route or sock is None or \
                not sock.can_route() or \
                self.tracer is not None or self.log.enabled('trace') or \
                codec.DECODE_REPLY_C is None or self.decoder is None or \
                self.decoder.dead:
            return
        sock.transport.route(True, self.reqs, self.xid_map,
                             self._routed_other, codec.DECODE_REPLY_C,
                             self.config.max_packet,
                             self.decoder.take_pending(),
                             codec.ENCODE_REQUEST_C,
                             self._routed_note if self.notes is None
                             else None)
        self.routing = True

    def route_state(self):
        """(max zxid, loop ms of the last frame) the router settled."""
        sock = self.socket
        if not self.routing or sock is None or sock.transport is None:
            return 0, 0.0
        z, rx, _ = sock.transport.route_state()
        return z, rx

    def _routed_note(self, pkt):
        """A NOTIFICATION the router decoded: to the session, as on_rx
        hands it over (lib/zk-session.js:227-238)."""
        self.emit('packet', pkt)

    def _routed_other(self, req, pkt):
        """A routed reply the transport does not hand straight to the
        request's ``then`` pair: an error reply, or a listener-style
        request (processReply's delivery, the entry already unlinked)."""
        if pkt['err'] == 'OK':
            req.settle('reply', pkt)
            return
        code = pkt['err']
        err = ZKError(code, consts.ERR_TEXT.get(code, str(code)))
        req.settle('error', err, pkt)

    # -- requests -------------------------------------------------------------

    def processReply(self, pkt):
        # the entry goes before the reply is delivered, as endRequest (the
        # first 'reply' listener) does at lib/connection-fsm.js:405-407
        req = self.reqs.pop(pkt['xid'], None)
        if self.tracer is not None and req is not None:
            self.tracer.record(pkt['xid'], pkt['opcode'], req.t_submit,
                               pkt['err'])
        self.log.trace({'xid': pkt['xid'], 'opcode': pkt['opcode'],
                        'errorCode': pkt['err']},
                       'server replied to request')
        if req is None:
            return
        if pkt['err'] == 'OK':
            req.settle('reply', pkt)
            return
        code = pkt['err']
        err = ZKError(code, consts.ERR_TEXT.get(code, str(code)))
        req.settle('error', err, pkt)

    def request(self, pkt, req=None):
        """Send ``pkt``; returns the request (``req``: an object with the
        ZKRequest surface the reply settles — the native watch engine's)."""
        if self._fsm_state != 'connected':
            raise Exception('Client must be connected to send requests')
        if req is None:
            req = ZKRequest(pkt)
            if self.tracer is not None:
                req.t_submit = time.perf_counter()
        with self.xid_lock:
            xid = self.xid
            self.xid = (xid + 1) & 0x7fffffff
        pkt['xid'] = xid
        if self.routing and pkt['opcode'] != 'SET_WATCHES' and \
                self.socket.transport.request(pkt, req):
            # encoded into the write buffer, entered in reqs / xid_map by
            # the native transport; the router settles the reply
            return req
        self.reqs[xid] = req      # removed by processReply / the fail paths
        self.log.trace({'xid': xid, 'opcode': pkt['opcode']},
                       'sent request to server')
        self.socket.write(self.encoder.request(pkt))
        return req

    def request_direct(self, pkt, on_reply, on_error):
        """:meth:`request` from a thread other than the loop's (the
        blocking helpers): the request is encoded and sent from the calling
        thread, the reply settled by the native router on the loop thread —
        one cross-thread hand-off instead of two.  The (reply, error) pair is
        attached before the request leaves, so a reply cannot beat it.
        Returns False (nothing sent) when the router is not on; the caller
        then goes through the loop."""
        if not self.routing or self._fsm_state != 'connected' or \
                pkt['opcode'] == 'SET_WATCHES':
            return False
        sock = self.socket
        t = sock.transport if sock is not None else None
        if t is None:
            return False
        req = ZKRequest(pkt)
        req.fast = (on_reply, on_error)
        with self.xid_lock:
            xid = self.xid
            self.xid = (xid + 1) & 0x7fffffff
        pkt['xid'] = xid
        r = t.request(pkt, req)
        if r is None:
            return False        # router went off meanwhile (xid skipped)
        if not r:
            # the transport is closing: the request fails as the loop
            # path's would once the connection reports the loss
            self.fsm_loop.call_soon(
                on_error, ZKProtocolError('CONNECTION_LOSS',
                                          'Connection closed.'))
        return True

    # -- bulk watch notifications (Client.watch_bulk) ------------------------

    def start_note_capture(self):
        """Keep this connection's NOTIFICATION frames for
        :meth:`take_notes` (loop thread): in the native transport (its read
        path frames the stream and keeps them; the partial frame Python's
        framer holds is handed over), else in :attr:`notes`."""
        if self.note_native or self.notes is not None:
            return
        sock = self.socket
        sess = self.session or self.client.getSession()
        self.note_sess = sess
        if sock is not None and sock.can_sink_notes():
            pre = self.decoder.take_pending() if self.decoder else b''
            sock.note_sink(True, self.config.max_packet, pre,
                           sess.watchers if sess is not None else None,
                           sess.bulk_watches if sess is not None else None)
            self.note_native = True
        else:
            self.notes = bytearray()
            self.notes_n = 0
        self.client.note_conns.add(self)

    def _note_keep(self, body):
        """Python twin of the native sink's filter (zk_loop.cpp note_take):
        keep a NOTIFICATION body in :attr:`notes`; True when the session
        should also get it (its path has a watcher())."""
        sess = self.note_sess
        keep, to_py = True, False
        if sess is not None and sess.watchers and len(body) >= 28:
            n = int.from_bytes(body[24:28], 'big', signed=True)
            if 0 <= n <= len(body) - 28:
                path = body[28:28 + n].decode('utf-8', 'replace')
                if path in sess.watchers:
                    to_py = True
                    keep = path in sess.bulk_watches
        if keep:
            self.notes += len(body).to_bytes(4, 'big')
            self.notes += body
            self.notes_n += 1
        return to_py

    def take_notes(self):
        """(bytes, frames) kept since the last call."""
        if self.note_native:
            sock = self.socket
            if sock is None:
                left, self.notes_left = self.notes_left, (b'', 0)
                return left
            return sock.take_notes()
        if not self.notes:
            return b'', 0
        b, n = bytes(self.notes), self.notes_n
        self.notes = bytearray()
        self.notes_n = 0
        return b, n

    # -- bulk (GPU-coded, pipelined) batches ----------------------------------

    def bulk_submit(self, batch, cb):
        """Send a :class:`~zkmi.models.bulk.BulkBatch`: reserve a contiguous
        xid range, encode (K10 on the GPU), one socket write.  ``cb(err,
        result)`` runs on the loop thread once every reply arrived."""
        if not self.isInState('connected'):
            raise ZKProtocolError('CONNECTION_LOSS', 'Not connected.')
        n = batch.n
        batch.cb = cb
        batch.t_submit = time.perf_counter()
        if n == 0:
            # nothing to send: no xids, no encode, an empty result
            self.fsm_loop.call_soon(lambda: cb(None, batch.finish()))
            return
        with self.xid_lock:
            x0 = self.xid
            if x0 + n > 0x7fffffff:
                x0 = 0
            self.xid = (x0 + n) & 0x7fffffff
        wire = batch.encode(x0)
        self.bulks.append(batch)
        if batch.device is not None and self.socket.can_capture() and \
                not any(b.capturing for b in self.bulks):
            # the native loop routes the batch's replies into pinned memory
            addr, size = batch.rx_buffer()
            batch.capturing = True
            self.socket.capture(
                x0, n, addr, size, self.config.max_packet,
                lambda st, nb, got, last, b=batch:
                    self._bulk_captured(b, st, nb, got, last),
                self.decoder.take_pending())
        batch.t['send0'] = time.perf_counter()
        if isinstance(wire, tuple):
            self.log.trace({'xid0': x0, 'n': n, 'bytes': wire[1]},
                           'sent bulk batch')
            self.socket.write_from(*wire)
        else:
            self.log.trace({'xid0': x0, 'n': n, 'bytes': len(wire)},
                           'sent bulk batch')
            self.socket.write(wire)
        batch.t['sent'] = time.perf_counter()

    def _bulk_captured(self, b, status, nbytes, got, last_off):
        """The transport's capture of ``b`` ended (loop thread)."""
        if b not in self.bulks:
            return
        if not b.captured(status, nbytes, got):
            return              # per-frame collection goes on (_bulk_rx)
        # one 'packet' for the batch: the last reply's zxid keeps the
        # session's lastZxid and expiry current
        hdr = bytes(b.rx_pin[last_off + 4:last_off + 16].numpy().tobytes())
        self.emit('packet', {'xid': int.from_bytes(hdr[:4], 'big',
                                                   signed=True),
                             'opcode': 'BULK',
                             'zxid': int.from_bytes(hdr[4:12], 'big',
                                                    signed=True)})
        self.bulks.remove(b)
        try:
            res = b.finish(nbytes)
        except Exception as e:                  # decode failure -> caller
            b.cb(e)
        else:
            b.cb(None, res)
        self._in_bulkdone()

    def _bulk_rx(self, xid, body):
        for b in self.bulks:
            if b.owns(xid):
                self.bulk_frames_py += 1
                # header zxid keeps the session's lastZxid / expiry current
                self.emit('packet', {'xid': xid, 'opcode': 'BULK',
                                     'zxid': int.from_bytes(body[4:12], 'big',
                                                            signed=True)})
                if b.add(body):
                    self.bulks.remove(b)
                    try:
                        res = b.finish()
                    except Exception as e:      # decode failure -> caller
                        b.cb(e)
                        return True
                    b.cb(None, res)
                return True
        return False

    def _fail_bulks(self, err):
        bulks, self.bulks = self.bulks, []
        for b in bulks:
            b.cb(err)

    def send(self, pkt):
        """Raw write of a handshake record (ConnectRequest)."""
        self.socket.write(self.encoder.connect_request(pkt))

    def ping(self, cb=None):
        if not self.isInState('connected'):
            raise Exception('Client must be connected to send packets')
        xid = consts.XID_PING
        cur = self.reqs.get(xid)
        if cur is not None:
            # Coalesce onto the outstanding ping (connection-fsm.js:425-435).
            cur.once('reply', lambda *_: cb and cb(None))
            cur.once('error', lambda err, *_: cb and cb(err))
            return
        pkt = {'xid': xid, 'opcode': 'PING'}
        req = ZKRequest(pkt)
        self.reqs[xid] = req
        T = self.session.getTimeout()
        cfg = self.config
        timeout = max(T / cfg.ping_timeout_divisor, cfg.ping_timeout_floor_ms)
        t1 = time.monotonic()

        def on_packet(pkt2):
            if self.reqs.get(xid) is req:
                del self.reqs[xid]
            timer.cancel()
            ms = (time.monotonic() - t1) * 1000.0
            self.log.trace('ping ok in %d ms', ms)
            if cb:
                cb(None, ms)

        def on_timeout():
            req.removeListener('reply', on_packet)
            self._in_ping_timeout()

        def on_error(err, *_):
            if self.reqs.get(xid) is req:
                del self.reqs[xid]
            timer.cancel()
            if cb:
                cb(err)
        req.once('reply', on_packet)
        req.once('error', on_error)
        timer = self.fsm_loop.call_later(timeout, on_timeout)
        self.socket.write(self.encoder.request(pkt))

    def setWatches(self, events, zxid, cb):
        if not self.isInState('connected'):
            raise Exception('Client must be connected to send packets (is '
                            'in state %s)' % self.getState())
        xid = consts.XID_SET_WATCHES
        cur = self.reqs.get(xid)
        if cur is not None:
            cur.once('reply', lambda *_: self.setWatches(events, zxid, cb))
            cur.once('error', lambda err, *_: cb(err))
            return
        pkt = {'xid': xid, 'opcode': 'SET_WATCHES', 'relZxid': zxid,
               'events': events}
        req = ZKRequest(pkt)
        self.reqs[xid] = req

        def on_packet(_pkt):
            if self.reqs.get(xid) is req:
                del self.reqs[xid]
            cb(None)

        def on_error(err, *_):
            if self.reqs.get(xid) is req:
                del self.reqs[xid]
            cb(err)
        req.once('reply', on_packet)
        req.once('error', on_error)
        self.socket.write(self.encoder.request(pkt))

    # -- test hooks (the reference tests poke conn.zcf_socket directly) ------

    @property
    def zcf_socket(self):
        return self.socket


class PyZKConnectionFSM(_ConnBase, FSM):
    """The connection's state graph as mooremachine-style state functions
    (``lib/connection-fsm.js:27-351``): the test oracle of the native machine
    (``ZKMI_PY_FSM=1``)."""

    def __init__(self, client, backend, log, loop, config, tracer=None):
        _ConnBase.__init__(self, client, backend, log, loop, config, tracer)
        FSM.__init__(self, 'init', loop)

    # -- reference method names ---------------------------------------------

    def connect(self):
        assert self.isInState('closed') or self.isInState('init')
        self.emit('connectAsserted')

    def setUnwanted(self):
        self.wanted = False
        self.log.debug('connection now unwanted')
        self.emit('unwanted')

    def close(self):
        if self.isInState('closed'):
            return
        self.emit('closeAsserted')

    def destroy(self):
        if self.isInState('closed'):
            return
        self.emit('destroyAsserted')

    # -- inputs (the native machine takes them as fire() calls) ------------

    def _in_rx(self, body, more):
        self.emit('_rx', body, more)

    def _in_rxerr(self, err):
        self.emit('_rxerr', err)

    def _in_ping_timeout(self):
        self.emit('pingTimeout')

    def _in_bulkdone(self):
        self.emit('_bulkdone')

    # -- states ---------------------------------------------------------------

    def state_init(self, S):
        S.on(self, 'connectAsserted', lambda: S.gotoState('connecting'))

    def state_connecting(self, S):
        self.decoder = ZKDecoder(self.config.max_packet)
        self.gpu = gpucodec.for_device(self.config.codec_device)
        self.encoder = ZKEncoder(self.xid_map, self.gpu)
        self.log = self.log.child(zkAddress=self.server['address'],
                                  zkPort=self.server['port'])
        self.log.trace('attempting new connection')
        sock = TcpSocket(self.fsm_loop)
        self.socket = sock
        sock.on('data', self._on_data)

        def on_error(err):
            self.last_error = err
            S.gotoState('error')
        S.on(sock, 'connect', lambda: S.gotoState('handshaking'))
        S.on(sock, 'error', on_error)
        S.on(sock, 'close', lambda: S.gotoState('closed'))
        S.on(self, 'closeAsserted', lambda: S.gotoState('closed'))
        S.on(self, 'destroyAsserted', lambda: S.gotoState('closed'))
        sock.connect(self.server['address'], self.server['port'])

    def state_handshaking(self, S):
        if not self.wanted:
            S.gotoState('closed')
            return
        if getattr(self.client, 'note_capture', False):
            self.start_note_capture()

        def on_rx(body, more):
            if more > 0:
                self.last_error = ZKProtocolError(
                    'UNEXPECTED_PACKET', 'Received unexpected additional '
                    'packet during connect phase')
                S.gotoState('error')
                return
            try:
                if self.gpu is not None:
                    pkt = self.gpu.connect_response(body)
                else:
                    pkt = codec.decode_connect_response(body)
            except (ZKDecodeError, ValueError) as e:
                self.last_error = ZKProtocolError(
                    'BAD_DECODE', 'Failed to decode ConnectResponse: %s: %s'
                    % (type(e).__name__, e))
                S.gotoState('error')
                return
            if pkt['protocolVersion'] != 0:
                self.last_error = ZKProtocolError(
                    'VERSION_INCOMPAT', 'Server version is not compatible')
                S.gotoState('error')
                return
            self.emit('packet', pkt)

        def on_error(err):
            self.last_error = err
            S.gotoState('error')

        def on_end():
            self.last_error = ZKProtocolError(
                'CONNECTION_LOSS', 'Connection closed unexpectedly.')
            S.gotoState('error')

        S.on(self, '_rx', on_rx)
        S.on(self, '_rxerr', on_error)
        S.on(self.socket, 'error', on_error)
        S.on(self.socket, 'end', on_end)
        S.on(self.socket, 'close', on_end)
        S.on(self, 'closeAsserted', lambda: S.gotoState('closed'))
        S.on(self, 'destroyAsserted', lambda: S.gotoState('closed'))
        S.on(self, 'unwanted', lambda: S.gotoState('closed'))

        self.session = self.client.getSession()
        if self.session is None:
            S.gotoState('closed')
            return
        if self.session.isAttaching():
            self.log.debug('found ZKSession in state %s while handshaking',
                           self.session.getState())
            self.last_error = Exception('ZKSession attaching to another '
                                        'connection')
            S.gotoState('error')
            return

        def on_session(st):
            # Only when the session attached through THIS connection.  The
            # reference advances on any 'attached', so after a reattach
            # revert (zk-session.js:298-320) the rejected connection would
            # turn 'connected', get preferred by the set, and kill the
            # connection the session actually lives on.
            if st == 'attached' and self.session.conn is self:
                S.gotoState('connected')
        S.on(self.session, 'stateChanged', on_session)
        self.session.attachAndSendCR(self)

    def state_connected(self, S):
        T = self.session.getTimeout()
        cfg = self.config
        interval = max(T / cfg.ping_interval_divisor, cfg.ping_floor_ms)
        S.interval(interval, lambda: self.ping()).unref()
        self.log = self.log.child(sessionId=self.session.getSessionId())

        def on_rx(body, more):
            if self.bulks and len(body) >= 16:
                xid = int.from_bytes(body[0:4], 'big', signed=True)
                if xid >= 0 and self._bulk_rx(xid, body):
                    return
            if self.notes is not None and len(body) >= 16 and \
                    body[0:4] == b'\xff\xff\xff\xff' and \
                    not self._note_keep(body):
                return
            try:
                pkt = self._decode_reply(body)
            except ZKProtocolError as e:
                self.last_error = e
                S.gotoState('error')
                return
            self.emit('packet', pkt)
            # Notifications are handled by the session (watchers).
            if pkt['opcode'] == 'NOTIFICATION':
                return
            self.processReply(pkt)

        def on_error(err):
            self.last_error = err
            S.gotoState('error')

        def on_end():
            self.last_error = ZKProtocolError(
                'CONNECTION_LOSS', 'Connection closed unexpectedly.')
            S.gotoState('error')

        def on_ping_timeout():
            self.last_error = ZKPingTimeoutError()
            S.gotoState('error')

        S.on(self, '_rx', on_rx)
        S.on(self, '_rxerr', on_error)
        S.on(self.socket, 'error', on_error)
        S.on(self.socket, 'end', on_end)
        S.on(self.socket, 'close', on_end)
        S.on(self, 'closeAsserted', lambda: S.gotoState('closing'))
        S.on(self, 'destroyAsserted', lambda: S.gotoState('closed'))
        S.on(self, 'pingTimeout', on_ping_timeout)
        self._route(True)
        S.immediate(lambda: self.emit('connect'))

    def state_closing(self, S):
        self._route(False)
        box = {'xid': None}

        def send_close_session():
            if box['xid'] is not None:
                return
            box['xid'] = xid = self.nextXid()
            self.log.info({'xid': xid}, 'sent CLOSE_SESSION request')
            data = self.encoder.request({'opcode': 'CLOSE_SESSION',
                                         'xid': xid})
            self.socket.end(data)

        def on_rx(body, more):
            if self.bulks and len(body) >= 16:
                xid = int.from_bytes(body[0:4], 'big', signed=True)
                if xid >= 0 and self._bulk_rx(xid, body):
                    if len(self.reqs) < 1 and not self.bulks:
                        send_close_session()
                    return
            try:
                pkt = self._decode_reply(body)
            except ZKProtocolError as e:
                self.last_error = e
                S.gotoState('closed')
                return
            if box['xid'] is None or pkt['xid'] != box['xid']:
                self.processReply(pkt)
                if len(self.reqs) < 1 and not self.bulks:
                    send_close_session()
            else:
                S.gotoState('closed')

        def on_error(err):
            self.last_error = err
            S.gotoState('closed')

        def on_bulk_done():
            if len(self.reqs) < 1 and not self.bulks:
                send_close_session()

        S.on(self, '_rx', on_rx)
        S.on(self, '_rxerr', on_error)
        S.on(self, '_bulkdone', on_bulk_done)
        S.on(self.socket, 'error', on_error)
        S.on(self.socket, 'end', lambda: S.gotoState('closed'))
        S.on(self.socket, 'close', lambda: S.gotoState('closed'))
        # destroy() is ignored while closing, as in the reference: the
        # CLOSE_SESSION exchange completes (or the socket dies).  In-flight
        # bulk batches drain like ordinary requests.
        if len(self.reqs) < 1 and not self.bulks:
            send_close_session()

    def state_error(self, S):
        self._route(False)
        err = self.last_error
        self.log.warn(err if isinstance(err, BaseException) else {},
                      'error communicating with ZK')
        reqs, self.reqs = self.reqs, {}
        for req in list(reqs.values()):
            req.settle('error', err)
        self._fail_bulks(err)
        # Not S.immediate: this must be emitted even though we leave the
        # state right away (lib/connection-fsm.js:318-323).
        self.fsm_loop.call_soon(self._emit_error, err)
        S.gotoState('closed')

    def _emit_error(self, err):
        if self.listenerCount('error') > 0:
            self.emit('error', err)

    def state_closed(self, S):
        self._route(False)
        self.encoder = None
        if self.socket is not None and self.note_native:
            # the notifications the transport kept outlive it
            self.notes_left = self.socket.take_notes()
        if self.socket is not None:
            self.socket.destroy()
        self.socket = None
        self.decoder = None

        def later():
            self.emit('close')
            err = ZKProtocolError('CONNECTION_LOSS', 'Connection closed.')
            reqs, self.reqs = self.reqs, {}
            for req in list(reqs.values()):
                req.settle('error', err)
            self._fail_bulks(err)
        S.immediate(later)


class NativeZKConnectionFSM(_ConnBase, EventEmitter):
    """The connection on the C++ machine (``_zkmach.Machine('connection')``,
    csrc/host/zk_machines.cpp): states, guards (the handshake's packet
    count and protocol version, the session's attach), the ping timer and
    the close handshake run there; the effect methods below do what the
    machine asks of the transport."""

    def __init__(self, client, backend, log, loop, config, tracer=None):
        EventEmitter.__init__(self)
        _ConnBase.__init__(self, client, backend, log, loop, config, tracer)
        self.fsm_loop = loop
        self._m = _zkmach.Machine('connection', self, loop)
        self._m.start('init')

    # -- FSM surface ----------------------------------------------------------

    def getState(self):
        return self._m.state

    _fsm_state = property(operator.attrgetter('_m.state'))

    def isInState(self, state):
        return self._m.in_state(state)

    @property
    def fsm_history(self):
        return self._m.history

    # -- reference method names ---------------------------------------------

    def connect(self):
        assert self.isInState('closed') or self.isInState('init')
        self._m.fire(_zkmach.CE_CONNECT)

    def setUnwanted(self):
        self.wanted = False
        self.log.debug('connection now unwanted')
        self._m.fire(_zkmach.CE_UNWANTED)

    def close(self):
        if self.isInState('closed'):
            return
        self._m.fire(_zkmach.CE_CLOSE)

    def destroy(self):
        if self.isInState('closed'):
            return
        self._m.fire(_zkmach.CE_DESTROY)

    # -- inputs -------------------------------------------------------------

    def _in_rx(self, body, more):
        self._m.fire(_zkmach.CE_RX, body, more)

    def _in_rxerr(self, err):
        self._m.fire(_zkmach.CE_RXERR, err)

    def _in_ping_timeout(self):
        self._m.fire(_zkmach.CE_PING_TIMEOUT)

    def _in_bulkdone(self):
        self._m.fire(_zkmach.CE_BULKDONE)

    # -- effects the machine asks for -----------------------------------------

    @staticmethod
    def _proto_error(code, msg):
        return ZKProtocolError(code, msg)

    @staticmethod
    def _ping_timeout_error():
        return ZKPingTimeoutError()

    def _fx_open(self):
        """connecting: framing, codec, a new socket (its data listener
        first; the machine's relays go on after)."""
        self.decoder = ZKDecoder(self.config.max_packet)
        self.gpu = gpucodec.for_device(self.config.codec_device)
        self.encoder = ZKEncoder(self.xid_map, self.gpu)
        self.log = self.log.child(zkAddress=self.server['address'],
                                  zkPort=self.server['port'])
        self.log.trace('attempting new connection')
        sock = TcpSocket(self.fsm_loop)
        self.socket = sock
        sock.on('data', self._on_data)

    def _fx_dial(self):
        self.socket.connect(self.server['address'], self.server['port'])

    def _decode_cr(self, body):
        """The ConnectResponse, or the error to fail with."""
        try:
            if self.gpu is not None:
                return self.gpu.connect_response(body)
            return codec.decode_connect_response(body)
        except (ZKDecodeError, ValueError) as e:
            return ZKProtocolError(
                'BAD_DECODE', 'Failed to decode ConnectResponse: %s: %s'
                % (type(e).__name__, e))

    def _fx_connected(self):
        self.log = self.log.child(sessionId=self.session.getSessionId())
        self._route(True)

    def _rx_connected(self, body):
        """A frame in 'connected': bulk batches, kept notifications, then
        the reply / notification path.  Returns the error to fail with."""
        if self.bulks and len(body) >= 16:
            xid = int.from_bytes(body[0:4], 'big', signed=True)
            if xid >= 0 and self._bulk_rx(xid, body):
                return None
        if self.notes is not None and len(body) >= 16 and \
                body[0:4] == b'\xff\xff\xff\xff' and \
                not self._note_keep(body):
            return None
        try:
            pkt = self._decode_reply(body)
        except ZKProtocolError as e:
            return e
        self.emit('packet', pkt)
        # Notifications are handled by the session (watchers).
        if pkt['opcode'] != 'NOTIFICATION':
            self.processReply(pkt)
        return None

    def _fx_route_off(self):
        self._route(False)

    def _fx_send_close(self, xid):
        self.log.info({'xid': xid}, 'sent CLOSE_SESSION request')
        data = self.encoder.request({'opcode': 'CLOSE_SESSION', 'xid': xid})
        self.socket.end(data)

    def _rx_closing(self, body, close_xid):
        """A frame in 'closing': 1 when it ends the exchange (the
        CLOSE_SESSION reply, or an undecodable frame), else 0."""
        if self.bulks and len(body) >= 16:
            xid = int.from_bytes(body[0:4], 'big', signed=True)
            if xid >= 0 and self._bulk_rx(xid, body):
                return 0
        try:
            pkt = self._decode_reply(body)
        except ZKProtocolError as e:
            self.last_error = e
            return 1
        if close_xid is None or pkt['xid'] != close_xid:
            self.processReply(pkt)
            return 0
        return 1

    def _fx_error(self):
        self._route(False)
        err = self.last_error
        self.log.warn(err if isinstance(err, BaseException) else {},
                      'error communicating with ZK')
        reqs, self.reqs = self.reqs, {}
        for req in list(reqs.values()):
            req.settle('error', err)
        self._fail_bulks(err)
        self.fsm_loop.call_soon(self._emit_error, err)

    def _emit_error(self, err):
        if self.listenerCount('error') > 0:
            self.emit('error', err)

    def _fx_closed(self):
        self._route(False)
        self.encoder = None
        if self.socket is not None and self.note_native:
            # the notifications the transport kept outlive it
            self.notes_left = self.socket.take_notes()
        if self.socket is not None:
            self.socket.destroy()
        self.socket = None
        self.decoder = None

    def _fx_closed_later(self):
        self.emit('close')
        err = ZKProtocolError('CONNECTION_LOSS', 'Connection closed.')
        reqs, self.reqs = self.reqs, {}
        for req in list(reqs.values()):
            req.settle('error', err)
        self._fail_bulks(err)
