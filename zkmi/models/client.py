"""L6 — the public ``Client`` (lifecycle FSM + data API).

Parity: ``ZKClient`` (``lib/client.js:31-601``): option handling
(``:34-83``), connection management (``:88-118``, ``:275-309``), lifecycle
states ``normal`` / ``closing`` / ``closed`` (``:127-181``), session event
wiring (``:187-262``) and the data API (``:318-601``).

Threading: every FSM runs on the client's :class:`~zkmi.runtime.loop.Loop`
thread.  Public methods may be called from any thread: arguments are
validated synchronously in the caller (bad arguments raise, like the
reference's ``assert-plus`` checks, ``test/nasty.test.js:197-221``), then
the operation is marshalled onto the loop.  Callbacks and events always run
on the loop thread.  ``*_sync`` helpers block the calling thread for a
result (they must not be called from the loop thread itself).
"""

import os
import threading
import time

from .. import consts
from ..config import ClientConfig
from ..errors import ZKNotConnectedError
from ..jute import DEFAULT_ACL, Stat  # noqa: F401  (re-export)
from ..runtime.emitter import EventEmitter
from ..runtime.fsm import FSM
from ..runtime.loop import default_loop
from ..utils.log import create_logger
from ..utils.metrics import create_collector, METRIC_ZK_EVENT_COUNTER
from .connection import ZKConnectionFSM
from .connection_set import ConnectionSet, StaticResolver

# call_sync's default poll window before it sleeps on the reply lock
# (ClientConfig.sync_spin_us): 100 us on hosts with >= 16 CPUs — on a GPU
# box the blocking get() RTT went 37-44 -> 20 us (a 30 us window is shorter
# than the round trip and does nothing); off on small hosts, where the
# poller competes with the loop thread for the GIL.
_SYNC_SPIN_US_AUTO = 100.0 if (os.cpu_count() or 1) >= 16 else 0.0
# ZKMI_SYNC_WAITER=0: call_sync waits on a bare lock even on the native loop
_SYNC_WAITER = os.environ.get('ZKMI_SYNC_WAITER', '1') == '1'
from .session import ZKSession, _zkmach, native_machines


def _check_str(v, name):
    if not isinstance(v, str):
        raise TypeError('%s (string) is required' % name)


def _check_func(v, name='callback'):
    if not callable(v):
        raise TypeError('%s (func) is required' % name)


def _check_bytes(v, name):
    if not isinstance(v, (bytes, bytearray, memoryview)):
        raise TypeError('%s (buffer) is required' % name)


def _check_int(v, name, optional=False):
    if v is None and optional:
        return
    if isinstance(v, bool) or not isinstance(v, int):
        raise TypeError('%s (number) is required' % name)


def _norm_options(options):
    if options is None:
        options = {}
    if not isinstance(options, dict):
        raise TypeError('options (object) is required')
    options = dict(options)
    acl = options.get('acl')
    if acl is not None and (not isinstance(acl, list) or
                            not all(isinstance(a, dict) for a in acl)):
        raise TypeError('options.acl ([object]) is required')
    flags = options.get('flags')
    if flags is not None and (not isinstance(flags, list) or
                              not all(isinstance(f, str) for f in flags)):
        raise TypeError('options.flags ([string]) is required')
    if acl is None:
        options['acl'] = [dict(a) for a in DEFAULT_ACL]
    if flags is None:
        options['flags'] = []
    for f in options['flags']:
        if f not in consts.CREATE_FLAGS:
            raise ValueError('unknown flag %r' % (f,))
    return options


class Client(FSM):
    """A ZooKeeper client.

    ``Client(address='127.0.0.1', port=2181)`` or
    ``Client(servers=[{'address':..., 'port':...}, ...])``; optional
    ``sessionTimeout`` (ms, default 30000), ``log``, ``collector``,
    ``loop``, ``config`` (:class:`~zkmi.config.ClientConfig`) and
    ``session`` (credentials from :meth:`credentials` to resume an existing
    session) and ``listeners`` (``{event: fn}`` or ``[(event, fn)]``,
    attached before the client starts, so none of its events is missed)."""

    def __init__(self, opts=None, **kw):
        o = dict(opts or {})
        o.update(kw)
        log = o.get('log')
        if log is None:
            self.log = create_logger('zkmi', component='ZKClient')
        else:
            self.log = log.child(component='ZKClient')
        self.collector = o.get('collector') or create_collector()
        self.collector.counter(METRIC_ZK_EVENT_COUNTER,
                               'Total number of zookeeper events')
        servers = o.get('servers')
        if servers is None:
            _check_str(o.get('address'), 'options.address')
            _check_int(o.get('port'), 'options.port')
            self.servers = [{'address': o['address'], 'port': o['port']}]
        else:
            if not isinstance(servers, list) or not servers:
                raise TypeError('options.servers ([object]) is required')
            for s in servers:
                _check_str(s.get('address'), 'servers[].address')
                _check_int(s.get('port'), 'servers[].port')
            self.servers = [dict(s) for s in servers]
        st = o.get('sessionTimeout')
        _check_int(st, 'options.sessionTimeout', optional=True)
        self.session_timeout = consts.DEFAULT_SESSION_TIMEOUT if st is None \
            else st
        self.config = o.get('config') or ClientConfig()
        self.loop = o.get('loop') or default_loop()
        # submissions from other threads still queued for the loop (_hop)
        self._hop_lock = threading.Lock()
        self._hops = 0
        self.tracer = o.get('tracer')
        # bulk codec device: None = the current GPU if any, False = host
        self.bulk_device = o.get('device')
        # bulk watches (watch_bulk): connections keep notification frames
        self.note_capture = False
        self.note_conns = set()
        self._resume_cred = o.get('session')
        # listeners attached before the FSM starts: a JS caller attaching
        # in the constructor's tick sees every event; on a loop thread that
        # only holds if the listeners are in place before the resolver runs
        self._early = list((o.get('listeners') or {}).items()) \
            if isinstance(o.get('listeners'), dict) \
            else list(o.get('listeners') or ())
        self.session = None
        self.old_session = None
        self.conns = {}
        self.hdls = {}
        self.loop.run(self._init_on_loop)

    def _init_on_loop(self):
        EventEmitter.__init__(self)
        for evt, fn in self._early:
            self.on(evt, fn)
        self._early = None
        self.resolver = StaticResolver(self.servers, consts.DEFAULT_PORT)
        self.cset = ConnectionSet(self.resolver, self._makeConnection,
                                 self.loop, self.log, self.config)
        self.cset.on('added', self._onSetAdded)
        self.cset.on('removed', self._onSetRemoved)
        self.cset.on('stateChanged', self._onSetStateChanged)
        if native_machines():
            # the lifecycle on the C++ machine (csrc/host/zk_machines.cpp
            # 'client'); FSM's getState / isInState read it as their core
            self.fsm_loop = self.loop
            self._fsm_core = _zkmach.Machine('client', self, self.loop)
            self._fsm_core.start('normal')
        else:
            FSM.__init__(self, 'normal', self.loop)

    # aliases matching the reference's private field names used by tests
    @property
    def zc_set(self):
        return self.cset

    # -- lifecycle ------------------------------------------------------------

    def _fx_normal(self):
        """Entering 'normal': the first session, then the resolver."""
        self._newSession()
        if self._resume_cred is not None:
            self.session.adopt_credentials(self._resume_cred)
            self._resume_cred = None
        self.resolver.start()

    # the lifecycle as state functions: the Python oracle (ZKMI_PY_FSM=1)
    # of the native machine

    def state_normal(self, S):
        self._fx_normal()
        S.on(self, 'closeAsserted', lambda: S.gotoState('closing'))

    def state_closing(self, S):
        box = {'done': 0}

        def bump():
            box['done'] += 1
            if box['done'] == 3:
                S.gotoState('closed')

        S.on(self.session, 'stateChanged',
             lambda st: bump() if st in ('closed', 'expired') else None)
        S.on(self.cset, 'stateChanged',
             lambda st: bump() if st == 'stopped' else None)
        S.on(self.resolver, 'stateChanged',
             lambda st: bump() if st == 'stopped' else None)
        if self.session.isInState('closed') or \
                self.session.isInState('expired'):
            box['done'] += 1
        if self.cset.isInState('stopped'):
            box['done'] += 1
        if self.resolver.isInState('stopped'):
            box['done'] += 1
        if box['done'] == 3:
            S.gotoState('closed')
            return
        self.cset.stop()
        self.resolver.stop()
        self.session.close()
        S.interval(self.config.close_log_interval_ms,
                   lambda: self.log.trace('still waiting for zk client to '
                                          'shut down, %d/3 done',
                                          box['done']))

    def state_closed(self, S):
        self.emit('close')

    def close(self, cb=None):
        """Close the client; ``cb`` (optional) runs on ``'close'`` (the
        reference documents it but ignores it)."""
        def go():
            if cb is not None:
                if self.isInState('closed'):
                    self.loop.call_soon(cb)
                else:
                    self.once('close', cb)
            self.emit('closeAsserted')
        self.loop.call_soon(go) if not self.loop.in_loop() else go()

    def _newSession(self):
        if not self.isInState('normal'):
            return
        s = ZKSession(self.session_timeout, self.log, self.collector,
                      self.loop, self.config)
        self.session = s

        def final_handler(st):
            if st == 'attached':
                self._emitAfterConnected('connect')
            elif st == 'detached':
                self.emit('disconnect')
            elif st == 'expired':
                self.emit('expire')

        def initial_handler(st):
            if st == 'attached':
                s.removeListener('stateChanged', initial_handler)
                s.on('stateChanged', final_handler)
                self._emitAfterConnected('session')
                self._emitAfterConnected('connect')
        s.on('stateChanged', initial_handler)

    def isConnected(self):
        conn = self.currentConnection()
        return conn is not None and conn.isInState('connected')

    is_connected = isConnected

    def _eventTrack(self, evt):
        if evt not in ('session', 'connect', 'failed'):
            return
        self.collector.getCollector(METRIC_ZK_EVENT_COUNTER).increment(
            {'evtype': evt})

    def _emitAfterConnected(self, evt):
        # Don't emit until list() etc. can safely be called
        # (client.js:237-262).
        c = self.currentConnection()
        if c is None:
            return
        if c.isInState('connected'):
            def later():
                self._eventTrack(evt)
                self.emit(evt)
            self.loop.call_soon(later)
        else:
            def on_conn_ch(cst):
                if cst == 'connected':
                    c.removeListener('stateChanged', on_conn_ch)
                    self._eventTrack(evt)
                    self.emit(evt)
            c.on('stateChanged', on_conn_ch)

    def getSession(self):
        if not self.isInState('normal'):
            return None
        if self.session.isInState('expired') or \
                self.session.isInState('closed'):
            self.old_session = self.session
            self._newSession()
        return self.session

    get_session = getSession

    def credentials(self):
        """Session credentials for resumption elsewhere (R3)."""
        return self.loop.run(lambda: self.session.credentials())

    def abandon(self):
        """Drop every connection WITHOUT closing the session on the server
        (a crash, or handing the session to another process that resumes it
        from :meth:`credentials`).  The client is unusable afterwards."""
        def go():
            self._resume_cred = None
            self.cset.stop()
            self.resolver.stop()
        self.loop.run(go)

    def _onSetAdded(self, key, conn, hdl):
        self.conns[key] = conn
        self.hdls[key] = hdl

    def _onSetRemoved(self, key):
        hdl = self.hdls.pop(key, None)
        conn = self.conns.pop(key, None)
        if conn is not None:
            conn.destroy()
        if hdl is not None:
            hdl.release()

    def _onSetStateChanged(self, st):
        if st == 'failed':
            def later():
                self._eventTrack('failed')
                self.emit('failed', Exception(
                    'Failed to connect to ZK (exhausted initial retry '
                    'policy)'))
            self.loop.call_soon(later)

    def _makeConnection(self, backend):
        c = ZKConnectionFSM(self, backend, self.log, self.loop, self.config,
                            tracer=self.tracer)
        c.connect()
        return c

    def currentConnection(self):
        sess = self.getSession()
        if sess is None:
            return None
        return sess.getConnection()

    # -- event registration is thread-safe enough under the GIL; events are
    # emitted on the loop thread.

    # -- data API ------------------------------------------------------------

    def _dispatch(self, fn, *args):
        if self.loop.in_loop():
            fn(*args)
        else:
            self._hop(fn, *args)

    def _hop(self, fn, *args):
        """Run ``fn(*args)`` on the loop thread, counted as a pending
        submission: while one is queued, requests from other threads do not
        go out directly (:meth:`_request`), so a later request never
        overtakes an earlier one from the same thread on the wire (a
        session's requests are FIFO, as on the reference's single loop)."""
        with self._hop_lock:
            self._hops += 1

        def run():
            try:
                fn(*args)
            finally:
                with self._hop_lock:
                    self._hops -= 1
        self.loop.call_soon(run)

    def _not_connected(self, cb):
        self.loop.call_soon(cb, ZKNotConnectedError())

    def _request(self, pkt, cb, on_reply):
        if self.loop.in_loop():
            self._issue(pkt, cb, on_reply)
            return
        if self.config.direct_send and self._hops == 0:
            # another thread: send from here when the live connection's
            # native router will settle the reply (request_direct) and no
            # earlier submission is still waiting for the loop
            sess = self.session
            conn = sess.conn if sess is not None and \
                self._fsm_state == 'normal' and \
                sess._fsm_state == 'attached' else None
            if conn is not None and conn.request_direct(
                    pkt, on_reply, lambda err, *_: cb(err)):
                return
        self._hop(self._issue, pkt, cb, on_reply)

    def _issue(self, pkt, cb, on_reply):
        # currentConnection() with the state checks inlined: this runs once
        # per data-API request
        sess = self.session
        if self._fsm_state != 'normal' or sess is None or \
                sess._fsm_state != 'attached':
            conn = self.currentConnection()
        else:
            conn = sess.conn
        if conn is None or conn._fsm_state != 'connected':
            self._not_connected(cb)
            return
        conn.request(pkt).then(on_reply, lambda err, *_: cb(err))

    def ping(self, cb):
        _check_func(cb)

        def go():
            conn = self.currentConnection()
            if conn is None or not conn.isInState('connected'):
                self._not_connected(cb)
                return
            conn.ping(lambda err=None, latency=None: cb(err))
        self._dispatch(go)

    def list(self, path, cb):
        _check_str(path, 'path')
        _check_func(cb)
        self._request({'opcode': 'GET_CHILDREN2', 'path': path,
                       'watch': False}, cb,
                      lambda pkt: cb(None, pkt['children'], pkt['stat']))

    def get(self, path, cb):
        if path.__class__ is not str or not callable(cb):
            _check_str(path, 'path')
            _check_func(cb)
        self._request({'opcode': 'GET_DATA', 'path': path, 'watch': False},
                      cb, lambda pkt: cb(None, pkt['data'], pkt['stat']))

    def create(self, path, data, options, cb):
        _check_str(path, 'path')
        _check_bytes(data, 'data')
        _check_func(cb)
        options = _norm_options(options)
        self._request({'opcode': 'CREATE', 'path': path, 'data': bytes(data),
                       'acl': options['acl'], 'flags': options['flags']},
                      cb, lambda pkt: cb(None, pkt['path']))

    def createWithEmptyParents(self, path, data, options, cb):
        """Create ``path`` and any missing parents (``client.js:412-481``).

        Parents are persistent nodes holding ``b'null'``; NODE_EXISTS on a
        parent is ignored; ``options`` apply to the final node only."""
        _check_str(path, 'path')
        _check_bytes(data, 'data')
        _check_func(cb)
        options = _norm_options(options)
        nodes = path.split('/')[1:]
        null = b'null'

        def go():
            conn = self.currentConnection()
            if conn is None or not conn.isInState('connected'):
                self._not_connected(cb)
                return
            state = {'i': 0, 'cur': '', 'last_path': None}

            def step():
                i = state['i']
                if i >= len(nodes):
                    cb(None, state['last_path'])
                    return
                state['cur'] = state['cur'] + '/' + nodes[i]
                last = (i == len(nodes) - 1)
                node_data = bytes(data) if last else null
                opts = options if last else {}

                def done(err, pkt_path=None):
                    if err is not None and (last or
                                            err.code != 'NODE_EXISTS'):
                        cb(err)
                        return
                    state['last_path'] = pkt_path
                    state['i'] += 1
                    step()
                self.create(state['cur'], node_data, opts, done)
            step()
        self._dispatch(go)

    create_with_empty_parents = createWithEmptyParents

    def set(self, path, data, version, cb):
        """``cb(err)``: the reference passes ``pkt.path`` which is always
        undefined for SET_DATA."""
        _check_str(path, 'path')
        _check_bytes(data, 'data')
        _check_int(version, 'version', optional=True)
        _check_func(cb)
        if version is None:
            version = -1
        self._request({'opcode': 'SET_DATA', 'path': path,
                       'data': bytes(data), 'version': version},
                      cb, lambda pkt: cb(None))

    def delete(self, path, version, cb):
        _check_str(path, 'path')
        _check_int(version, 'version')
        _check_func(cb)
        self._request({'opcode': 'DELETE', 'path': path, 'version': version},
                      cb, lambda pkt: cb(None))

    def stat(self, path, cb):
        _check_str(path, 'path')
        _check_func(cb)
        self._request({'opcode': 'EXISTS', 'path': path, 'watch': False},
                      cb, lambda pkt: cb(None, pkt['stat']))

    def getACL(self, path, cb):
        _check_str(path, 'path')
        _check_func(cb)
        self._request({'opcode': 'GET_ACL', 'path': path}, cb,
                      lambda pkt: cb(None, pkt['acl']))

    get_acl = getACL

    def sync(self, path, cb):
        _check_str(path, 'path')
        _check_func(cb)
        self._request({'opcode': 'SYNC', 'path': path}, cb,
                      lambda pkt: cb(None))

    # -- bulk (GPU-coded, pipelined) API (models/bulk.py) ---------------------

    BULK_OPS = ('GET_DATA', 'EXISTS', 'GET_CHILDREN', 'GET_CHILDREN2',
                'CREATE', 'SET_DATA', 'DELETE', 'SYNC', 'GET_ACL')

    def bulk(self, requests, cb):
        """Pipeline many requests as one batch on the current connection:
        encoded by K10 on the GPU, one socket write, replies collected by
        xid range and decoded by K1-K8 on the GPU.  ``requests`` are dicts
        ``{'opcode': 'GET_DATA', 'path': ...}`` (CREATE: ``data``, ``acl``,
        ``flags``; SET_DATA / DELETE: ``version``, default -1).  Watches are
        not supported here (use :meth:`watcher`).  ``cb(err, BulkResult)``;
        replies are in request order.  Not in the reference, whose requests
        go one by one through ``ZKEncodeStream`` (lib/zk-streams.js:109-148).
        """
        from .bulk import BulkBatch
        _check_func(cb)
        if not isinstance(requests, (list, tuple)):
            raise TypeError('requests ([object]) is required')
        pkts = []
        for r in requests:
            if not isinstance(r, dict) or r.get('opcode') not in self.BULK_OPS:
                raise ValueError('bulk request needs opcode in %r' %
                                 (self.BULK_OPS,))
            if 'path' in r:
                _check_str(r['path'], 'path')
            if r.get('watch'):
                raise ValueError('watches are not supported in bulk()')
            p = dict(r)
            op = p['opcode']
            p.setdefault('path', '')
            if op in ('GET_DATA', 'EXISTS', 'GET_CHILDREN', 'GET_CHILDREN2'):
                p['watch'] = False
            elif op == 'CREATE':
                o = _norm_options({'acl': p.get('acl'),
                                   'flags': p.get('flags')})
                p['acl'], p['flags'] = o['acl'], o['flags']
                p['data'] = bytes(p.get('data') or b'')
            elif op == 'SET_DATA':
                p['data'] = bytes(p.get('data') or b'')
                p['version'] = p.get('version', -1)
            elif op == 'DELETE':
                p['version'] = p.get('version', -1)
            pkts.append(p)

        def go():
            conn = self.currentConnection()
            if conn is None or not conn.isInState('connected'):
                self._not_connected(cb)
                return
            try:
                conn.bulk_submit(BulkBatch(pkts, self.bulk_device), cb)
            except Exception as e:
                self.loop.call_soon(cb, e)
        self._dispatch(go)

    def bulk_get(self, paths, cb, watch=False):
        """:meth:`bulk` of GET_DATA for every path: ``paths`` is a list of
        strings, or (GPU) a device ``(arena, off, len)`` triple of path
        bytes (uint8 / int64 / int32 tensors), packed straight into the
        request batch without per-request Python objects.  ``watch``: each
        read arms a data watch whose notification goes to the bulk watch
        sink (:meth:`watch_bulk`), not to a :meth:`watcher`."""
        from .bulk import BulkBatch
        _check_func(cb)
        if isinstance(paths, tuple) and len(paths) == 3 and \
                hasattr(paths[0], 'device'):
            from .bulk import _gpu_device
            if _gpu_device(self.bulk_device) is None:
                raise ValueError('bulk_get: a device (arena, off, len) '
                                 'triple needs a GPU bulk device')
            batch = BulkBatch.gets(paths, self.bulk_device, watch=watch)
        elif isinstance(paths, (list, tuple)):
            for p in paths:
                _check_str(p, 'path')
            batch = BulkBatch.gets(list(paths), self.bulk_device, watch=watch)
        else:
            raise TypeError('paths ([string]) is required')
        self._submit_bulk(batch, cb)

    def _submit_bulk(self, batch, cb):
        def go():
            conn = self.currentConnection()
            if conn is None or not conn.isInState('connected'):
                self._not_connected(cb)
                return
            try:
                conn.bulk_submit(batch, cb)
            except Exception as e:
                self.loop.call_soon(cb, e)
        self._dispatch(go)

    def bulk_set(self, paths, data, cb, version=-1):
        """:meth:`bulk` of SET_DATA of one ``data`` value at ``version`` to
        every path (strings, or a device ``(arena, off, len)`` triple),
        packed like :meth:`bulk_get` without per-request Python objects."""
        from .bulk import BulkBatch
        _check_func(cb)
        if not isinstance(data, (bytes, bytearray)):
            raise TypeError('data (bytes) is required')
        if isinstance(paths, tuple) and len(paths) == 3 and \
                hasattr(paths[0], 'device'):
            from .bulk import _gpu_device
            if _gpu_device(self.bulk_device) is None:
                raise ValueError('bulk_set: a device (arena, off, len) '
                                 'triple needs a GPU bulk device')
        elif isinstance(paths, (list, tuple)):
            for p in paths:
                _check_str(p, 'path')
            paths = list(paths)
        else:
            raise TypeError('paths ([string]) is required')
        batch = BulkBatch.sets(paths, data, self.bulk_device, version)
        self._submit_bulk(batch, cb)

    def watcher(self, path):
        _check_str(path, 'path')
        return self.loop.run(lambda: self.getSession().watcher(path))

    # -- bulk watches (the node-wide fan-out, zkmi/parallel/fanout.py) --------

    def watch_bulk(self, paths):
        """Data watches on ``paths`` kept in bulk, for the node-wide fan-out:
        from now on every connection keeps NOTIFICATION frames in its
        transport (the native loop's note sink; no Python object per event)
        for :meth:`take_notes`, and a session that moves re-arms these paths
        with SET_WATCHES at its last zxid like any watcher's.  Arm them with
        ``bulk_get(paths, cb, watch=True)``.  Not in the reference, whose
        watchers handle each notification on the event loop
        (lib/zk-session.js:853-854)."""
        for p in paths:
            _check_str(p, 'path')

        def go():
            self.note_capture = True
            self.getSession().add_bulk_watches(paths)
            conn = self.currentConnection()
            if conn is not None:
                conn.start_note_capture()
        self.loop.run(go)

    def take_notes(self):
        """(bytes, frames): the NOTIFICATION frames every connection of this
        client kept since the last call, in arrival order per connection
        (length prefixes included)."""
        def go():
            parts, n = [], 0
            for c in list(self.note_conns):
                b, k = c.take_notes()
                if k:
                    parts.append(b)
                    n += k
                if c.isInState('closed') or c.isInState('error'):
                    self.note_conns.discard(c)
            return b''.join(parts), n
        return self.loop.run(go)

    # -- blocking helpers -----------------------------------------------------

    def call_sync(self, method, *args, timeout=30.0):
        """Call ``method(*args, cb)`` and block for the callback.  Returns the
        callback's non-error arguments (a single value is unwrapped); raises
        the callback's error."""
        if self.loop.in_loop():
            raise RuntimeError('call_sync must not be used on the loop '
                               'thread')
        box = {}
        spin = self.config.sync_spin_us
        spin = (_SYNC_SPIN_US_AUTO if spin is None else spin) / 1e6
        mk = getattr(self.loop, 'waiter', None) if _SYNC_WAITER else None
        if mk is not None:
            # the native loop's Waiter: this thread waits in C with the GIL
            # released, and the loop flips the flag only after letting go of
            # the GIL — no GIL hand-over sleeps on the reply's way back
            w = mk()

            def cb(err=None, *res):
                if 'err' in box:
                    return      # settled already (one callback per call)
                box['err'] = err
                box['res'] = res
                w.set()
            getattr(self, method)(*args, cb)
            if not w.wait(spin, timeout):
                raise TimeoutError('%s%r timed out' % (method, args))
            return self._sync_result(box)
        # a bare lock, released by the loop thread: the cheapest cross-thread
        # wake-up CPython has (threading.Event adds a Condition round)
        done = threading.Lock()
        done.acquire()

        def cb(err=None, *res):
            if 'err' in box:
                return          # settled already (one callback per call)
            box['err'] = err
            box['res'] = res
            done.release()
        getattr(self, method)(*args, cb)
        got = False
        if spin > 0:
            # a short poll before sleeping on the lock: the reply usually
            # lands within tens of us, and a sleeping thread's wake-up costs
            # about that much again (ClientConfig.sync_spin_us)
            t_end = time.perf_counter() + spin
            while not got and time.perf_counter() < t_end:
                got = done.acquire(False)
                if not got:
                    time.sleep(0)
        if not got and not done.acquire(timeout=timeout):
            raise TimeoutError('%s%r timed out' % (method, args))
        return self._sync_result(box)

    @staticmethod
    def _sync_result(box):
        if box['err'] is not None:
            raise box['err']
        res = box['res']
        if len(res) == 0:
            return None
        if len(res) == 1:
            return res[0]
        return res

    def wait_connected(self, timeout=30.0):
        """Block until the client is connected (or raise TimeoutError)."""
        ev = threading.Event()

        def check():
            if self.isConnected():
                ev.set()
            else:
                self.once('connect', lambda *_: ev.set())
        self.loop.run(check)
        if not ev.wait(timeout):
            raise TimeoutError('client did not connect within %.1fs'
                               % timeout)
        return self

    def close_sync(self, timeout=30.0):
        ev = threading.Event()
        self.close(lambda *_: ev.set())
        if not ev.wait(timeout):
            raise TimeoutError('client did not close within %.1fs' % timeout)
