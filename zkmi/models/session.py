"""L5 — the (virtual) ZooKeeper session and the watch subsystem.

Parity:
  * ``ZKSession`` FSM — ``lib/zk-session.js:38-375``;
  * watch registry, notification dispatch, SET_WATCHES resume —
    ``:377-480``;
  * ``ZKWatcher`` per-path emitter — ``:527-614``;
  * ``ZKWatchEvent`` FSM (one server-side watch) — ``:616-1005``.

Design change: session expiry is a *deadline* (``last_rx + timeout``)
checked by one lazily re-armed timer, instead of a ``clearTimeout`` +
``setTimeout`` pair on every received packet (``zk-session.js:99-108``;
SURVEY §7.1 "Expiry is a deadline, not a timer per packet").
"""

import operator
import os
import random
import re
import threading
import time

from .. import jute
from ..runtime.emitter import EventEmitter

try:
    from .. import _zkwatch
except ImportError:                      # not built: the Python FSMs
    _zkwatch = None

from ..runtime import fsm as _fsm
from ..runtime.fsm import FSM
from ..utils.metrics import METRIC_ZK_NOTIFICATION_COUNTER


def _load_machines():
    """The native machines (csrc/host/zk_machines.cpp): the in-tree
    extension, or the one at ``ZKMI_MACHINES_PATH`` (the sanitizer build,
    tools/sanitize_host.sh); None when not built (the Python FSMs)."""
    path = os.environ.get('ZKMI_MACHINES_PATH')
    if path:
        import importlib.util
        spec = importlib.util.spec_from_file_location('_zkmach', path)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        return mod
    try:
        from .. import _zkmach as mod
    except ImportError:
        return None
    return mod


_zkmach = _load_machines()


class ExpiryTimer(EventEmitter):
    """Emits ``'timeout'`` once ``now - last_reset >= timeout``."""

    def __init__(self, loop):
        EventEmitter.__init__(self)
        self.loop = loop
        self.deadline = None
        self.timeout_ms = None
        self._h = None
        # () -> ms (loop clock) of the last reply the connection's native
        # router settled, or None: those replies reset the timer lazily,
        # here, instead of one reset() each
        self.probe = None

    def reset(self, timeout_ms):
        now = self.loop.time_ms()
        shorter = self.timeout_ms is not None and timeout_ms < self.timeout_ms
        self.timeout_ms = timeout_ms
        self.deadline = now + timeout_ms
        if self._h is not None and shorter:
            # a shorter negotiated timeout (a reattach to another server):
            # the pending wake-up would fire late, re-arm it
            # (lib/zk-session.js:99-108 clears and re-sets on every reset)
            self._h.cancel()
            self._h = None
        if self._h is None:
            self._h = self.loop.call_later(timeout_ms, self._fire)

    def _fire(self):
        self._h = None
        if self.deadline is None:
            return
        if self.probe is not None:
            last = self.probe()
            if last is not None and last + self.timeout_ms > self.deadline:
                self.deadline = last + self.timeout_ms
        rem = self.deadline - self.loop.time_ms()
        if rem > 0.5:
            self._h = self.loop.call_later(rem, self._fire)
            return
        self.deadline = None
        self.emit('timeout')

    def cancel(self):
        self.deadline = None
        if self._h is not None:
            self._h.cancel()
            self._h = None


_CAMEL = {}


def _camel(evt_type):
    """``DATA_CHANGED`` -> ``dataChanged`` (``zk-session.js:401``);
    memoised (one lookup per notification)."""
    c = _CAMEL.get(evt_type)
    if c is None:
        c = _CAMEL[evt_type] = re.sub(r'_[a-z]',
                                      lambda m: m.group(0)[1].upper(),
                                      evt_type.lower())
    return c


def native_machines():
    """True when new sessions / connections / clients run on the C++
    machines (csrc/host/zk_machines.cpp); ``ZKMI_PY_FSM=1`` selects the
    Python state functions below, kept as the test oracle."""
    return _zkmach is not None and _fsm.native()


def ZKSession(timeout, log, collector, loop, config):
    """The session: the native machine, or the Python oracle."""
    cls = NativeZKSession if native_machines() else PyZKSession
    return cls(timeout, log, collector, loop, config)


class _SessionBase(object):
    """What the session is besides its state graph: credentials, liveness,
    the watch registry and dispatch, SET_WATCHES resume."""

    def __init__(self, timeout, log, collector, loop, config):
        self.conn = None
        self.old_conn = None
        self.last_pkt = None              # monotonic seconds of last rx
        self.expiry = ExpiryTimer(loop)
        self.watchers = {}
        self.timeout = timeout
        self.log = log.child(component='ZKSession')
        self.collector = collector
        self.config = config
        self.last_attach = 0
        self._last_zxid = 0
        self.expiry.probe = self._routed_last_rx
        # paths with bulk data watches (Client.watch_bulk): re-armed on a
        # move like the watchers' (their notifications go to the fan-out)
        self.bulk_watches = set()
        self._bulk_packed = None    # bulk_watches as an encoded vector
                                    # (in the order they were added)
        self.rearmed = 0            # watches re-armed by SET_WATCHES resumes
        self.resumes = []           # (relZxid, watches) of each resume
        self.session_id = 0
        self.passwd = b'\0' * 8
        collector.counter(METRIC_ZK_NOTIFICATION_COUNTER,
                          'Notifications received from ZooKeeper')
        # the watch events: the native engine (one table, the Python side
        # keeps only the listeners) or one ZKWatchEvent FSM per (path, event)
        self.wt = None
        if _zkwatch is not None and getattr(config, 'native_watch', True):
            self.wt = _zkwatch.WatchTable(self._wt_emit, loop,
                                          float(config.doublecheck_ms),
                                          float(config.doublecheck_rand_ms))

    def _fsm_entered(self, state):
        # after every transition (the FSM runtime's hook)
        if self.wt is not None:
            self._wt_sync()

    # -- queries --------------------------------------------------------------

    def isAttaching(self):
        return self.isInState('attaching') or self.isInState('reattaching')

    def isAlive(self):
        last = self.last_pkt
        rx = self._routed_last_rx()
        if rx is not None and (last is None or rx / 1e3 > last):
            last = rx / 1e3
        if last is None:
            return False
        return (time.monotonic() - last) * 1000.0 < self.timeout

    # -- replies settled by the connection's native router ------------------
    # (ZKConnectionFSM.route_state): they carry zxids and keep the session
    # alive like the packets on_packet sees, but are folded in only when
    # read (lastZxidSeen, expiry, isAlive), or when the router stops.

    def _routed(self):
        for c in (self.conn, self.old_conn):
            if c is not None and c.routing:
                yield c.route_state()

    def _routed_last_rx(self):
        last = None
        for _, rx in self._routed():
            if rx > 0 and (last is None or rx > last):
                last = rx
        return last

    @property
    def last_zxid(self):
        z = self._last_zxid
        for rz, _ in self._routed():
            if rz > z:
                z = rz
        return z

    @last_zxid.setter
    def last_zxid(self, z):
        self._last_zxid = z

    def fold_routed(self, zxid, last_rx_ms):
        """A connection's router stopped: keep what it saw."""
        if zxid > self._last_zxid:
            self._last_zxid = zxid
        if last_rx_ms > 0:
            t = last_rx_ms / 1e3
            if self.last_pkt is None or t > self.last_pkt:
                self.last_pkt = t
            ex = self.expiry
            if ex.deadline is not None and ex.timeout_ms is not None and \
                    last_rx_ms + ex.timeout_ms > ex.deadline:
                ex.deadline = last_rx_ms + ex.timeout_ms

    def resetExpiryTimer(self):
        self.last_pkt = time.monotonic()
        self.expiry.reset(self.timeout)

    def getTimeout(self):
        return self.timeout

    def getConnection(self):
        if not self.isInState('attached'):
            return None
        return self.conn

    def getSessionId(self):
        return '%016x' % (self.session_id & 0xffffffffffffffff)

    def credentials(self):
        """What a peer (or a restarted process) needs to resume this session:
        ``sessionId``, ``passwd``, ``lastZxid``, ``timeout`` (SURVEY §5
        checkpoint/resume; shared across GPU ranks by R3)."""
        return {'sessionId': self.session_id, 'passwd': bytes(self.passwd),
                'lastZxid': self.last_zxid, 'timeout': self.timeout}

    def adopt_credentials(self, cred):
        """Resume an existing session on the next attach (must be detached)."""
        assert self.isInState('detached')
        self.session_id = cred['sessionId']
        self.passwd = bytes(cred['passwd'])
        self.last_zxid = cred.get('lastZxid', 0)
        self.timeout = cred.get('timeout', self.timeout)
        self.last_pkt = time.monotonic()

    def _connect_request(self):
        return {'protocolVersion': 0, 'lastZxidSeen': self.last_zxid,
                'timeOut': self.timeout, 'sessionId': self.session_id,
                'passwd': self.passwd}

    # -- watches --------------------------------------------------------------

    def watchersDisconnected(self):
        if self.wt is not None:
            self.wt.disconnected()
        for w in list(self.watchers.values()):
            for ev in w.events():
                ev.disconnected()

    def _wt_emit(self, path, evt, *args):
        """The native engine's user-visible events, to the path's
        ZKWatcher listeners."""
        w = self.watchers.get(path)
        if w is not None:
            EventEmitter.emit(w, evt, *args)

    def _wt_sync(self):
        """Tell the native engine whether watch requests can go out: the
        session attached and its connection connected (the reference's
        wait_session / wait_connected)."""
        wt = self.wt
        conn = self.conn
        if self.isInState('attached') and conn is not None and \
                conn.isInState('connected'):
            wt.ready(conn)
        else:
            wt.unready()

    def processNotification(self, pkt):
        if pkt['state'] != 'SYNC_CONNECTED':
            self.log.warn({'xid': pkt['xid'], 'state': pkt['state'],
                           'type': pkt['type']},
                          'received notification with bad state %s',
                          pkt['state'])
            return
        watcher = self.watchers.get(pkt['path'])
        evt = _camel(pkt['type'])
        self.log.trace({'zxid': pkt['zxid'], 'type': pkt['type']},
                       'notification %s for %s', evt, pkt['path'])
        self.collector.getCollector(METRIC_ZK_NOTIFICATION_COUNTER) \
            .increment({'event': evt})
        if watcher is not None:
            watcher.notify(evt)

    def resumeWatches(self):
        events = {'dataChanged': [], 'createdOrDestroyed': [],
                  'childrenChanged': []}
        count = 0
        all_evts = []
        for path, w in list(self.watchers.items()):
            cod = False
            for ev in w.events():
                if isinstance(ev, _NativeWatchEvent) or \
                        not ev.isInState('resuming'):
                    continue               # (the engine's: resume_lists)
                e = ev.getEvent()
                if e == 'createdOrDeleted':
                    if cod:
                        continue
                    events['createdOrDestroyed'].append(path)
                    cod = True
                elif e == 'dataChanged':
                    events['dataChanged'].append(path)
                elif e == 'childrenChanged':
                    events['childrenChanged'].append(path)
                else:
                    raise AssertionError('unknown event: ' + e)
                count += 1
                all_evts.append(ev)
        batch = None
        if self.wt is not None:
            batch, dw, ew, cw = self.wt.resume_lists()
            events['dataChanged'] += dw
            events['createdOrDestroyed'] += ew
            events['childrenChanged'] += cw
            count += len(dw) + len(ew) + len(cw)
        if self.bulk_watches:
            events['dataChanged'] = events['dataChanged'] + self._bulk_packed
            count += self._bulk_packed.n
        if count < 1:
            return
        zxid = self.last_zxid
        self.log.info('re-arming %d node watchers at zxid %x', count, zxid)
        self.rearmed += count
        if len(self.resumes) < 64:
            self.resumes.append((zxid, count))

        def done(err):
            if err is not None:
                # The reference emits 'pingTimeout' on the session here,
                # which nothing listens to.  The events
                # stay in 'resuming' and are re-sent on the next attach.
                self.log.warn(err, 'SET_WATCHES failed; will retry on '
                              'next attach')
                return
            for ev in all_evts:
                ev.resume()
            if batch is not None:
                self.wt.resumed(batch)
        self.conn.setWatches(events, zxid, done)

    def add_bulk_watches(self, paths):
        """Paths watched in bulk (:meth:`~zkmi.models.client.Client.
        watch_bulk`): every resume re-arms them with the session's other
        watches."""
        new = [p for p in dict.fromkeys(paths) if p not in self.bulk_watches]
        if not new:
            return
        self.bulk_watches.update(new)
        self._bulk_packed = (self._bulk_packed or jute.PackedStrings()) + new

    def watcher(self, path):
        w = self.watchers.get(path)
        if w is None:
            w = ZKWatcher(self, path, self.log)
            self.watchers[path] = w
        return w


class PyZKSession(_SessionBase, FSM):
    """The session's state graph as mooremachine-style state functions
    (``lib/zk-session.js:38-375``): the test oracle of the native machine
    (``ZKMI_PY_FSM=1``)."""

    def __init__(self, timeout, log, collector, loop, config):
        _SessionBase.__init__(self, timeout, log, collector, loop, config)
        FSM.__init__(self, 'detached', loop)

    def attachAndSendCR(self, conn):
        if not self.isInState('detached') and not self.isInState('attached'):
            raise Exception('ZKSession#attachAndSendCR may only be called in '
                            'state "attached" or "detached" (is in %s)'
                            % self.getState())
        self.emit('assertAttach', conn)

    def close(self):
        self.emit('closeAsserted')

    # -- states ---------------------------------------------------------------

    def state_detached(self, S):
        if self.conn is not None:
            self.conn.destroy()
        self.conn = None

        def on_attach(conn):
            self.conn = conn
            S.gotoState('attaching')
        S.on(self, 'assertAttach', on_attach)
        S.on(self, 'closeAsserted', lambda: S.gotoState('closed'))
        S.on(self.expiry, 'timeout', lambda: S.gotoState('expired'))
        self.watchersDisconnected()

    def state_attaching(self, S):
        def on_error(*_):
            if self.isAlive():
                S.gotoState('detached')
            elif self.session_id != 0:
                S.gotoState('expired')
            else:
                S.gotoState('detached')

        S.on(self.conn, 'error', on_error)
        # Can happen separately from 'error' when the set times out the
        # connect attempt (zk-session.js:159-163).
        S.on(self.conn, 'close', on_error)

        def on_packet(pkt):
            sid = pkt['sessionId']
            if sid == 0:
                S.gotoState('expired')
                return
            verb = 'resumed' if self.session_id != 0 else 'created'
            self.log.info('%s zookeeper session %016x with timeout %d ms',
                          verb, sid & 0xffffffffffffffff, pkt['timeOut'])
            self.log = self.log.child(id='%016x' % (sid & 0xffffffffffffffff))
            self.timeout = pkt['timeOut']
            self.session_id = sid
            self.passwd = pkt['passwd']
            self.resetExpiryTimer()
            S.gotoState('attached')
        S.on(self.conn, 'packet', on_packet)
        S.on(self.expiry, 'timeout', lambda: S.gotoState('expired'))
        S.on(self, 'closeAsserted', lambda: S.gotoState('closing'))
        self.conn.send(self._connect_request())

    def state_attached(self, S):
        self.last_attach = time.time()
        conn = self.conn

        def on_lost(*_):
            if self.isAlive():
                S.gotoState('detached')
            else:
                S.gotoState('expired')
        S.on(conn, 'close', on_lost)
        S.on(conn, 'error', on_lost)

        def on_packet(pkt):
            self.resetExpiryTimer()
            if pkt['opcode'] != 'NOTIFICATION':
                z = pkt['zxid']
                if z > self._last_zxid:
                    self._last_zxid = z
                return
            self.processNotification(pkt)
        S.on(conn, 'packet', on_packet)
        S.on(self.expiry, 'timeout', lambda: S.gotoState('expired'))
        S.on(self, 'closeAsserted', lambda: S.gotoState('closing'))

        def on_conn_state(st):
            if st == 'connected':
                if self.old_conn is not None:
                    self.old_conn.destroy()
                    self.old_conn = None
                self.resumeWatches()
            if self.wt is not None:
                self._wt_sync()          # (after the SET_WATCHES)
        S.on(conn, 'stateChanged', on_conn_state)

        def on_attach(newconn):
            self.old_conn = self.conn
            self.conn = newconn
            S.gotoState('reattaching')
        S.on(self, 'assertAttach', on_attach)

    def state_reattaching(self, S):
        cur_sid = self.session_id
        assert self.old_conn is not None, 'reattaching requires oldConn'
        old = self.old_conn
        new = self.conn

        def revert(*_):
            if self.isAlive() and old.isInState('connected'):
                self.log.warn('reverted move of session %016x (on %s:%d) to '
                              'new backend (%s:%d)',
                              cur_sid & 0xffffffffffffffff,
                              old.server['address'], old.server['port'],
                              new.server['address'], new.server['port'])
                self.conn = old
                self.old_conn = None
                S.gotoState('attached')
            elif self.isAlive():
                old.destroy()
                S.gotoState('detached')
            else:
                old.close()
                S.gotoState('expired')

        def on_packet(pkt):
            sid = pkt['sessionId']
            if sid == 0:
                revert()
                return
            # The old connection is torn down once the new one reaches
            # 'connected' (state_attached's stateChanged handler).
            self.log.info('moved zookeeper session %016x to more preferred '
                          'backend (%s:%d) with timeout %d ms',
                          sid & 0xffffffffffffffff, new.server['address'],
                          new.server['port'], pkt['timeOut'])
            self.timeout = pkt['timeOut']
            self.session_id = sid
            self.passwd = pkt['passwd']
            self.resetExpiryTimer()
            self.watchersDisconnected()
            S.gotoState('attached')

        S.on(new, 'packet', on_packet)
        S.on(new, 'error', revert)
        S.on(new, 'close', revert)
        S.on(self.expiry, 'timeout', revert)

        def on_close():
            old.close()
            S.gotoState('closing')
        S.on(self, 'closeAsserted', on_close)
        self.log.debug('attempting to move zookeeper session %016x from '
                       '%s:%d to %s:%d', cur_sid & 0xffffffffffffffff,
                       old.server['address'], old.server['port'],
                       new.server['address'], new.server['port'])
        new.send(self._connect_request())

    def state_closing(self, S):
        S.on(self.conn, 'error', lambda *_: S.gotoState('closed'))
        S.on(self.conn, 'close', lambda *_: S.gotoState('closed'))
        S.on(self.expiry, 'timeout', lambda: S.gotoState('closed'))
        self.conn.close()

    def state_expired(self, S):
        if self.conn is not None:
            self.conn.destroy()
        self.conn = None
        self.expiry.cancel()
        if self.wt is not None:
            self.wt.close()       # its watches are dead: no more timers
        self.log.warn('ZK session expired')

    def state_closed(self, S):
        if self.conn is not None:
            self.conn.destroy()
        self.conn = None
        self.expiry.cancel()
        if self.wt is not None:
            self.wt.close()
        self.log.info('ZK session closed')


class NativeZKSession(_SessionBase, EventEmitter):
    """The session on the C++ machine (``_zkmach.Machine('session')``,
    csrc/host/zk_machines.cpp): its transitions, guards and entry actions
    run there; this object keeps the API, the listener surface and the
    watch registry."""

    def __init__(self, timeout, log, collector, loop, config):
        EventEmitter.__init__(self)
        _SessionBase.__init__(self, timeout, log, collector, loop, config)
        self.fsm_loop = loop
        self._m = _zkmach.Machine('session', self, loop)
        self._m.watch(self.expiry, 'timeout', _zkmach.SE_EXPIRY)
        self._m.start('detached')

    def getState(self):
        return self._m.state

    _fsm_state = property(operator.attrgetter('_m.state'))

    def isInState(self, state):
        return self._m.in_state(state)

    @property
    def fsm_history(self):
        return self._m.history

    def attachAndSendCR(self, conn):
        if not self.isInState('detached') and not self.isInState('attached'):
            raise Exception('ZKSession#attachAndSendCR may only be called in '
                            'state "attached" or "detached" (is in %s)'
                            % self.getState())
        self._m.fire(_zkmach.SE_ATTACH, conn)

    def close(self):
        self._m.fire(_zkmach.SE_CLOSE)


class ZKWatcher(EventEmitter):
    """User-facing per-path emitter (``zk-session.js:527-614``).

    Events: ``created(stat)``, ``deleted()``, ``dataChanged(data, stat)``,
    ``childrenChanged(children, stat)``.  The first listener for an event
    arms the corresponding server watch; ``created``/``deleted`` share one
    existence watch."""

    _NOTIFY = {
        'created': ('createdOrDeleted', 'dataChanged'),
        'deleted': ('createdOrDeleted', 'dataChanged', 'childrenChanged'),
        'dataChanged': ('dataChanged', 'createdOrDeleted'),
        'childrenChanged': ('childrenChanged',),
    }

    def __init__(self, session, path, log):
        EventEmitter.__init__(self)
        self._lk = threading.Lock()
        self.path = path
        self.session = session
        self.evts = {}
        self.log = log.child(component='ZKWatcher', path=path)

    def events(self):
        return [self.evts[k] for k in ('createdOrDeleted', 'dataChanged',
                                       'childrenChanged') if k in self.evts]

    def once(self, *a):
        raise Exception('ZKWatcher does not support once() (use on)')

    def notify(self, evt):
        wt = self.session.wt
        if wt is not None and wt.has(self.path):
            wt.notify(self.path, evt)
            return
        types = self._NOTIFY.get(evt)
        if types is None:
            raise Exception('Unknown notification type: ' + evt)
        notified = False
        for t in types:
            ev = self.evts.get(t)
            if ev is not None and not ev.isInState('disarmed'):
                ev.notify()
                notified = True
        if not notified:
            # Our picture of which ZK events hit which watches is wrong; we
            # cannot guarantee a working watcher, so fail loudly
            # (zk-session.js:584-592).
            raise Exception('Got notification for %s but have no matching '
                            'events on %s' % (evt, self.path))

    def on(self, evt, cb):
        if not isinstance(evt, str):
            raise TypeError('event must be a string')
        if not callable(cb):
            raise TypeError('callback must be a function')
        # The listener is registered right here, in the caller's thread, so
        # several on() calls in a row are all in place before any reply to
        # the arming they trigger can be dispatched (the reference registers
        # synchronously within one tick).  Arming drives FSMs, which live on
        # the loop thread only: it is queued there.
        with self._lk:
            first = self.listenerCount(evt) < 1
            EventEmitter.on(self, evt, cb)
        if evt != 'error' and first:
            loop = self.session.fsm_loop
            if loop.in_loop():
                self._armEvent(evt)
            else:
                loop.call_soon(self._armEvent, evt)
        return self

    def removeListener(self, evt, cb):
        with self._lk:
            return EventEmitter.removeListener(self, evt, cb)

    addListener = on

    def _armEvent(self, evt):
        if evt in ('deleted', 'created'):
            evt = 'createdOrDeleted'
        if evt not in ('createdOrDeleted', 'dataChanged', 'childrenChanged'):
            return
        wt = self.session.wt
        if wt is not None:
            if evt not in self.evts:
                self.evts[evt] = _NativeWatchEvent(wt, self.path, evt)
            wt.arm(self.path, evt)
            return
        ev = self.evts.get(evt)
        if ev is None:
            ev = ZKWatchEvent(self.session, self.path, self, evt, self.log)
            self.evts[evt] = ev
        if ev.isInState('disarmed'):
            ev.arm()


class _NativeWatchEvent(object):
    """A watch event held by the native engine: the ZKWatchEvent queries
    (state, history) read from its table."""

    def __init__(self, wt, path, evt):
        self.wt = wt
        self.path = path
        self.evt = evt

    def getEvent(self):
        return self.evt

    def getState(self):
        return self.wt.state(self.path, self.evt)

    def isInState(self, st):
        cur = self.getState() or ''
        return cur == st or cur.startswith(st + '.')

    @property
    def fsm_history(self):
        return self.wt.history(self.path, self.evt)

    # (the session drives the engine as a whole: these are no-ops here)
    def disconnected(self):
        pass

    def resume(self):
        pass


class ZKWatchEvent(FSM):
    """One server-side watch (``zk-session.js:616-1005``)::

        disarmed -> wait_session -> wait_connected -> arming -> armed
                        ^   ^              |             |  \\-> wait_node
                        |   \\______________/             |        |
                        \\____________ (notify) _________armed      |
                        \\__________________________________________/
        armed -> resuming (disconnect) -> armed (SET_WATCHES ok)
        armed -> armed.doublecheck (4h + U(0,8h)) -> armed
    """

    def __init__(self, session, path, emitter, evt, log):
        self.path = path
        self.session = session
        self.emitter = emitter
        self.evt = evt
        self.prev_zxid = None
        self.log = log.child(event=evt)
        FSM.__init__(self, 'disarmed', session.fsm_loop)

    def getEvent(self):
        return self.evt

    def arm(self):
        self.emit('armAsserted')

    def notify(self):
        if self.isInState('armed') or self.isInState('resuming'):
            self.emit('notifyAsserted')

    def disconnected(self):
        if self.isInState('armed'):
            self.emit('disconnectAsserted')

    def resume(self):
        if self.isInState('resuming'):
            self.emit('resumeAsserted')

    def state_disarmed(self, S):
        def on_arm():
            self.log.trace('arming watcher')
            S.gotoState('wait_session')
        S.on(self, 'armAsserted', on_arm)

    def state_wait_session(self, S):
        if self.session.isInState('attached'):
            S.gotoState('wait_connected')
            return

        def on_state(st):
            if st == 'attached':
                S.gotoState('wait_connected')
        S.on(self.session, 'stateChanged', on_state)
        self.log.trace('deferring watcher arm until after reconnect')

    def state_wait_connected(self, S):
        conn = self.session.getConnection()
        if conn is None or not conn.isInState('connected'):
            # Not synchronously: give the connection a turn of the loop to
            # reach 'connected' (zk-session.js:780-791).
            S.immediate(lambda: S.gotoState('wait_session'))
            return
        S.gotoState('arming')

    def _packet(self):
        op = {'createdOrDeleted': 'EXISTS', 'dataChanged': 'GET_DATA',
              'childrenChanged': 'GET_CHILDREN2'}[self.evt]
        return {'opcode': op, 'path': self.path, 'watch': True}

    toPacket = _packet

    def state_arming(self, S):
        conn = self.session.getConnection()
        req = conn.request(self._packet())
        evt = self.evt

        def on_reply(pkt):
            stat = pkt['stat']
            if evt == 'createdOrDeleted':
                zxid = stat.czxid
                args = ('created', stat)
            elif evt == 'dataChanged':
                zxid = stat.mzxid
                args = ('dataChanged', pkt['data'], stat)
            else:
                zxid = stat.pzxid
                args = ('childrenChanged', pkt['children'], stat)
            self.log.trace({'zxid': zxid, 'prevZxid': self.prev_zxid},
                           'got reply to arm request')
            if self.prev_zxid is not None and zxid == self.prev_zxid:
                S.gotoState('armed')
                return
            EventEmitter.emit(self.emitter, *args)
            self.prev_zxid = zxid
            S.gotoState('armed')

        def on_error(err, *_):
            code = getattr(err, 'code', None)
            if code == 'PING_TIMEOUT':
                S.gotoState('wait_session')
                return
            if evt == 'createdOrDeleted' and code == 'NO_NODE':
                # Existence watches arm on a missing node.
                EventEmitter.emit(self.emitter, 'deleted')
                S.gotoState('armed')
                return
            if code == 'NO_NODE':
                S.gotoState('wait_node')
                return
            self.log.trace(err, 'watcher attach failure; will retry')
            S.gotoState('wait_session')
        S.on(req, 'reply', on_reply)
        S.on(req, 'error', on_error)

    def state_wait_node(self, S):
        # Subscribing to 'created' implicitly arms an existence watch through
        # ZKWatcher.on (zk-session.js:891 -> :595-603).
        S.on(self.emitter, 'created', lambda *_: S.gotoState('wait_session'))

    def state_armed(self, S):
        S.on(self, 'notifyAsserted', lambda: S.gotoState('wait_session'))
        S.on(self, 'disconnectAsserted', lambda: S.gotoState('resuming'))
        cfg = self.session.config
        ms = round(cfg.doublecheck_ms + random.random() *
                   cfg.doublecheck_rand_ms)
        S.timeout(ms, lambda: S.gotoState('armed.doublecheck')).unref()

    def state_armed__doublecheck(self, S):
        if not self.session.isInState('attached'):
            S.gotoState('armed')
            return
        conn = self.session.getConnection()
        if conn is None or not conn.isInState('connected'):
            S.gotoState('armed')
            return
        req = conn.request({'path': self.path, 'opcode': 'EXISTS',
                            'watch': False})
        evt = self.evt

        def on_reply(pkt):
            stat = pkt['stat']
            zxid = {'createdOrDeleted': stat.czxid,
                    'dataChanged': stat.mzxid,
                    'childrenChanged': stat.pzxid}[evt]
            self.log.trace({'zxid': zxid, 'prevZxid': self.prev_zxid},
                           'got reply to doublecheck request')
            if self.prev_zxid is None or zxid != self.prev_zxid:
                raise Exception('ZKWatchEvent double-check failed: zkmi has '
                                'missed a ZK event wakeup, this is a bug')
            S.gotoState('armed')
        S.on(req, 'reply', on_reply)
        S.on(req, 'error', lambda *_: S.gotoState('armed'))

    def state_resuming(self, S):
        S.on(self, 'resumeAsserted', lambda: S.gotoState('armed'))
        S.on(self, 'notifyAsserted', lambda: S.gotoState('wait_session'))
