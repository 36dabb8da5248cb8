"""Backend resolution + connection pool with backoff — the re-provided
``cueball`` contract the client relies on.

The reference configures ``cueball.StaticIpResolver`` and
``cueball.ConnectionSet`` (``lib/client.js:88-118``) and reacts to
``added(key, conn, hdl)``, ``removed(key)`` and ``stateChanged('failed' |
'stopped')`` (``:275-299``).  This module implements that contract directly
rather than cloning cueball's slot FSMs:

* Backends are kept in a *preference order* (the given order, optionally
  shuffled).  Every ``decoherence_interval`` the order rotates, so the set
  opens a connection to the new favourite and — once it is usable — retires
  the old one; the session migrates with it (``zk-session.js:265-339``).
* At most one connection attempt is in flight; the set keeps ``target``
  usable connections and never more than ``maximum`` objects.
* A connection counts as usable when it emits ``'connect'`` (i.e. after the
  ZooKeeper handshake, ``connection-fsm.js:258-260``); an attempt that does
  not get there within ``connect_policy.timeout`` is destroyed.
* Failures back off per backend: ``delay * 2^(n-1)`` capped at
  ``max_delay``.  While no connection has ever been made, once every backend
  has failed more than ``retries`` times the set enters ``failed`` (the
  client's ``'failed'`` event, ``client.js:290-299``) and keeps retrying in
  monitor mode.
"""

import random

from ..runtime.emitter import EventEmitter


class StaticResolver(EventEmitter):
    """``cueball.StaticIpResolver`` equivalent: a fixed backend list."""

    def __init__(self, backends, default_port=2181):
        EventEmitter.__init__(self)
        self.backends = []
        for b in backends:
            self.backends.append({'address': b['address'],
                                  'port': b.get('port') or default_port})
        self.state = 'stopped'

    def _set(self, st):
        self.state = st
        self.emit('stateChanged', st)

    def isInState(self, st):
        return self.state == st

    def start(self):
        if self.state == 'running':
            return
        self._set('running')
        for b in self.backends:
            self.emit('added', '%s:%d' % (b['address'], b['port']), b)

    def stop(self):
        if self.state == 'stopped':
            return
        self._set('stopped')


class ConnectionHandle(object):

    def __init__(self, cset, key):
        self.cset = cset
        self.key = key
        self.released = False

    def release(self):
        self.released = True

    close = release


class _Backend(object):
    __slots__ = ('key', 'backend', 'failures', 'next_try', 'ever_ok')

    def __init__(self, key, backend):
        self.key = key
        self.backend = backend
        self.failures = 0
        self.next_try = 0.0
        self.ever_ok = False


class ConnectionSet(EventEmitter):

    def __init__(self, resolver, constructor, loop, log, config):
        EventEmitter.__init__(self)
        self.resolver = resolver
        self.constructor = constructor
        self.loop = loop
        self.log = log.child(component='ConnectionSet')
        self.cfg = config
        self.order = []                 # preference order of backend keys
        self.backends = {}
        self.conns = {}                 # key -> conn (attempting or usable)
        self.usable = set()             # keys whose conn emitted 'connect'
        self.pending = None             # key of the in-flight attempt
        self.state = 'starting'
        self.ever_connected = False
        self._timer = None
        self._decoh = None
        resolver.on('added', self._on_backend)

    # -- reference-compatible surface --------------------------------------

    def isInState(self, st):
        return self.state == st

    def getState(self):
        return self.state

    @property
    def cs_keys(self):
        return self.order

    @property
    def cs_backends(self):
        return {k: b.backend for k, b in self.backends.items()}

    def _set_state(self, st):
        if self.state == st:
            return
        self.state = st
        self.emit('stateChanged', st)

    def _on_backend(self, key, backend):
        if key in self.backends:
            return
        self.backends[key] = _Backend(key, backend)
        self.order.append(key)
        if self.cfg.shuffle_backends:
            random.shuffle(self.order)
        if self.state == 'starting':
            self._set_state('running')
            iv = self.cfg.decoherence_interval_s
            if iv and iv > 0:
                self._decoh = self.loop.call_later(iv * 1000.0,
                                                   self._decohere)
        self._kick()

    def stop(self):
        if self.state in ('stopped', 'stopping'):
            return
        self._cancel_timer()
        if self._decoh is not None:
            self._decoh.cancel()
            self._decoh = None
        self._set_state('stopping')

        # Asynchronous like cueball's stop(): the owner gets a turn to start
        # a clean CLOSE_SESSION before the connections are retired.
        def finish():
            for key in list(self.conns):
                self._drop(key)
            self._set_state('stopped')
        self.loop.call_soon(finish)

    # -- core -----------------------------------------------------------------

    def _now(self):
        return self.loop.time_ms()

    def _cancel_timer(self):
        if self._timer is not None:
            self._timer.cancel()
            self._timer = None

    def _kick(self):
        """Open a connection if we are below target and nothing is in
        flight."""
        if self.state not in ('running', 'failed'):
            return
        if self.pending is not None:
            return
        if len(self.usable) >= self.cfg.target:
            # Decoherence may want a more preferred backend.
            best = self.order[0] if self.order else None
            if best is None or best in self.usable or \
                    len(self.conns) >= self.cfg.maximum:
                return
            cand = [best] if self.backends[best].next_try <= self._now() \
                else []
        else:
            cand = [k for k in self.order if k not in self.conns]
        if not cand:
            return
        now = self._now()
        ready = [k for k in cand if self.backends[k].next_try <= now]
        if not ready:
            wake = min(self.backends[k].next_try for k in cand) - now
            self._cancel_timer()
            self._timer = self.loop.call_later(max(wake, 1), self._on_timer)
            return
        self._open(ready[0])

    def _on_timer(self):
        self._timer = None
        self._kick()

    def _open(self, key):
        b = self.backends[key]
        self.pending = key
        policy = self.cfg.connect_policy if not b.ever_ok else \
            self.cfg.default_policy
        conn = self.constructor(b.backend)
        self.conns[key] = conn
        box = {'done': False}

        def settle():
            if box['done']:
                return False
            box['done'] = True
            t.cancel()
            return True

        def on_connect():
            if not settle():
                return
            self.pending = None
            b.failures = 0
            b.ever_ok = True
            self.ever_connected = True
            self.usable.add(key)
            if self.state == 'failed':
                self._set_state('running')
            hdl = ConnectionHandle(self, key)
            self.emit('added', key, conn, hdl)
            self._trim()
            self._kick()

        def on_fail(*_):
            if key in self.usable:
                # A usable connection died: retry it at once, back off on
                # further failures.
                self.usable.discard(key)
                self.conns.pop(key, None)
                b.failures = 1
                b.next_try = self._now()
                self.emit('removed', key)
                self._kick()
                return
            if not settle():
                return
            if self.pending == key:
                self.pending = None
            self.conns.pop(key, None)
            conn.destroy()
            self._failed(b, policy)
            self._kick()

        def on_timeout():
            if box['done']:
                return
            self.log.debug('connect attempt to %s timed out', key)
            on_fail()

        t = self.loop.call_later(policy.timeout, on_timeout)
        conn.on('connect', on_connect)
        conn.on('error', on_fail)
        conn.on('close', on_fail)

    def _failed(self, b, policy):
        b.failures += 1
        delay = min(policy.delay * (2 ** (b.failures - 1)), policy.max_delay)
        b.next_try = self._now() + delay
        if not self.ever_connected and self.state == 'running':
            if all(x.failures > policy.retries
                   for x in self.backends.values()):
                self.log.warn('all backends failed their initial retry '
                              'policy')
                self._set_state('failed')

    def _drop(self, key):
        conn = self.conns.pop(key, None)
        if key == self.pending:
            self.pending = None
        if key in self.usable:
            self.usable.discard(key)
            self.emit('removed', key)
        elif conn is not None:
            conn.destroy()

    def _trim(self):
        """Retire usable connections beyond target, least preferred first."""
        extra = len(self.usable) - self.cfg.target
        if extra <= 0:
            return
        ranked = sorted(self.usable, key=self.order.index)
        for key in ranked[::-1][:extra]:
            self._drop(key)

    def _decohere(self):
        self._decoh = None
        if self.state not in ('running', 'failed'):
            return
        if len(self.order) > 1:
            self.order.append(self.order.pop(0))
            self.log.debug('decoherence: preferring %s', self.order[0])
            self._kick()
        self._decoh = self.loop.call_later(
            self.cfg.decoherence_interval_s * 1000.0, self._decohere)
