"""FSM runtime — the re-provided ``mooremachine`` contract.

Every state machine in the client (ZKClient, ZKConnectionFSM, ZKSession,
ZKWatchEvent, the ConnectionSet slots and the fake server) is written as
``state_<name>(self, S)`` methods.  ``S`` is a state handle; anything
registered through it (listeners, timers, immediates, callbacks) is torn
down automatically when the state is left, which is what makes the
reference's race fixes (e.g. #39, ``test/basic.test.js:1173-1174``) hold.

The runtime itself is native: each machine's transitions, handles, timers
and sub-states live in a ``_zkfsm.Core`` (csrc/host/zk_fsm.cpp).
:class:`PyCore` is the same contract in Python — the test oracle, and what
runs when the extension is not built or ``ZKMI_PY_FSM=1``.

Semantics implemented (inferred from the reference's use):
  * ``S.on(emitter, evt, cb)`` — auto-unsubscribed on state exit;
  * ``S.timeout(ms, cb)``, ``S.interval(ms, cb)``, ``S.immediate(cb)``;
  * ``S.callback(fn)`` — a wrapper that becomes a no-op after exit;
  * ``S.gotoState(name)`` — may be called synchronously inside a state
    function; transitions requested while one is in progress are queued and
    applied in order, and ``'stateChanged'`` is emitted *after* each state
    function has run (so listeners registered in the entry function see the
    FSM's next transitions);
  * sub-states ``'parent.child'`` (method ``state_parent__child``): entering a
    child keeps the parent's handles; ``isInState('parent')`` is true in the
    child; leaving to anything else (including re-entering the parent)
    disposes both;
  * a machine that defines ``_fsm_entered(state)`` gets it called after
    every transition (after ``stateChanged``).
"""

import operator
import os

from .emitter import EventEmitter

# the native runtime (csrc/host/zk_fsm.cpp)
try:
    from .. import _zkfsm
except ImportError:                  # not built: PyCore
    _zkfsm = None


def native():
    """True when new machines run on the native runtime."""
    return _zkfsm is not None and os.environ.get('ZKMI_PY_FSM', '') != '1'


class StateHandle(object):

    def __init__(self, core, state, loop):
        self._core = core
        self._state = state
        self._loop = loop
        self._disposers = []
        self._valid = True
        self._used = False

    # -- registration -------------------------------------------------------

    def on(self, emitter, evt, cb):
        if not self._valid:
            return
        emitter.on(evt, cb)
        self._disposers.append(lambda: emitter.removeListener(evt, cb))

    def timeout(self, ms, cb):
        h = self._loop.call_later(ms, self._guard(cb))
        self._disposers.append(h.cancel)
        return h

    def interval(self, ms, cb):
        box = {}
        guarded = self._guard(cb)

        def tick():
            if not self._valid:
                return
            box['h'] = self._loop.call_later(ms, tick)
            guarded()
        box['h'] = self._loop.call_later(ms, tick)

        class _Interval(object):
            def cancel(_self):
                box['h'].cancel()

            def unref(_self):
                return _self
        iv = _Interval()
        self._disposers.append(iv.cancel)
        return iv

    def immediate(self, cb):
        h = self._loop.call_soon(self._guard(cb))
        self._disposers.append(h.cancel)
        return h

    def callback(self, cb):
        return self._guard(cb)

    def _guard(self, cb):
        def g(*args):
            if self._valid:
                return cb(*args)
            return None
        return g

    # -- transitions ---------------------------------------------------------

    def gotoState(self, state):
        if not self._valid or self._used:
            raise AssertionError(
                'FSM %s: gotoState(%r) through a handle for state %r that '
                'was already left or used (now %r)' % (
                    type(self._core.owner).__name__, state, self._state,
                    self._core.state))
        self._used = True
        self._core.request(state)

    def _dispose(self):
        if not self._valid:
            return
        self._valid = False
        ds = self._disposers
        self._disposers = []
        for d in reversed(ds):
            d()


class PyCore(object):
    """One machine's runtime state in Python (see _zkfsm.Core)."""

    def __init__(self, owner, loop):
        self.owner = owner
        self.loop = loop
        self.state = None
        self._handles = []          # [(state_name, handle)] outer->inner
        self._busy = False
        self._queue = []
        self.history = []
        self._entered = getattr(owner, '_fsm_entered', None)

    def in_state(self, state):
        cur = self.state
        if cur is None:
            return False
        return cur == state or cur.startswith(state + '.')

    def handles(self):
        return list(self._handles)

    def request(self, state):
        self._queue.append(state)
        if self._busy:
            return
        self._busy = True
        try:
            while self._queue:
                nxt = self._queue.pop(0)
                self._enter(nxt)
        finally:
            self._busy = False

    def _enter(self, state):
        owner = self.owner
        fn = getattr(owner, 'state_' + state.replace('.', '__'), None)
        if fn is None:
            raise AssertionError('%s has no state %r' %
                                 (type(owner).__name__, state))
        # Keep handles of ancestors only when entering a strict descendant
        # of the current state (parent -> parent.child).
        cur = self.state
        keep = 0
        if cur is not None and state.startswith(cur + '.'):
            keep = len(self._handles)
            for _, h in self._handles:
                h._used = False     # the parent may transition again later
        for _, h in reversed(self._handles[keep:]):
            h._dispose()
        del self._handles[keep:]
        # Any handle of an abandoned level must not run gotoState again;
        # pending transitions requested through them are dropped above.
        self.state = state
        if len(self.history) > 64:
            del self.history[:32]
        self.history.append(state)
        h = StateHandle(self, state, self.loop)
        self._handles.append((state, h))
        fn(h)
        owner.emit('stateChanged', state)
        if self._entered is not None:
            self._entered(state)


class FSM(EventEmitter):
    """Base class; subclasses call ``FSM.__init__(self, initial, loop)``
    at the *end* of their constructor, like ``mod_fsm.FSM.call``."""

    def __init__(self, initial, loop):
        if not hasattr(self, '_listeners'):
            EventEmitter.__init__(self)
        self.fsm_loop = loop
        self._fsm_core = (_zkfsm.Core(self, loop) if native()
                          else PyCore(self, loop))
        self._fsm_core.request(initial)

    # (a C-level getter: read on every data-API request)
    _fsm_state = property(operator.attrgetter('_fsm_core.state'))

    @property
    def fsm_history(self):
        return self._fsm_core.history

    def getState(self):
        return self._fsm_core.state

    def isInState(self, state):
        return self._fsm_core.in_state(state)

    def allStateEvents(self):
        return [s for s in dir(self) if s.startswith('state_')]

    def _fsm_request(self, state):
        self._fsm_core.request(state)
