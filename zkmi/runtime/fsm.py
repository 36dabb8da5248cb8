"""FSM runtime — the re-provided ``mooremachine`` contract.

Every state machine in the client (ZKClient, ZKConnectionFSM, ZKSession,
ZKWatchEvent, the ConnectionSet slots and the fake server) is written as
``state_<name>(self, S)`` methods.  ``S`` is a :class:`StateHandle`; anything
registered through it (listeners, timers, immediates, callbacks) is torn
down automatically when the state is left, which is what makes the
reference's race fixes (e.g. #39, ``test/basic.test.js:1173-1174``) hold.

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
    disposes both.
"""

from .emitter import EventEmitter


class StateHandle(object):

    def __init__(self, fsm, state, loop):
        self._fsm = fsm
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
                    type(self._fsm).__name__, state, self._state,
                    self._fsm.getState()))
        self._used = True
        self._fsm._fsm_request(state)

    def _dispose(self):
        if not self._valid:
            return
        self._valid = False
        ds = self._disposers
        self._disposers = []
        for d in reversed(ds):
            d()


class FSM(EventEmitter):
    """Base class; subclasses call ``FSM.__init__(self, initial, loop)``
    at the *end* of their constructor, like ``mod_fsm.FSM.call``."""

    def __init__(self, initial, loop):
        if not hasattr(self, '_listeners'):
            EventEmitter.__init__(self)
        self.fsm_loop = loop
        self._fsm_state = None
        self._fsm_handles = []          # [(state_name, handle)] outer->inner
        self._fsm_busy = False
        self._fsm_queue = []
        self.fsm_history = []
        self._fsm_request(initial)

    def getState(self):
        return self._fsm_state

    def isInState(self, state):
        cur = self._fsm_state
        if cur is None:
            return False
        return cur == state or cur.startswith(state + '.')

    def allStateEvents(self):
        return [s for s in dir(self) if s.startswith('state_')]

    def _fsm_request(self, state):
        self._fsm_queue.append(state)
        if self._fsm_busy:
            return
        self._fsm_busy = True
        try:
            while self._fsm_queue:
                nxt = self._fsm_queue.pop(0)
                self._fsm_enter(nxt)
        finally:
            self._fsm_busy = False

    def _fsm_enter(self, state):
        fn = getattr(self, 'state_' + state.replace('.', '__'), None)
        if fn is None:
            raise AssertionError('%s has no state %r' %
                                 (type(self).__name__, state))
        # Keep handles of ancestors only when entering a strict descendant
        # of the current state (parent -> parent.child).
        cur = self._fsm_state
        keep = 0
        if cur is not None and state.startswith(cur + '.'):
            keep = len(self._fsm_handles)
            for _, h in self._fsm_handles:
                h._used = False     # the parent may transition again later
        for _, h in reversed(self._fsm_handles[keep:]):
            h._dispose()
        del self._fsm_handles[keep:]
        # Any handle of an abandoned level must not run gotoState again;
        # pending transitions requested through them are dropped above.
        self._fsm_state = state
        if len(self.fsm_history) > 64:
            del self.fsm_history[:32]
        self.fsm_history.append(state)
        h = StateHandle(self, state, self.fsm_loop)
        self._fsm_handles.append((state, h))
        fn(h)
        self.emit('stateChanged', state)
