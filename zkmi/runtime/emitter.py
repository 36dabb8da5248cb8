"""Minimal Node-style EventEmitter.

The reference builds every component on ``events.EventEmitter`` (e.g.
``lib/zk-session.js:527``, ``lib/connection-fsm.js:378``).  Semantics kept:
listeners run synchronously in registration order; ``once`` listeners are
removed before they run; emitting ``'error'`` with no listener raises the
error (Node throws it).
"""


class _Once(object):
    __slots__ = ('fn', 'emitter', 'evt', 'fired')

    def __init__(self, emitter, evt, fn):
        self.emitter = emitter
        self.evt = evt
        self.fn = fn
        self.fired = False

    def __call__(self, *args):
        if self.fired:
            return None
        self.fired = True
        self.emitter.removeListener(self.evt, self)
        return self.fn(*args)


class EventEmitter(object):

    def __init__(self):
        self._listeners = {}

    def on(self, evt, fn):
        self._listeners.setdefault(evt, []).append(fn)
        return self

    addListener = on

    def once(self, evt, fn):
        return EventEmitter.on(self, evt, _Once(self, evt, fn))

    def removeListener(self, evt, fn):
        lst = self._listeners.get(evt)
        if not lst:
            return self
        for i, l in enumerate(lst):
            if l is fn or (isinstance(l, _Once) and l.fn is fn):
                del lst[i]
                break
        if not lst:
            del self._listeners[evt]
        return self

    off = removeListener

    def removeAllListeners(self, evt=None):
        if evt is None:
            self._listeners.clear()
        else:
            self._listeners.pop(evt, None)
        return self

    def listeners(self, evt):
        return list(self._listeners.get(evt, ()))

    def listenerCount(self, evt):
        return len(self._listeners.get(evt, ()))

    def emit(self, evt, *args):
        lst = self._listeners.get(evt)
        if not lst:
            if evt == 'error':
                err = args[0] if args else Exception('Unhandled error')
                if isinstance(err, BaseException):
                    raise err
                raise Exception('Unhandled error: %r' % (err,))
            return False
        for fn in tuple(lst):
            fn(*args)
        return True
