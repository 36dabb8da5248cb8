"""L0 — error classes.

Parity: ``lib/errors.js:19-54``.  ``message = code + ': ' + msg`` exactly as
the
reference formats it, and ``.code`` / ``.name`` carry the same strings so
callers can switch on them the same way.
"""


class ZKProtocolError(Exception):
    """Client-side / protocol error (``lib/errors.js:19-26``)."""

    name = 'ZKProtocolError'

    def __init__(self, code, msg):
        self.code = code
        self.message = '%s: %s' % (code, msg)
        super().__init__(self.message)

    def __str__(self):
        return '%s: %s' % (self.name, self.message)


class ZKError(Exception):
    """Server-returned error code (``lib/errors.js:47-54``)."""

    name = 'ZKError'

    def __init__(self, code, msg):
        self.code = code
        self.message = '%s: %s' % (code, msg)
        super().__init__(self.message)

    def __str__(self):
        return '%s: %s' % (self.name, self.message)


class ZKPingTimeoutError(ZKProtocolError):
    """Ping not answered in time (``lib/errors.js:28-35``)."""

    name = 'ZKPingTimeoutError'

    def __init__(self):
        super().__init__('PING_TIMEOUT', 'The server failed to answer a ping '
                         'within the required interval')


class ZKNotConnectedError(ZKProtocolError):
    """Request issued while not connected (``lib/errors.js:37-45``)."""

    name = 'ZKNotConnectedError'

    def __init__(self):
        super().__init__('CONNECTION_LOSS', 'The ZooKeeper client is not '
                         'currently connected and cannot accept new '
                         'requests.')


class ZKDecodeError(Exception):
    """Raised by the codecs on malformed input; the framing layer turns it
    into ``ZKProtocolError('BAD_DECODE', ...)``
    (``lib/zk-streams.js:74-95``)."""
