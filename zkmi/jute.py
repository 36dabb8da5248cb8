"""L1/L2 — Jute record codec in pure Python.

This is the *test oracle* for the native codecs (the C++ host codec in
``csrc/host`` and the HIP batch kernels in ``csrc/kernels``) and the fallback
used on machines where the native host codec has not been built.

Parity map (reference ``lib/``):
  * primitives — ``jute-buffer.js:14-189`` (i32 BE, 8-byte longs, length
    prefixed buffers where an *empty* buffer is written as length -1
    (``:127-130``) and any negative length reads as empty (``:99-100``),
    bools that must be 0/1 (``:51-56``));
  * handshake records — ``zk-buffer.js:22-56``;
  * request bodies — ``zk-buffer.js:97-273`` (client encode) and
    ``:58-95``/``:138-253`` (server-mode decode);
  * reply decode — ``zk-buffer.js:275-370``;
  * ACL / perms / Stat — ``zk-buffer.js:372-442``.

Deliberate fix vs the reference: ``readPerms`` has an operator-precedence bug
(``zk-buffer.js:399``) that returns all five perms iff the
READ bit is set.  We decode the mask correctly; the only reference test that
covers it (all perms set) passes either way.

Extension vs the reference: ``encode_response`` (server-mode reply encode) is
missing in the reference (``zk-streams.js:140``) and is provided here for the
fake server and the GPU synthetic server.
"""

import struct

from . import consts
from .errors import ZKDecodeError

_I32 = struct.Struct('>i')
_I64 = struct.Struct('>q')
_HDR_REQ = struct.Struct('>ii')          # xid, opcode
_HDR_REPLY = struct.Struct('>iqi')       # xid, zxid, err
_STAT = struct.Struct('>qqqqiiiqiiq')    # 68 bytes
_NOTIF = struct.Struct('>ii')            # type, state

assert _STAT.size == consts.STAT_SIZE


class Stat(object):
    """A ZooKeeper ``Stat`` record (``zk-buffer.js:428-442``).

    Field names match the reference / ZooKeeper.  zxids, ``ephemeralOwner``
    and the ms timestamps are Python ints (the reference used 8-byte Buffers
    and ``LongDate``).
    """

    __slots__ = ('czxid', 'mzxid', 'ctime', 'mtime', 'version', 'cversion',
                 'aversion', 'ephemeralOwner', 'dataLength', 'numChildren',
                 'pzxid')

    def __init__(self, czxid=0, mzxid=0, ctime=0, mtime=0, version=0,
                 cversion=0, aversion=0, ephemeralOwner=0, dataLength=0,
                 numChildren=0, pzxid=0):
        self.czxid = czxid
        self.mzxid = mzxid
        self.ctime = ctime
        self.mtime = mtime
        self.version = version
        self.cversion = cversion
        self.aversion = aversion
        self.ephemeralOwner = ephemeralOwner
        self.dataLength = dataLength
        self.numChildren = numChildren
        self.pzxid = pzxid

    @classmethod
    def from_tuple(cls, t):
        s = cls.__new__(cls)
        (s.czxid, s.mzxid, s.ctime, s.mtime, s.version, s.cversion,
         s.aversion, s.ephemeralOwner, s.dataLength, s.numChildren,
         s.pzxid) = t
        return s

    def as_tuple(self):
        return (self.czxid, self.mzxid, self.ctime, self.mtime, self.version,
                self.cversion, self.aversion, self.ephemeralOwner,
                self.dataLength, self.numChildren, self.pzxid)

    def to_bytes(self):
        return _STAT.pack(*self.as_tuple())

    def ctime_date(self):
        import datetime
        return datetime.datetime.fromtimestamp(self.ctime / 1000.0)

    def mtime_date(self):
        import datetime
        return datetime.datetime.fromtimestamp(self.mtime / 1000.0)

    # snake_case aliases
    @property
    def ephemeral_owner(self):
        return self.ephemeralOwner

    @property
    def data_length(self):
        return self.dataLength

    @property
    def num_children(self):
        return self.numChildren

    def __eq__(self, other):
        return isinstance(other, Stat) and self.as_tuple() == other.as_tuple()

    def __hash__(self):
        return hash(self.as_tuple())

    def __repr__(self):
        return 'Stat(%s)' % ', '.join('%s=%r' % (k, getattr(self, k))
                                       for k in self.__slots__)


# --------------------------------------------------------------------------
# Primitive reader / writer
# --------------------------------------------------------------------------

class JuteReader(object):
    """Cursor over a bytes-like object (``jute-buffer.js:14-105``)."""

    __slots__ = ('buf', 'off', 'end')

    def __init__(self, buf, off=0, end=None):
        self.buf = buf
        self.off = off
        self.end = len(buf) if end is None else end

    def _need(self, n):
        if self.off + n > self.end:
            raise ZKDecodeError('read of %d bytes at offset %d overruns '
                                'record of %d bytes' % (n, self.off, self.end))

    def at_end(self):
        return self.off >= self.end

    def read_int(self):
        self._need(4)
        v = _I32.unpack_from(self.buf, self.off)[0]
        self.off += 4
        return v

    def read_long(self):
        self._need(8)
        v = _I64.unpack_from(self.buf, self.off)[0]
        self.off += 8
        return v

    def read_bool(self):
        self._need(1)
        v = self.buf[self.off]
        self.off += 1
        if v not in (0, 1):
            raise ZKDecodeError('bad bool byte %d' % v)
        return v == 1

    def read_buffer(self):
        n = self.read_int()
        if n < 0:
            n = 0
        self._need(n)
        v = bytes(self.buf[self.off:self.off + n])
        self.off += n
        return v

    def read_ustring(self):
        return self.read_buffer().decode('utf-8')

    def read_stat(self):
        self._need(consts.STAT_SIZE)
        t = _STAT.unpack_from(self.buf, self.off)
        self.off += consts.STAT_SIZE
        return Stat.from_tuple(t)

    def read_perms(self):
        val = self.read_int()
        return [k for k, m in consts.PERM_MASKS.items() if (val & m) != 0]

    def read_id(self):
        scheme = self.read_ustring()
        ident = self.read_ustring()
        return {'scheme': scheme, 'id': ident}

    def read_acl(self):
        n = self.read_int()
        acl = []
        for _ in range(max(n, 0)):
            perms = self.read_perms()
            ident = self.read_id()
            acl.append({'perms': perms, 'id': ident})
        return acl

    def read_string_vector(self):
        n = self.read_int()
        return [self.read_ustring() for _ in range(max(n, 0))]


class JuteWriter(object):
    """Growable output buffer (``jute-buffer.js:107-189``)."""

    __slots__ = ('buf',)

    def __init__(self):
        self.buf = bytearray()

    def write_int(self, v):
        self.buf += _I32.pack(v)

    def write_long(self, v):
        self.buf += _I64.pack(v)

    def write_bool(self, v):
        self.buf.append(1 if v else 0)

    def write_buffer(self, v):
        if v is None or len(v) == 0:
            # Empty buffers go on the wire as length -1
            # (jute-buffer.js:127-130).
            self.buf += _I32.pack(-1)
            return
        self.buf += _I32.pack(len(v))
        self.buf += v

    def write_ustring(self, s):
        self.write_buffer(s.encode('utf-8'))

    def write_perms(self, perms):
        self.write_int(perms_to_mask(perms))

    def write_acl(self, acl):
        self.write_int(len(acl))
        for line in acl:
            self.write_perms(line['perms'])
            self.write_ustring(line['id']['scheme'])
            self.write_ustring(line['id']['id'])

    def write_stat(self, stat):
        self.buf += stat.to_bytes()

    def write_string_vector(self, v):
        self.write_int(len(v))
        if isinstance(v, PackedStrings):
            self.buf += v.blob
            return
        for s in v:
            self.write_ustring(s)

    def getvalue(self):
        return bytes(self.buf)


class PackedStrings(object):
    """A jute string vector kept encoded: ``n`` entries, ``blob`` their
    length-prefixed UTF-8 bytes (the vector without its count).  For a large
    vector re-sent unchanged — the bulk watches every SET_WATCHES resume
    carries — so a resume copies bytes instead of encoding each path again.
    ``a + b`` concatenates (either side may be a list of strings)."""

    __slots__ = ('n', 'blob')

    def __init__(self, n=0, blob=b''):
        self.n = n
        self.blob = blob

    @classmethod
    def of(cls, strings):
        if isinstance(strings, PackedStrings):
            return strings
        enc = [s.encode('utf-8') for s in strings]
        return cls(len(enc), b''.join(len(e).to_bytes(4, 'big') + e
                                      for e in enc))

    def __add__(self, other):
        o = PackedStrings.of(other)
        return PackedStrings(self.n + o.n, self.blob + o.blob)

    def __radd__(self, other):
        return PackedStrings.of(other) + self

    def __len__(self):
        return self.n

    def __iter__(self):
        b, k = self.blob, 0
        for _ in range(self.n):
            ln = int.from_bytes(b[k:k + 4], 'big')
            yield b[k + 4:k + 4 + ln].decode('utf-8')
            k += 4 + ln


def packed_events(events):
    """True when a SET_WATCHES ``events`` dict holds a :class:`PackedStrings`
    (encode it with this module's :func:`encode_request`)."""
    return any(isinstance(v, PackedStrings) for v in events.values())


def perms_to_mask(perms):
    """Upper-case names OR'd into a mask (``zk-buffer.js:405-414``).

    Accepts an int mask as a convenience."""
    if isinstance(perms, int):
        return perms
    val = 0
    for k in perms:
        m = consts.PERM_MASKS.get(k.upper())
        if m is None:
            raise ValueError('unknown permission %r' % (k,))
        val |= m
    return val


def flags_to_mask(flags):
    if isinstance(flags, int):
        return flags
    val = 0
    for k in flags:
        m = consts.CREATE_FLAGS.get(k)
        if m is None:
            raise ValueError('unknown flag %r' % (k,))
        val |= m
    return val


def mask_to_flags(mask):
    return [k for k, m in consts.CREATE_FLAGS.items() if (mask & m) == m]


DEFAULT_ACL = [{'id': {'scheme': 'world', 'id': 'anyone'},
                'perms': ['read', 'write', 'create', 'delete', 'admin']}]


# --------------------------------------------------------------------------
# Handshake records (zk-buffer.js:22-56)
# --------------------------------------------------------------------------

def encode_connect_request(pkt):
    w = JuteWriter()
    w.write_int(pkt.get('protocolVersion', 0))
    w.write_long(pkt.get('lastZxidSeen', 0))
    w.write_int(pkt['timeOut'])
    w.write_long(pkt.get('sessionId', 0))
    w.write_buffer(pkt.get('passwd', b'\0' * 8))
    return w.getvalue()


def decode_connect_request(body):
    r = JuteReader(body)
    pkt = {}
    pkt['protocolVersion'] = r.read_int()
    pkt['lastZxidSeen'] = r.read_long()
    pkt['timeOut'] = r.read_int()
    pkt['sessionId'] = r.read_long()
    pkt['passwd'] = r.read_buffer()
    # ZooKeeper >= 3.4 clients append readOnly; tolerate it.
    return pkt


def encode_connect_response(pkt, read_only=None):
    w = JuteWriter()
    w.write_int(pkt.get('protocolVersion', 0))
    w.write_int(pkt['timeOut'])
    w.write_long(pkt['sessionId'])
    w.write_buffer(pkt.get('passwd', b''))
    if read_only is not None:
        w.write_bool(read_only)
    return w.getvalue()


def decode_connect_response(body):
    r = JuteReader(body)
    pkt = {}
    pkt['protocolVersion'] = r.read_int()
    pkt['timeOut'] = r.read_int()
    pkt['sessionId'] = r.read_long()
    pkt['passwd'] = r.read_buffer()
    return pkt


# --------------------------------------------------------------------------
# Requests (client encode, server decode)
# --------------------------------------------------------------------------

def encode_request(pkt):
    """Request header + per-opcode body (``zk-buffer.js:97-136``)."""
    op = pkt['opcode']
    w = JuteWriter()
    w.buf += _HDR_REQ.pack(pkt['xid'], consts.OP_CODES[op])
    if op in ('GET_CHILDREN', 'GET_CHILDREN2', 'GET_DATA', 'EXISTS'):
        w.write_ustring(pkt['path'])
        w.write_bool(pkt.get('watch', False))
    elif op == 'CREATE':
        w.write_ustring(pkt['path'])
        w.write_buffer(pkt.get('data', b''))
        w.write_acl(pkt.get('acl', []))
        w.write_int(flags_to_mask(pkt.get('flags', [])))
    elif op == 'DELETE':
        w.write_ustring(pkt['path'])
        w.write_int(pkt['version'])
    elif op in ('GET_ACL', 'SYNC'):
        w.write_ustring(pkt['path'])
    elif op == 'SET_DATA':
        w.write_ustring(pkt['path'])
        w.write_buffer(pkt.get('data', b''))
        w.write_int(pkt.get('version', -1))
    elif op == 'SET_WATCHES':
        w.write_long(pkt['relZxid'])
        ev = pkt['events']
        w.write_string_vector(ev.get('dataChanged', []))
        w.write_string_vector(ev.get('createdOrDestroyed', []))
        w.write_string_vector(ev.get('childrenChanged', []))
    elif op in ('PING', 'CLOSE_SESSION'):
        pass
    else:
        raise ValueError('Unsupported opcode %s' % op)
    return w.getvalue()


def decode_request(body):
    """Server-mode request decode (``zk-buffer.js:58-95``, ``:138-253``)."""
    r = JuteReader(body)
    pkt = {}
    pkt['xid'] = r.read_int()
    code = r.read_int()
    op = consts.OP_CODE_LOOKUP.get(code)
    pkt['opcode'] = op
    if op in ('GET_CHILDREN', 'GET_CHILDREN2', 'GET_DATA', 'EXISTS'):
        pkt['path'] = r.read_ustring()
        pkt['watch'] = r.read_bool()
    elif op == 'CREATE':
        pkt['path'] = r.read_ustring()
        pkt['data'] = r.read_buffer()
        pkt['acl'] = r.read_acl()
        pkt['flags'] = mask_to_flags(r.read_int())
    elif op == 'DELETE':
        pkt['path'] = r.read_ustring()
        pkt['version'] = r.read_int()
    elif op in ('GET_ACL', 'SYNC'):
        pkt['path'] = r.read_ustring()
    elif op == 'SET_DATA':
        pkt['path'] = r.read_ustring()
        pkt['data'] = r.read_buffer()
        pkt['version'] = r.read_int()
    elif op == 'SET_WATCHES':
        pkt['relZxid'] = r.read_long()
        pkt['events'] = {
            'dataChanged': r.read_string_vector(),
            'createdOrDestroyed': r.read_string_vector(),
            'childrenChanged': r.read_string_vector(),
        }
    elif op in ('PING', 'CLOSE_SESSION'):
        pass
    else:
        raise ZKDecodeError('Unsupported opcode %r' % (code,))
    return pkt


# --------------------------------------------------------------------------
# Responses (client decode, server encode)
# --------------------------------------------------------------------------

def decode_response(body, xid_map):
    """Reply header + body, resolving the opcode from the special-xid table or
    the xid->opcode map recorded at encode time (``zk-buffer.js:275-331``).
    The body is decoded only when ``err == 'OK'`` (``:292``)."""
    r = JuteReader(body)
    if r.end < 16:
        raise ZKDecodeError('reply shorter than its 16-byte header')
    xid, zxid, err = _HDR_REPLY.unpack_from(body, 0)
    r.off = 16
    errname = consts.ERR_LOOKUP.get(err, err)
    op = consts.SPECIAL_XIDS.get(xid)
    if op is None:
        op = xid_map.get(xid)
    if op is None:
        raise ZKDecodeError('reply packet must match a request (xid %d)'
                            % xid)
    pkt = {'xid': xid, 'zxid': zxid, 'err': errname, 'opcode': op}
    if errname != 'OK':
        return pkt
    if op in ('GET_CHILDREN', 'GET_CHILDREN2'):
        pkt['children'] = r.read_string_vector()
        if op == 'GET_CHILDREN2':
            pkt['stat'] = r.read_stat()
    elif op == 'CREATE':
        pkt['path'] = r.read_ustring()
    elif op in ('EXISTS', 'SET_DATA'):
        pkt['stat'] = r.read_stat()
    elif op == 'GET_ACL':
        pkt['acl'] = r.read_acl()
        pkt['stat'] = r.read_stat()
    elif op == 'GET_DATA':
        pkt['data'] = r.read_buffer()
        pkt['stat'] = r.read_stat()
    elif op == 'NOTIFICATION':
        t = r.read_int()
        s = r.read_int()
        pkt['type'] = consts.NOTIFICATION_TYPE_LOOKUP.get(t, t)
        pkt['state'] = consts.STATE_LOOKUP.get(s, s)
        pkt['path'] = r.read_ustring()
    elif op in ('SET_WATCHES', 'PING', 'SYNC', 'DELETE', 'CLOSE_SESSION',
                'AUTH'):
        pass
    else:
        raise ZKDecodeError('Unsupported opcode %s' % op)
    return pkt


def encode_response(pkt):
    """Server-mode reply encode (missing in the reference,
    ``zk-streams.js:140``).  ``pkt`` has xid, zxid, err (name or int), opcode
    and, for OK replies, the body fields ``decode_response`` produces."""
    err = pkt.get('err', 'OK')
    code = consts.ERR_CODES[err] if isinstance(err, str) else err
    w = JuteWriter()
    w.buf += _HDR_REPLY.pack(pkt['xid'], pkt.get('zxid', 0), code)
    if code != 0:
        return w.getvalue()
    op = pkt['opcode']
    if op in ('GET_CHILDREN', 'GET_CHILDREN2'):
        w.write_string_vector(pkt['children'])
        if op == 'GET_CHILDREN2':
            w.write_stat(pkt['stat'])
    elif op == 'CREATE':
        w.write_ustring(pkt['path'])
    elif op in ('EXISTS', 'SET_DATA'):
        w.write_stat(pkt['stat'])
    elif op == 'GET_ACL':
        w.write_acl(pkt['acl'])
        w.write_stat(pkt['stat'])
    elif op == 'GET_DATA':
        w.write_buffer(pkt['data'])
        w.write_stat(pkt['stat'])
    elif op == 'NOTIFICATION':
        t = pkt['type']
        s = pkt.get('state', 'SYNC_CONNECTED')
        w.write_int(consts.NOTIFICATION_TYPE[t] if isinstance(t, str) else t)
        w.write_int(consts.STATE[s] if isinstance(s, str) else s)
        w.write_ustring(pkt['path'])
    return w.getvalue()


def frame(body):
    """Length-prefix one record (``jute-buffer.js:181-189``)."""
    return _I32.pack(len(body)) + body


# --------------------------------------------------------------------------
# Stream framing (zk-streams.js:25-148) — the pure-Python reference for K1.
# --------------------------------------------------------------------------

def scan_frames(buf, start=0, end=None, max_packet=consts.MAX_PACKET):
    """Split ``buf[start:end]`` into complete length-prefixed frames.

    Returns ``(frames, consumed, bad_at)`` where ``frames`` is a list of
    ``(body_offset, body_length)``, ``consumed`` is the offset just past the
    last complete frame, and ``bad_at`` is the offset of the first frame whose
    length prefix is negative or exceeds ``max_packet`` (``-1`` if none).
    Framing stops at a bad length exactly as the reference stalls there
    (``zk-streams.js:47-53``)."""
    if end is None:
        end = len(buf)
    frames = []
    off = start
    while end - off >= 4:
        n = _I32.unpack_from(buf, off)[0]
        if n < 0 or n > max_packet:
            return frames, off, off
        if end - off - 4 < n:
            break
        frames.append((off + 4, n))
        off += 4 + n
    return frames, off, -1
