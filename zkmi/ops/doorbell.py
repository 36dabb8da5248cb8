"""Persistent doorbell codec (csrc/kernels/doorbell.hip): one resident GPU
wave serves single-record encode / decode requests through a ring of slots
in host-coherent memory, so an interactive op costs a host<->GPU round trip
rather than a kernel launch.

The wave is started per :class:`DoorbellCodec` and always leaves on its own
after ``max_seconds`` (an in-kernel s_memrealtime deadline), so a forgotten
or crashed owner cannot leave it spinning; :meth:`close` (also called by
``with`` and at interpreter exit) stops it at once.

Encodes GET_DATA / EXISTS / GET_CHILDREN(2) / GET_ACL / SYNC / DELETE / PING
/ CLOSE_SESSION requests and decodes reply headers plus GET_DATA / EXISTS /
SET_DATA bodies, byte-identical to :mod:`zkmi.jute` (tests/test_doorbell.py).
"""

import atexit
import ctypes
import weakref

from .. import consts
from ..errors import ZKDecodeError
from ..jute import Stat
from . import _lib

P, I32, I64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64

_SIGS = {
    'zk_db_slot_bytes': (I64, []),
    'zk_db_create': (P, [I32]),
    'zk_db_start': (I32, [P, I64]),
    'zk_db_stop': (I32, [P]),
    'zk_db_destroy': (None, [P]),
    'zk_db_encode': (I32, [P, I32, I32, I32, ctypes.c_char_p, I32, P, I32,
                           I64]),
    'zk_db_decode': (I32, [P, I32, ctypes.c_char_p, I32, P, I64]),
    'zk_db_served': (I64, [P]),
}

_live = weakref.WeakSet()
_L = None


def _lib_db():
    """The doorbell's control functions in libzkmi_hip.so.  Unlike the
    batch codec (torch.ops.zkmi) they move no tensors: an opaque handle to
    host-coherent slot memory and per-record host buffers, so they are
    bound directly."""
    global _L
    if _L is None:
        _lib.lib()                    # torch + the op library (and HIP) first
        L = ctypes.CDLL(_lib.HIP_LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _L = L
    return _L


@atexit.register
def _close_all():
    for c in list(_live):
        c.close()


class DoorbellCodec(object):

    def __init__(self, nslots=8, max_seconds=10.0, timeout_s=2.0):
        L = _lib_db()
        self._L = L
        self._h = L.zk_db_create(nslots)
        if not self._h:
            raise RuntimeError('zk_db_create failed')
        self.timeout_us = int(timeout_s * 1e6)
        self._out = ctypes.create_string_buffer(1056)
        self._res = (ctypes.c_int64 * 16)()
        rc = L.zk_db_start(self._h, int(max_seconds * 1000))
        if rc != 0:
            L.zk_db_destroy(self._h)
            self._h = None
            raise RuntimeError('zk_db_start failed (%d)' % rc)
        _live.add(self)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def close(self):
        if self._h:
            self._L.zk_db_destroy(self._h)
            self._h = None

    @property
    def served(self):
        return self._L.zk_db_served(self._h) if self._h else 0

    def _check(self, rc, what):
        if rc == -2:
            raise TimeoutError('doorbell %s timed out' % what)
        if rc == -3:
            raise RuntimeError('doorbell wave has left (deadline or stop)')
        if rc < 0:
            raise ValueError('doorbell %s rejected the record' % what)

    def encode_request(self, pkt):
        """Framed request bytes for ``pkt`` (the dicts :mod:`zkmi.jute`
        takes)."""
        op = pkt['opcode']
        code = consts.OP_CODES[op]
        path = pkt.get('path', '').encode('utf-8')
        if op == 'DELETE':
            arg = pkt.get('version', -1)
        else:
            arg = 1 if pkt.get('watch') else 0
        n = self._L.zk_db_encode(self._h, pkt['xid'], code, arg, path,
                                 len(path), ctypes.addressof(self._out), 1056,
                                 self.timeout_us)
        self._check(n, 'encode')
        return self._out.raw[:n]

    def decode_response(self, body, opcode):
        """Decode a reply body whose request opcode is ``opcode`` -> the
        dict :func:`zkmi.jute.decode_response` returns."""
        code = consts.OP_CODES[opcode]
        rc = self._L.zk_db_decode(self._h, code, bytes(body), len(body),
                                  ctypes.addressof(self._res),
                                  self.timeout_us)
        self._check(rc, 'decode')
        r = list(self._res)
        if r[0] == 3:                    # ST_BAD_OPCODE
            raise ValueError('doorbell decode: opcode %s not handled' % opcode)
        if r[0] != 0:
            raise ZKDecodeError('BAD_DECODE', 'doorbell decode failed')
        err = consts.ERR_LOOKUP.get(r[3], r[3])
        pkt = {'xid': r[1], 'zxid': r[2], 'err': err, 'opcode': opcode}
        if err != 'OK':
            return pkt
        if opcode in ('GET_DATA', 'EXISTS', 'SET_DATA'):
            dl = r[15] & 0xffffffff
            st = Stat(czxid=r[6], mzxid=r[7], ctime=r[8], mtime=r[9],
                      version=r[12], cversion=r[13], aversion=r[14],
                      ephemeralOwner=r[10],
                      dataLength=dl - (1 << 32) if dl & 0x80000000 else dl,
                      numChildren=r[15] >> 32, pzxid=r[11])
            pkt['stat'] = st
        if opcode == 'GET_DATA':
            pkt['data'] = bytes(body[r[4]:r[4] + r[5]])
        return pkt
