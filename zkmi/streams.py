"""L3 — length-prefixed stream framing (host side of the interactive path).

Parity: ``ZKDecodeStream`` / ``ZKEncodeStream`` (``lib/zk-streams.js:25-148``).

Differences by design:
  * The reference copies every packet out and memmoves the remainder of its
    buffer per packet (``zk-streams.js:54-60``, O(bytes x packets) per chunk,
    SURVEY §6).  :class:`ZKDecoder` frames a whole chunk in one pass and
    compacts its buffer once per chunk.
  * Framing and decoding are split: :meth:`ZKDecoder.feed` only returns
    complete frame bodies; the connection decodes each body according to its
    state at dispatch time (handshake vs. reply), which is the reference's
    ``fsm.isInState('handshaking')`` switch (``zk-streams.js:66-99``).
  * The encoder prunes nothing itself; the connection removes xid->opcode
    entries when the reply arrives (fixes SURVEY Appendix C-4's leak).

The per-record byte work goes through :mod:`zkmi.codec`, which is the native
C++ host codec when it has been built (``csrc/host``) and the pure-Python
oracle otherwise.  Batched GPU framing/decoding lives in :mod:`zkmi.ops`.
"""

from . import consts
from . import codec
from . import jute
from .errors import ZKProtocolError


class ZKDecoder(object):
    """Inbound framing with carry across chunks."""

    __slots__ = ('buf', 'dead', 'max_packet', 'frames_in', 'bytes_in')

    def __init__(self, max_packet=consts.MAX_PACKET):
        self.buf = bytearray()
        self.dead = False
        self.max_packet = max_packet
        self.frames_in = 0
        self.bytes_in = 0

    def feed(self, chunk):
        """Append ``chunk``; return ``(bodies, err)``.

        ``bodies`` is a list of complete frame bodies (bytes).  ``err`` is a
        ``ZKProtocolError('BAD_LENGTH')`` when a frame header is negative or
        larger than ``MAX_PACKET``; after that the decoder is dead and ignores
        further input, as the reference stream stalls
        (``zk-streams.js:47-53``)."""
        if self.dead:
            return [], None
        self.bytes_in += len(chunk)
        buf = self.buf
        if buf:
            buf += chunk
            data = buf
        else:
            data = chunk
        frames, consumed, bad_at = codec.scan_frames(data, 0, len(data),
                                                    self.max_packet)
        bodies = [bytes(data[o:o + n]) for (o, n) in frames]
        self.frames_in += len(bodies)
        err = None
        if bad_at >= 0:
            self.dead = True
            self.buf = bytearray()
            err = ZKProtocolError('BAD_LENGTH', 'Invalid ZK packet length')
        elif data is buf:
            del buf[:consumed]
        else:
            self.buf = bytearray(data[consumed:])
        return bodies, err

    def pending(self):
        return len(self.buf)

    def take_pending(self):
        """Hand the buffered partial frame to another framer (the native
        transport's bulk capture) and forget it."""
        b = bytes(self.buf)
        self.buf = bytearray()
        return b


class ZKEncoder(object):
    """Outbound framing; records ``xid -> opcode`` for the decoder
    (``zk-streams.js:145``)."""

    __slots__ = ('xid_map', 'frames_out', 'gpu')

    def __init__(self, xid_map, gpu=None):
        self.xid_map = xid_map
        self.frames_out = 0
        # GpuControlCodec (models/gpucodec.py): K9 / K11 for the handshake
        # and SET_WATCHES records when the client has a codec device
        self.gpu = gpu

    def connect_request(self, pkt):
        self.frames_out += 1
        if self.gpu is not None:
            return self.gpu.connect_request(pkt)
        return codec.frame(codec.encode_connect_request(pkt))

    def request(self, pkt):
        xid = pkt['xid']
        if not isinstance(xid, int):
            raise TypeError('xid must be an int')
        if pkt['opcode'] == 'SET_WATCHES' and \
                jute.packed_events(pkt['events']):
            # the bulk watches' vector is already encoded: a byte copy
            out = jute.frame(jute.encode_request(pkt))
        elif self.gpu is not None and pkt['opcode'] == 'SET_WATCHES':
            out = self.gpu.set_watches(pkt)
        else:
            out = codec.frame(codec.encode_request(pkt))
        self.xid_map[xid] = pkt['opcode']
        self.frames_out += 1
        return out
