"""Bulk (pipelined, GPU-coded) requests on a live connection.

The reference sends every request through ``ZKEncodeStream`` one object at a
time and decodes every reply on the event loop (``lib/zk-streams.js:39-148``,
``lib/connection-fsm.js:384-408``).  A :class:`BulkBatch` carries N requests
as ONE unit through the same connection, with the byte work on the GPU:

  submit   K10 encodes the N requests (xids = a contiguous range reserved on
           the connection, opcodes recorded in an HBM xid table) into one
           framed byte stream; one D2H copy into a pinned TX buffer, which
           the native loop queues straight from that memory (write_from).
  collect  the native loop's read path frames the inbound stream itself and
           copies every reply frame whose xid falls in the range into a
           pinned RX buffer (Transport.capture, csrc/host/zk_loop.cpp): no
           reply of the batch becomes a Python object.  Notifications,
           pings and ordinary requests keep flowing through the normal path
           (ZooKeeper answers a session's requests in order).
  finish   one H2D copy of the pinned RX buffer, K1 frame scan, K2-K8 decode
           into SoA tensors (:class:`~zkmi.ops.batch.ReplyBatch`); a CUDA
           event marks completion, readers wait on it.

Fallbacks: on the asyncio loop, or when the replies outgrow the RX buffer,
the connection routes reply frames to :meth:`BulkBatch.add` one by one (the
frames captured so far are kept).

Loop stall: ``encode`` (one D2H copy of the encoded stream) and ``finish``
(one H2D copy, then a wait on the decode) run on the connection's loop
thread, so every FSM on that loop (pings, expiry timers, watch delivery)
waits for them.  For a 1M-request batch that is a few milliseconds, well
under the ping interval (max(T/8, 2 s)); keep batches around 1M requests
or fewer, or run huge batches on a client of their own so only its loop
stalls.

Without a GPU (CPU-only hosts, the CPU test suite) the same object encodes
and decodes with the host codec (:mod:`zkmi.codec`), so the API works
everywhere; on a GPU box the HIP path is the one that runs.
"""

import time

from .. import codec, consts, jute
from ..errors import ZKProtocolError


def _gpu_device(device):
    """The torch device the batch codes on, or None for the host codec."""
    if device is False:
        return None
    try:
        import torch
    except ImportError:           # pragma: no cover - torch is a dependency
        return None
    if device is not None:
        return torch.device(device)
    if not torch.cuda.is_available():
        return None
    return torch.device('cuda', torch.cuda.current_device())


class BulkResult(object):
    """Decoded replies of one bulk batch, in request order.

    On the GPU path ``replies`` is a :class:`~zkmi.ops.batch.ReplyBatch` of
    device tensors and ``buf`` the device copy of the reply stream (data
    payloads are ``buf[pay_off:pay_off+pay_len]``); :meth:`packets` converts
    to the per-request dicts the interactive API produces.  On the host path
    the packets are decoded directly."""

    def __init__(self, n, replies=None, buf=None, packets=None, device=None,
                 event=None):
        self.n = n
        self.phases = {}
        self.replies = replies
        self.buf = buf
        self.device = device
        self._packets = packets
        self.event = event

    def wait(self):
        """Block until the GPU decode finished (no-op on the host path)."""
        if self.event is not None:
            self.event.synchronize()
        return self

    def packets(self):
        self.wait()
        if self._packets is None:
            from ..ops import batch as B
            self._packets = B.replies_to_packets(self.buf, self.replies,
                                                 self.n)
        return self._packets

    def errors(self):
        """Per-request error names ('OK', 'NO_NODE', ...)."""
        self.wait()
        if self.replies is not None and self._packets is None:
            errs = self.replies.err[:self.n].cpu().tolist()
            return [consts.ERR_LOOKUP.get(e, e) for e in errs]
        return [p.get('err') for p in self.packets()]

    def ok_count(self):
        self.wait()
        if self.replies is not None:
            r = self.replies
            return int(((r.err[:self.n] == 0) & (r.status[:self.n] == 0))
                       .sum().item())
        return sum(1 for p in self.packets() if p.get('err') == 'OK')


class BulkBatch(object):
    """N requests (dicts as :func:`zkmi.jute.encode_request` takes them,
    without xids) submitted, collected and decoded as one unit."""

    # reply bytes reserved per request in the pinned RX buffer (a GET_DATA
    # of 100 bytes is 192); bigger replies overflow into the per-frame path
    RX_PER_REQ = 224

    def __init__(self, pkts, device=None, reqs=None):
        """``pkts``: request dicts; or ``reqs`` = a device
        :class:`~zkmi.ops.batch.RequestBatch` already packed on the GPU
        (xids are assigned at submit), then ``pkts`` is None."""
        self.pkts = list(pkts) if pkts is not None else None
        self.reqs = reqs
        self.n = reqs.n if reqs is not None else len(self.pkts)
        self.device = _gpu_device(device)
        if reqs is not None and self.device is None:
            raise ValueError('a device request batch needs a GPU')
        self.capturing = False
        self.tx_pin = None
        self.rx_pin = None
        self.x0 = 0
        self.rx = bytearray()
        self.got = 0
        self.cb = None
        self.t_submit = None
        # phase clock (perf_counter): submit, encoded (K10 + D2H into the
        # pinned TX buffer done), sent (queued on the transport), captured
        # (every reply in the pinned RX buffer), finished (H2D + decode
        # enqueued); BulkResult.phases reports them
        self.t = {}
        self.done = False
        self.xid_map = None
        self.xt = None

    # -- encode ---------------------------------------------------------------

    @classmethod
    def gets(cls, paths, device=None, watch=False):
        """GET_DATA of every path (strings, or a device ``(arena u8, off
        i64, len i32)`` triple of path bytes) packed straight into a device
        request batch (no per-request dict).  ``watch``: each read arms a
        data watch (the re-arm of a bulk watch, see
        :meth:`~zkmi.models.client.Client.watch_bulk`)."""
        return cls._uniform('GET_DATA', paths, device, 1 if watch else 0)

    @classmethod
    def sets(cls, paths, data, device=None, version=-1):
        """SET_DATA of ``data`` (one bytes value for every path) at
        ``version`` to every path, packed like :meth:`gets`."""
        return cls._uniform('SET_DATA', paths, device, version,
                            bytes(data or b''))

    @classmethod
    def _uniform(cls, opcode, paths, device, arg, data=None):
        """One opcode over many paths (the arg and data shared): packed on
        the device with array ops, or as dicts on the host path."""
        dev = _gpu_device(device)
        if dev is None:
            if opcode == 'GET_DATA':
                return cls([{'opcode': opcode, 'path': p,
                             'watch': bool(arg)} for p in paths], False)
            return cls([{'opcode': opcode, 'path': p, 'data': data,
                         'version': arg} for p in paths], False)
        import numpy as np
        import torch
        from ..ops import batch as B
        if isinstance(paths, tuple):
            arena, off, ln = paths
            n = off.numel()
        else:
            enc = [p.encode('utf-8') for p in paths]
            n = len(enc)
            lens = np.fromiter((len(e) for e in enc), np.int32, n)
            offs = np.zeros(n, np.int64)
            if n > 1:
                np.cumsum(lens[:-1], out=offs[1:])
            blob = b''.join(enc) or b'\0'
            arena = torch.frombuffer(bytearray(blob), dtype=torch.uint8) \
                .to(dev)
            off = torch.from_numpy(offs).to(dev)
            ln = torch.from_numpy(lens).to(dev)
        z32 = torch.zeros(n, dtype=torch.int32, device=dev)
        z64 = torch.zeros(n, dtype=torch.int64, device=dev)
        op = torch.full((n,), consts.OP_CODES[opcode], dtype=torch.int32,
                        device=dev)
        a = torch.full((n,), arg, dtype=torch.int32, device=dev) \
            if arg else z32
        if data:
            darena = torch.frombuffer(bytearray(data), dtype=torch.uint8) \
                .to(dev)
            dlen = torch.full((n,), len(data), dtype=torch.int32, device=dev)
        else:
            darena, dlen = arena, z32
        rb = B.RequestBatch(n, op, z32, a, off, ln, z64, dlen, z32, arena,
                            darena, torch.zeros(1, dtype=torch.int64,
                                                device=dev),
                            torch.zeros(1, dtype=torch.int32, device=dev),
                            torch.zeros(16, dtype=torch.uint8, device=dev))
        return cls(None, dev, reqs=rb)

    def encode(self, x0):
        """Assign xids ``x0 .. x0+n-1`` and return the framed request
        stream for the socket: bytes, or on the GPU path ``(addr, n)`` of
        the pinned TX buffer holding it."""
        self.x0 = x0
        if self.pkts is not None:
            for i, p in enumerate(self.pkts):
                p['xid'] = x0 + i
        if self.device is None:
            self.xid_map = {}
            out = []
            for p in self.pkts:
                self.xid_map[p['xid']] = p['opcode']
                out.append(jute.frame(codec.encode_request(p)))
            return b''.join(out)
        import torch
        from ..ops import batch as B
        with torch.cuda.device(self.device):
            if self.reqs is not None:
                rb = self.reqs
                rb.xid = torch.arange(x0, x0 + self.n, dtype=torch.int32,
                                      device=self.device)
            else:
                rb = B.pack_requests(self.pkts, self.device)
            bits = max(12, (max(self.n, 1) - 1).bit_length() + 1)
            self.xt = B.XidTable(bits=bits, device=self.device)
            tx, _, total, err = B.encode_requests(rb, self.xt)
            te = torch.cat([total, err.to(torch.int64)]).cpu().tolist()
            ntx = te[0]
            if te[1] != 0:
                raise ZKProtocolError('BAD_ARGUMENTS',
                                      'bulk request encode failed')
            self.tx_pin = torch.empty(max(ntx, 1), dtype=torch.uint8,
                                      pin_memory=True)
            self.tx_pin[:ntx].copy_(tx[:ntx])
            self.t['encoded'] = time.perf_counter()
            return (self.tx_pin.data_ptr(), ntx)

    def rx_buffer(self):
        """(addr, size) of the pinned RX buffer the transport captures the
        batch's reply frames into."""
        import torch
        size = self.n * self.RX_PER_REQ + (1 << 16)
        self.rx_pin = torch.empty(size, dtype=torch.uint8, pin_memory=True)
        return self.rx_pin.data_ptr(), size

    def captured(self, status, nbytes, got):
        """The transport's capture ended.  ``status`` 0: all replies are in
        the RX buffer.  Otherwise the batch falls back to per-frame
        collection, keeping what was captured."""
        self.capturing = False
        self.t['captured'] = time.perf_counter()
        if status == 0:
            return True
        self.rx = bytearray(self.rx_pin[:nbytes].numpy().tobytes())
        self.got = got
        self.rx_pin = None
        return False

    # -- collect --------------------------------------------------------------

    def owns(self, xid):
        return self.x0 <= xid < self.x0 + self.n

    def add(self, body):
        """Append one reply frame body; True when the batch is complete."""
        self.rx += len(body).to_bytes(4, 'big')
        self.rx += body
        self.got += 1
        return self.got >= self.n

    # -- decode ---------------------------------------------------------------

    def finish(self, nbytes=None):
        """Decode the collected replies.  ``nbytes``: the replies are the
        first ``nbytes`` of the pinned RX buffer (capture path)."""
        if self.device is None:
            pk = []
            data = bytes(self.rx)
            frames, _, _ = codec.scan_frames(data, 0, len(data),
                                             consts.MAX_PACKET)
            for (o, ln) in frames:
                pk.append(codec.decode_response(data[o:o + ln], self.xid_map))
            res = BulkResult(self.n, packets=pk)
            res.raw = data              # (the reply frames as received)
            return res
        import numpy as np
        import torch
        from ..ops import batch as B
        with torch.cuda.device(self.device):
            if nbytes is not None:
                host = self.rx_pin[:max(nbytes, 1)]
            else:
                nbytes = len(self.rx)
                host = torch.from_numpy(np.frombuffer(
                    bytes(self.rx) or b'\0', np.uint8).copy()).pin_memory()
            buf = host.to(self.device, non_blocking=True)
            ft = B.frame_scan(buf, nbytes, cap=max(self.n, 1))
            rep = B.decode_replies(buf, ft, self.xt)
            ev = torch.cuda.Event()
            ev.record()
        # the pinned buffers stay referenced by the result until the copy
        # the event covers has run
        res = BulkResult(self.n, replies=rep, buf=buf, device=self.device,
                         event=ev)
        res.frames = ft                 # (the reply frames' offsets)
        res.nbytes = nbytes
        self.t['finished'] = time.perf_counter()
        res.phases = dict(self.t, submit=self.t_submit)
        res._hold = (host, self.tx_pin)
        self.rx_pin = self.tx_pin = None
        return res

    def elapsed_ms(self):
        return (time.perf_counter() - self.t_submit) * 1e3
