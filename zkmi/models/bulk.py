"""Bulk (pipelined, GPU-coded) requests on a live connection.

The reference sends every request through ``ZKEncodeStream`` one object at a
time and decodes every reply on the event loop (``lib/zk-streams.js:39-148``,
``lib/connection-fsm.js:384-408``).  A :class:`BulkBatch` carries N requests
as ONE unit through the same connection, with the byte work on the GPU:

  submit   K10 encodes the N requests (xids = a contiguous range reserved on
           the connection, opcodes recorded in an HBM xid table) into one
           framed byte stream; one D2H copy, one socket write.
  collect  the connection's host framer routes every reply frame whose xid
           falls in the range into the batch's RX buffer (notifications,
           pings and ordinary requests keep flowing through the normal path,
           ZooKeeper answers a session's requests in order).
  finish   one H2D copy of the collected reply stream, K1 frame scan,
           K2-K8 decode into SoA tensors (:class:`~zkmi.ops.batch.ReplyBatch`).

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

    def __init__(self, n, replies=None, buf=None, packets=None, device=None):
        self.n = n
        self.replies = replies
        self.buf = buf
        self.device = device
        self._packets = packets

    def packets(self):
        if self._packets is None:
            from ..ops import batch as B
            self._packets = B.replies_to_packets(self.buf, self.replies,
                                                 self.n)
        return self._packets

    def errors(self):
        """Per-request error names ('OK', 'NO_NODE', ...)."""
        if self.replies is not None and self._packets is None:
            errs = self.replies.err[:self.n].cpu().tolist()
            return [consts.ERR_LOOKUP.get(e, e) for e in errs]
        return [p.get('err') for p in self.packets()]

    def ok_count(self):
        if self.replies is not None:
            r = self.replies
            return int(((r.err[:self.n] == 0) & (r.status[:self.n] == 0))
                       .sum().item())
        return sum(1 for p in self.packets() if p.get('err') == 'OK')


class BulkBatch(object):
    """N requests (dicts as :func:`zkmi.jute.encode_request` takes them,
    without xids) submitted, collected and decoded as one unit."""

    def __init__(self, pkts, device=None):
        self.pkts = list(pkts)
        self.n = len(self.pkts)
        self.device = _gpu_device(device)
        self.x0 = 0
        self.rx = bytearray()
        self.got = 0
        self.cb = None
        self.t_submit = None
        self.done = False
        self.xid_map = None
        self.xt = None

    # -- encode ---------------------------------------------------------------

    def encode(self, x0):
        """Assign xids ``x0 .. x0+n-1`` and return the framed request
        stream (bytes) for the socket."""
        self.x0 = x0
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
            rb = B.pack_requests(self.pkts, self.device)
            bits = max(12, (max(self.n, 1) - 1).bit_length() + 1)
            self.xt = B.XidTable(bits=bits, device=self.device)
            tx, _, total, err = B.encode_requests(rb, self.xt)
            ntx = int(total.item())
            if int(err.item()) != 0:
                raise ZKProtocolError('BAD_ARGUMENTS',
                                      'bulk request encode failed')
            return bytes(tx[:ntx].cpu().numpy().tobytes())

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

    def finish(self):
        if self.device is None:
            pk = []
            data = bytes(self.rx)
            frames, _, _ = codec.scan_frames(data, 0, len(data),
                                             consts.MAX_PACKET)
            for (o, ln) in frames:
                pk.append(codec.decode_response(data[o:o + ln], self.xid_map))
            return BulkResult(self.n, packets=pk)
        import numpy as np
        import torch
        from ..ops import batch as B
        with torch.cuda.device(self.device):
            host = torch.from_numpy(np.frombuffer(bytes(self.rx) or b'\0',
                                                  np.uint8).copy())
            buf = host.pin_memory().to(self.device, non_blocking=True)
            ft = B.frame_scan(buf, len(self.rx), cap=max(self.n, 1))
            rep = B.decode_replies(buf, ft, self.xt)
            torch.cuda.current_stream().synchronize()
        return BulkResult(self.n, replies=rep, buf=buf, device=self.device)

    def elapsed_ms(self):
        return (time.perf_counter() - self.t_submit) * 1e3
