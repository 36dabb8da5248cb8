"""R1 — the node-wide watch fan-out, as ZooKeeper wire frames.

A watched path has one owner rank (``owner_of``); only the owner's session
holds the server watch.  What it forwards to every rank are the frames its
connection already received — the NOTIFICATION (xid -1, type, state, path)
and the reply of the GET_DATA that re-armed the watch (data + Stat) — as
raw bytes: the native loop keeps the notifications in the transport (the
note sink, ``csrc/host/zk_loop.cpp``), the re-arm replies arrive in the
pinned RX buffer of a bulk batch (``Transport.capture``) and are already on
the GPU after its decode.  Nothing is decoded into Python objects or
re-encoded on the way (round 2 re-encoded every event in Python).

:meth:`FrameFanout.gather` moves every rank's framed stream to every rank:
one size exchange (W int64 sizes and frame counts, one host read), one
padded ``all_gather_into_tensor`` on the collective device (HBM over
RCCL/xGMI with ``nccl``, host memory with gloo), and the padding gaps
closed on the device.  :meth:`FrameFanout.decode` runs K1 + K2-K8 on the
gathered stream (GPU), or the host codec (CPU rehearsal).  The reply frames'
xids are the owner's bulk xids; :meth:`FrameFanout.forward_replies` rewrites
them on the device to one forwarding xid every rank's xid table maps to
GET_DATA.

Users: :class:`zkmi.parallel.ensemble.EnsembleWorkload` (BASELINE config 4),
:class:`zkmi.parallel.group.SessionGroup` (the DistributedWatcher API) and
:class:`zkmi.bench.synthetic.WatchPipeline` (the GPU server's write-fired
notifications).  Reference: ``lib/zk-session.js:853-854`` (one watcher's
events to every listener), ``:421-471`` (re-arm on a move).
"""

import collections
import zlib

import torch
import torch.distributed as dist

from .. import codec
from .. import consts
from .. import jute

XID_FWD = 0x7ffffff0          # the forwarded replies' xid (-> GET_DATA)
XID_FWD_KIDS = 0x7ffffff1     # (-> GET_CHILDREN2)
XID_FWD_STAT = 0x7ffffff2     # (-> EXISTS)
FWD_XIDS = {XID_FWD: 'GET_DATA', XID_FWD_KIDS: 'GET_CHILDREN2',
            XID_FWD_STAT: 'EXISTS'}


def owner_of(path, world):
    """Deterministic owner rank of a path (same on every rank)."""
    return zlib.crc32(path.encode('utf-8')) % world


class Gathered(object):
    """Every rank's framed stream, in rank order, without padding: ``buf``
    (uint8 tensor), ``nbytes`` / ``frames`` per rank (host lists),
    ``total`` bytes."""

    def __init__(self, buf, nbytes, frames):
        self.buf = buf
        self.nbytes = nbytes
        self.frames = frames
        self.total = sum(nbytes)


class FrameFanout(object):
    """Collective: every rank calls :meth:`gather` together."""

    def __init__(self, group=None, device=None, coll_device=None):
        on = dist.is_available() and dist.is_initialized()
        self.group = group
        self.world = dist.get_world_size(group) if on else 1
        self.rank = dist.get_rank(group) if on else 0
        backend = dist.get_backend(group) if on else None
        if device is None and torch.cuda.is_available():
            device = torch.device('cuda', torch.cuda.current_device())
        self.dev = torch.device(device) if device is not None else None
        if self.dev is not None and self.dev.type != 'cuda':
            self.dev = None
        # collective tensors live where the backend moves them: HBM for
        # RCCL, host memory for gloo
        self.coll = self.dev if backend in (None, 'nccl') and self.dev \
            else torch.device('cpu')
        if coll_device is not None:
            self.coll = torch.device(coll_device)
        self.stats = collections.Counter()
        self.xt = None
        self._slots = {}
        if self.dev is not None:
            from ..ops import batch as B
            self.B = B
            self.xt = B.XidTable(bits=12, device=self.dev)
            for x, op in FWD_XIDS.items():
                self.xt.tab[x & self.xt.mask] = \
                    (x << 32) | consts.OP_CODES[op]
            self._x4 = torch.tensor(list(XID_FWD.to_bytes(4, 'big')),
                                    dtype=torch.uint8, device=self.dev)

    # -- the collective -------------------------------------------------------

    def gather(self, stream, nframes):
        """Send this rank's framed ``stream`` (uint8 tensor on any device,
        or bytes) of ``nframes`` frames; receive every rank's."""
        if isinstance(stream, (bytes, bytearray)):
            stream = torch.frombuffer(bytearray(stream or b'\0'),
                                      dtype=torch.uint8)[:len(stream)]
        n = stream.numel()
        W = self.world
        out_dev = self.dev if self.dev is not None else torch.device('cpu')
        if W == 1:
            self.stats['exchanges'] += 1
            self.stats['bytes'] += n
            return Gathered(stream.to(out_dev, non_blocking=True), [n],
                            [nframes])
        hdr = torch.tensor([n, nframes], dtype=torch.int64, device=self.coll)
        allh = torch.empty(2 * W, dtype=torch.int64, device=self.coll)
        dist.all_gather_into_tensor(allh, hdr, group=self.group)
        h = allh.cpu().tolist()                  # the one host read
        sizes, frames = h[0::2], h[1::2]
        mx = max(max(sizes), 1)
        buf = torch.zeros(mx, dtype=torch.uint8, device=self.coll)
        if n:
            buf[:n].copy_(stream, non_blocking=True)
        rx = torch.empty(W * mx, dtype=torch.uint8, device=self.coll)
        dist.all_gather_into_tensor(rx, buf, group=self.group)
        rx = rx.to(out_dev, non_blocking=True)
        # close the padding gaps (rank order kept)
        parts = [rx[r * mx:r * mx + s] for r, s in enumerate(sizes) if s]
        body = torch.cat(parts) if parts else rx[:0]
        self.stats['exchanges'] += 1
        self.stats['bytes'] += sum(sizes)
        return Gathered(body, sizes, frames)

    def gather_slots(self, buf, rec_off, count, cap, total, slot):
        """The fixed-slot transport: no host read, so a step can be
        graph-captured.  This rank's framed stream (``buf``, ``total`` bytes,
        ``count`` records starting at ``rec_off``, at most ``cap``; all
        device tensors) is cut into one ``slot``-byte segment ({bytes,
        records} header + frames, ``seg_pack``), every rank's segment is
        all-gathered, and the payloads are concatenated on the device in
        rank order (``seg_unpack``).  Returns ``(rx, nrx, src_counts,
        overflow)``: the stream, its device length, the records per source
        rank and the pack stats (``overflow[0]``: a stream that did not fit
        its slot went empty).  Buffers are kept per slot size."""
        from ..ops import _lib
        L = _lib.lib()
        W = self.world
        dev = buf.device
        st = self._slots.get(slot)
        if st is None:
            u8 = torch.uint8
            st = self._slots[slot] = {
                'send': torch.empty(slot, dtype=u8, device=dev),
                'big': torch.empty(W * slot, dtype=u8, device=dev),
                'rx': torch.empty(W * (slot - 16) + 64, dtype=u8, device=dev),
                'nrx': torch.zeros(1, dtype=torch.int64, device=dev),
                'src': torch.zeros(W, dtype=torch.int64, device=dev),
                'pstats': torch.zeros(3, dtype=torch.int64, device=dev)}
        L.seg_pack(buf, rec_off, count, cap, total, count, 1, 0, slot,
                   st['send'], st['pstats'])
        big = st['send']
        if W > 1:
            big = st['big']
            if self.coll == dev:
                dist.all_gather_into_tensor(big, st['send'], group=self.group)
            else:
                o = torch.empty(big.shape, dtype=torch.uint8,
                                device=self.coll)
                dist.all_gather_into_tensor(o, st['send'].to(self.coll),
                                            group=self.group)
                big.copy_(o)
        L.seg_unpack(big, W, self.rank, slot, st['rx'], st['nrx'], st['src'],
                     None)
        self.stats['slot_exchanges'] += 1
        return st['rx'], st['nrx'], st['src'], st['pstats']

    # -- helpers for the owner side -------------------------------------------

    def forward_replies(self, res):
        """The reply frames of a bulk batch (:class:`~zkmi.models.bulk.
        BulkResult` on the GPU path) as a forwardable device stream: their
        xids rewritten to :data:`XID_FWD`.  Returns the uint8 tensor."""
        buf = res.buf[:res.nbytes].clone()
        off = res.frames.off[:res.n]             # body offsets: the xid
        idx = off.unsqueeze(1) + torch.arange(4, device=buf.device)
        buf[idx.reshape(-1)] = self._x4.repeat(res.n)
        return buf

    # -- decode ---------------------------------------------------------------

    def decode(self, g):
        """The gathered stream decoded: on the GPU a (frame table,
        :class:`~zkmi.ops.batch.ReplyBatch`) pair of device tensors; on the
        host a list of packet dicts."""
        if self.dev is None:
            raw = bytes(g.buf.numpy().tobytes()) if g.total else b''
            frames, _, bad = codec.scan_frames(raw, 0, len(raw),
                                               consts.MAX_PACKET)
            if bad >= 0:
                raise RuntimeError('fan-out stream: bad frame')
            xmap = dict(FWD_XIDS)
            self.stats['decoded_host'] += len(frames)
            return [codec.decode_response(raw[o:o + ln], xmap)
                    for o, ln in frames]
        B = self.B
        nf = sum(g.frames)
        ft = B.frame_scan(g.buf, g.total, cap=max(nf, 1),
                          window=B.frame_window(512))
        rep = B.decode_replies(g.buf, ft, self.xt)
        self.stats['decoded_gpu'] += nf
        return ft, rep

    def decode_packets(self, g):
        """The gathered stream as packet dicts (:func:`zkmi.jute.
        decode_response`'s), for listeners that take Python values: decoded
        on the GPU (K1 + K2-K8) when there is one, else by the host codec."""
        if self.dev is None:
            return self.decode(g)
        if g.total == 0:
            return []
        ft, rep = self.decode(g)
        return self.B.replies_to_packets(g.buf, rep, n=sum(g.frames))

    @staticmethod
    def pair_index(frames, device):
        """For streams laid out per rank as [n notifications][n replies]:
        the global frame indices of every notification and of its reply
        (device int64 tensors, rank order)."""
        m = torch.tensor([f // 2 for f in frames], dtype=torch.int64)
        base = torch.zeros(len(frames), dtype=torch.int64)
        if len(frames) > 1:
            base[1:] = torch.cumsum(2 * m, 0)[:-1]
        tot = int(m.sum())
        if tot == 0:
            z = torch.zeros(0, dtype=torch.int64, device=device)
            return z, z
        seg = torch.repeat_interleave(torch.arange(len(frames)), m)
        first = torch.zeros(len(frames), dtype=torch.int64)
        if len(frames) > 1:
            first[1:] = torch.cumsum(m, 0)[:-1]
        k = torch.arange(tot) - first[seg]
        nidx = base[seg] + k
        ridx = nidx + m[seg]
        return nidx.to(device), ridx.to(device)


def notification_frames(paths, evtype=-1):
    """NOTIFICATION frames (xid -1, state SyncConnected) for ``paths``,
    host-encoded: the initial value of a bulk watch is forwarded as a
    notification of type ``evtype`` (-1: none, the watch's first value)
    followed by its GET_DATA reply, like every later change."""
    out = []
    for p in paths:
        body = jute.encode_response({
            'xid': consts.XID_NOTIFICATION, 'zxid': -1, 'err': 'OK',
            'opcode': 'NOTIFICATION', 'type': evtype,
            'state': 'SYNC_CONNECTED', 'path': p})
        out.append(len(body).to_bytes(4, 'big') + body)
    return b''.join(out)


def path_ids(buf, off, ln, digits):
    """The integer in the last ``digits`` bytes of each path (device): the
    workloads name paths ``.../pNNNNN``."""
    pos = (off + ln - digits).unsqueeze(1) + \
        torch.arange(digits, device=buf.device)
    d = buf[pos.reshape(-1)].reshape(-1, digits).to(torch.int64) - 48
    w = torch.tensor([10 ** (digits - 1 - i) for i in range(digits)],
                     dtype=torch.int64, device=buf.device)
    return (d * w).sum(1)

