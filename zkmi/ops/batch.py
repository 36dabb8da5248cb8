"""Batched GPU codec: torch-tensor API over the HIP kernels.

Every function here runs on the current HIP stream and allocates its outputs
with the torch caching allocator (cheap after warm-up).  Record counts that
the GPU discovers (frames in a byte stream) stay on the device as int64
scalars, so a pipeline of these calls needs no host synchronisation; call
``.item()`` only where a host decision is needed.

Kernel map: K1 :func:`frame_scan`; K2-K8
:func:`decode_replies` (+ :func:`expand_strings` / :func:`expand_acl` for the
ragged vectors); K9 handshake records stay on the host (one per connect);
K10 :func:`encode_requests`; K11 :func:`encode_set_watches`; K12
:func:`decode_requests`; K13 :func:`encode_responses`.
"""

import os
from dataclasses import dataclass

import numpy as np

import torch

from .. import consts
from .. import jute
from . import _lib

SENTINEL_XID = -(1 << 63)          # xid table entry that matches no xid
I64 = torch.int64
I32 = torch.int32
U8 = torch.uint8



# K1 tiles a wave takes on streams of large frames (FrameScanner group;
# ZKMI_FS_GROUP: 1, 2, 4, 8 or 16)
_FS_GROUP = int(os.environ.get('ZKMI_FS_GROUP', '8'))

def _dev(device):
    return torch.device(device) if device is not None else \
        torch.device('cuda', torch.cuda.current_device())


class XidTable(object):
    """Per-connection xid -> opcode map in HBM (``zk-streams.js:145``).

    A direct-mapped ring of ``2**bits`` int64 entries ``(xid << 32) | op``;
    the decoder verifies the stored xid, so a stale slot can never be
    mistaken for a live request."""

    def __init__(self, bits=20, device=None):
        self.bits = bits
        self.mask = (1 << bits) - 1
        self.tab = torch.full((1 << bits,), SENTINEL_XID, dtype=I64,
                              device=_dev(device))

    def reset(self):
        self.tab.fill_(SENTINEL_XID)


# ---------------------------------------------------------------------------
# Request batches (K10)
# ---------------------------------------------------------------------------

@dataclass
class RequestBatch:
    n: int
    opcode: torch.Tensor
    xid: torch.Tensor
    arg: torch.Tensor
    path_off: torch.Tensor
    path_len: torch.Tensor
    data_off: torch.Tensor
    data_len: torch.Tensor
    acl_id: torch.Tensor
    path_arena: torch.Tensor
    data_arena: torch.Tensor
    acl_off: torch.Tensor
    acl_len: torch.Tensor
    acl_arena: torch.Tensor

    def tensors(self):
        """The descriptor list torch.ops.zkmi takes (zk_abi.h order)."""
        return [self.opcode, self.xid, self.arg, self.path_off,
                self.path_len, self.data_off, self.data_len, self.acl_id,
                self.path_arena, self.data_arena, self.acl_off, self.acl_len,
                self.acl_arena]


def _acl_bytes(acl):
    w = jute.JuteWriter()
    w.write_acl(acl)
    return w.getvalue()


def pack_requests(pkts, device=None):
    """Host packing of request dicts (as :func:`zkmi.jute.encode_request`
    takes them) into a device :class:`RequestBatch`.  Used by tests and by
    the client's batched API; the benchmark builds its batches on the GPU."""
    n = len(pkts)
    opcode = np.zeros(n, np.int32)
    xid = np.zeros(n, np.int32)
    arg = np.zeros(n, np.int32)
    path_off = np.zeros(n, np.int64)
    path_len = np.zeros(n, np.int32)
    data_off = np.zeros(n, np.int64)
    data_len = np.zeros(n, np.int32)
    acl_id = np.zeros(n, np.int32)
    parena = bytearray()
    darena = bytearray()
    acls = {}
    acl_blobs = []
    for i, p in enumerate(pkts):
        op = p['opcode']
        opcode[i] = consts.OP_CODES[op]
        xid[i] = p['xid']
        path = p.get('path', '').encode('utf-8')
        path_off[i] = len(parena)
        path_len[i] = len(path)
        parena += path
        d = p.get('data', b'') or b''
        data_off[i] = len(darena)
        data_len[i] = len(d)
        darena += d
        if op in ('GET_DATA', 'EXISTS', 'GET_CHILDREN', 'GET_CHILDREN2'):
            arg[i] = 1 if p.get('watch') else 0
        elif op == 'CREATE':
            arg[i] = jute.flags_to_mask(p.get('flags', []))
            blob = _acl_bytes(p.get('acl', []))
            if blob not in acls:
                acls[blob] = len(acl_blobs)
                acl_blobs.append(blob)
            acl_id[i] = acls[blob]
        elif op in ('DELETE', 'SET_DATA'):
            arg[i] = p.get('version', -1)
    if not acl_blobs:
        acl_blobs.append(_acl_bytes([]))
    aoff = np.zeros(len(acl_blobs), np.int64)
    alen = np.zeros(len(acl_blobs), np.int32)
    aarena = bytearray()
    for k, b in enumerate(acl_blobs):
        aoff[k] = len(aarena)
        alen[k] = len(b)
        aarena += b
    dev = _dev(device)

    def T(a):
        return torch.from_numpy(a).to(dev)

    def B(b):
        a = np.frombuffer(bytes(b) if b else b'\0', np.uint8)
        return torch.from_numpy(a.copy()).to(dev)
    return RequestBatch(n, T(opcode), T(xid), T(arg), T(path_off),
                        T(path_len), T(data_off), T(data_len), T(acl_id),
                        B(parena), B(darena), T(aoff), T(alen), B(aarena))


def _total_err(dev):
    """The encoders' (total, err) device scalars.  Both are written whole
    by the encode (scan / writer's block 0, or a memset for an empty
    batch), so no fill launch precedes it."""
    z = torch.empty(2, dtype=I64, device=dev)
    return z[0:1], z[1:2].view(I32)[0:1]


def encode_requests(batch, xid_table=None, out=None, stream=None,
                    terminate=False, presized=None):
    """K10: encode ``batch`` into one framed byte stream.

    Returns ``(stream_bytes, rec_off, total)`` — ``total`` is a device
    int64 scalar; ``stream_bytes`` is the full output buffer (use
    ``[:total]``).  When ``out`` is None a buffer sized on the host from the
    batch is allocated (one small D2H copy).  ``terminate``: four 0xFF bytes
    follow the stream when they fit, so :func:`frame_scan` over any host
    upper bound of its length stops exactly at its end (BAD_LENGTH there).
    ``presized`` = (sizes, bsum): the batch's producer already wrote each
    frame's bytes and each 256-request block's sum (``bench_gen_get``), so
    the encode skips its sizes pass."""
    L = _lib.lib()
    n = batch.n
    dev = batch.opcode.device
    sizes = presized[0] if presized is not None else \
        torch.empty(max(n, 1), dtype=I64, device=dev)
    rec_off = torch.empty(max(n, 1), dtype=I64, device=dev)
    total, err = _total_err(dev)
    ws = torch.empty(L.scan_workspace(max(n, 1)), dtype=I64, device=dev)
    if out is None:
        # Upper bound: 4+8 header, 4+path, 4+data, acl, 8 ints.
        ub = int(n * 40 + batch.path_arena.numel() + batch.data_arena.numel()
                 + int(batch.acl_len.max().item() if n else 0) * max(n, 1))
        out = torch.empty(max(ub, 16), dtype=U8, device=dev)
    tab = xid_table.tab if xid_table is not None else None
    mask = xid_table.mask if xid_table is not None else 0
    with _on(stream):
        if presized is not None:
            L.encode_requests_presized(batch.tensors(), n, sizes, presized[1],
                                       rec_off, total, ws, out, tab, mask,
                                       err, bool(terminate))
        else:
            L.encode_requests(batch.tensors(), n, sizes, rec_off, total, ws,
                              out, tab, mask, err, bool(terminate))
    return out, rec_off[:n], total, err


def _on(stream):
    """Context running the ops on ``stream`` (None: the current one)."""
    import contextlib
    return torch.cuda.stream(stream) if stream is not None else \
        contextlib.nullcontext()


def encode_set_watches(rel_zxid, data_paths, exist_paths, child_paths,
                       device=None, stream=None):
    """K11: one SET_WATCHES frame (xid -8) for three path lists."""
    L = _lib.lib()
    dev = _dev(device)
    paths = list(data_paths) + list(exist_paths) + list(child_paths)
    n = len(paths)
    arena = bytearray()
    poff = np.zeros(max(n, 1), np.int64)
    plen = np.zeros(max(n, 1), np.int32)
    for i, p in enumerate(paths):
        b = p.encode('utf-8')
        poff[i] = len(arena)
        plen[i] = len(b)
        arena += b
    t_poff = torch.from_numpy(poff).to(dev)
    t_plen = torch.from_numpy(plen).to(dev)
    t_ar = torch.from_numpy(np.frombuffer(bytes(arena) or b'\0',
                                          np.uint8).copy()).to(dev)
    sizes = torch.empty(max(n, 1), dtype=I64, device=dev)
    off = torch.zeros(max(n, 1), dtype=I64, device=dev)
    total = torch.zeros(1, dtype=I64, device=dev)
    ws = torch.empty(L.scan_workspace(max(n, 1)), dtype=I64, device=dev)
    cap = 64 + len(arena) + 4 * n
    out = torch.empty(cap, dtype=U8, device=dev)
    err = torch.zeros(1, dtype=I32, device=dev)
    with _on(stream):
        L.encode_set_watches(t_poff, t_plen, t_ar, n, len(data_paths),
                             len(exist_paths), rel_zxid, sizes, off, total,
                             ws, out, err)
    frame_len = 32 + len(arena) + 4 * n
    return out[:frame_len]


# ---------------------------------------------------------------------------
# K9 handshake records (batched across a node's sessions)
# ---------------------------------------------------------------------------

def encode_connect_requests(reqs, device=None, stream=None):
    """``reqs``: list of dicts as :func:`zkmi.jute.encode_connect_request`
    takes them.  Returns the framed stream (uint8 device tensor)."""
    L = _lib.lib()
    dev = _dev(device)
    n = len(reqs)
    arena = bytearray()
    pwo, pwl = [], []
    for r in reqs:
        pw = r.get('passwd', b'\0' * 8)
        pwo.append(len(arena))
        pwl.append(len(pw))
        arena += pw
    T = lambda v, dt: torch.tensor(v, dtype=dt, device=dev)  # noqa: E731
    proto = T([r.get('protocolVersion', 0) for r in reqs], I32)
    zx = T([r.get('lastZxidSeen', 0) for r in reqs], I64)
    tmo = T([r['timeOut'] for r in reqs], I32)
    sid = T([r.get('sessionId', 0) for r in reqs], I64)
    t_pwo, t_pwl = T(pwo, I64), T(pwl, I32)
    t_ar = torch.from_numpy(np.frombuffer(bytes(arena) or b'\0',
                                          np.uint8).copy()).to(dev)
    sizes = torch.empty(max(n, 1), dtype=I64, device=dev)
    off = torch.empty(max(n, 1), dtype=I64, device=dev)
    total = torch.zeros(1, dtype=I64, device=dev)
    ws = torch.empty(L.scan_workspace(max(n, 1)), dtype=I64, device=dev)
    size = n * 32 + len(arena)           # frame len + 28 fixed + passwd
    cap = size + 16
    out = torch.empty(cap, dtype=U8, device=dev)
    with _on(stream):
        L.encode_connect_requests(proto, zx, tmo, sid, t_pwo, t_pwl, t_ar, n,
                                  sizes, off, total, ws, out)
    return out[:size]


def decode_connect_responses(buf, frames, n, stream=None):
    """Decode ``n`` ConnectResponse frames -> dict of device tensors
    (protocolVersion, timeOut, sessionId, passwd_off, passwd_len, status)."""
    L = _lib.lib()
    dev = buf.device
    e = lambda dt: torch.empty(max(n, 1), dtype=dt, device=dev)  # noqa
    o = {'protocolVersion': e(I32), 'timeOut': e(I32), 'sessionId': e(I64),
         'passwd_off': e(I64), 'passwd_len': e(I32), 'status': e(I32)}
    with _on(stream):
        L.decode_connect_responses(
            buf, frames.off, frames.length, n, o['protocolVersion'],
            o['timeOut'], o['sessionId'], o['passwd_off'], o['passwd_len'],
            o['status'])
    return {k: v[:n] for k, v in o.items()}


# ---------------------------------------------------------------------------
# K1 frame scan
# ---------------------------------------------------------------------------

@dataclass
class FrameTable:
    off: torch.Tensor        # int64 [cap] body offsets
    length: torch.Tensor     # int32 [cap] body lengths
    result: torch.Tensor     # int64 [4]: n_frames, consumed, bad, overflow

    @property
    def count(self):
        return self.result[0:1]

    def host_result(self):
        r = self.result.cpu().tolist()
        return {'frames': r[0], 'consumed': r[1], 'bad': bool(r[2]),
                'overflow': bool(r[3])}


FS_WINDOWS = (256, 512, 1024, 2048)
# frame_window() values with this bit ask K1 for its long-frame mode: the
# window is below the stream's largest frame, so fs_tile runs its frontier
# again past the window when a long frame leaves no walker alive, and takes
# survivor exits past the window as the next tile's entry
FS_WIN_LONG = 1 << 16
# the largest window chosen on its own.  Round 3's frontier made a 2 KiB
# window dear (32 walkers a lane) and capped it at 1 KiB; with the chain map
# the window only widens the entry positions, and long-frame mode at 1 KiB
# left a 0-1024 B GET reply stream (frames to 1116 B) without speculation
# in hundreds of tiles: 750.7 us a scan at a 1 KiB cap, 244.2 us at 2 KiB
# (profiles/r4_k1_microbench.md)
FS_WINDOW_AUTO_MAX = 2048


def frame_window(max_frame):
    """The K1 entry window for a stream whose frames are at most
    ``max_frame`` bytes (length prefix included): the smallest window
    covering them, up to 2 KiB; past that (or past the module's
    ``FS_WINDOW_AUTO_MAX``, which a test lowers) the window is the cap in
    long-frame mode.  Frames longer than the window are framed exactly
    either way."""
    cap = FS_WINDOW_AUTO_MAX
    cap = min(max(cap, FS_WINDOWS[0]), FS_WINDOWS[-1])
    for w in FS_WINDOWS:
        if max_frame <= w and w <= cap:
            return w
    top = max(w for w in FS_WINDOWS if w <= cap)
    return top | FS_WIN_LONG


def _scan_len(buf, n):
    """(device length pointer or None, capacity) of a K1 call: ``n`` is a
    host int (scan ``buf[:n]``) or a device int64 scalar tensor holding the
    length (an encoder's ``total``; the scan reads it on the GPU and
    covers at most ``buf.numel()`` bytes)."""
    if n is None:
        return None, buf.numel()
    if isinstance(n, torch.Tensor):
        if n.dtype != I64 or n.device != buf.device or n.numel() < 1:
            raise TypeError('frame_scan: device length must be an int64 '
                            'tensor on the buffer\'s device')
        return n, buf.numel()
    n = int(n)
    if n > buf.numel():
        raise ValueError('frame_scan: n=%d past the buffer (%d bytes)'
                         % (n, buf.numel()))
    return None, n


class FrameScanner:
    """Reusable K1 state for a stream that is scanned again and again (a
    connection's RX ring, the benchmark's request / reply streams): the
    workspace and the frame table are allocated once and grown on demand,
    so a scan issued right after a host read-back starts with one launch
    instead of four allocations."""

    def __init__(self, cap, device, window=2048,
                 max_packet=consts.MAX_PACKET, frame_hint=None, group=None):
        self.cap = cap
        self.window = window
        # the stream's usual frame size: >= 128 bytes within a small window
        # lets a wave take a group of tiles (the chain map once, then the
        # chain walked on; csrc/kernels/frame_scan.hip fs_group_rest).
        # GET reply stream (192-byte frames): 8 tiles a wave 77.4 us, 4
        # tiles 93.0 us (profiles/r4_k1_microbench.md)
        if group is None:
            group = _FS_GROUP if frame_hint is not None and \
                frame_hint >= 128 else 1
        self.group = group
        self.max_packet = max_packet
        self.table = FrameTable(torch.empty(cap, dtype=I64, device=device),
                                torch.empty(cap, dtype=I32, device=device),
                                torch.empty(4, dtype=I64, device=device))
        self.ws = torch.empty(0, dtype=U8, device=device)
        self.ws_for = -1            # stream length the workspace covers
        self.clean_for = -1         # n_cap whose flags the last scan cleared

    def scan(self, buf, n, stream=None, nospec=False, misspec=0):
        """Frame ``buf[:n]``; ``n`` may be a device int64 length (see
        :func:`frame_scan`) — then nothing is read back to the host.
        ``nospec`` (tests): no tile takes a speculated entry, every link
        goes through the repair; ``misspec`` = P > 0 (tests): every P-th
        tile takes a garbage entry (one byte past the speculated one)."""
        L = _lib.lib()
        n_dev, ncap = _scan_len(buf, n)
        if ncap > self.ws_for:
            cover = max(ncap, 2 * self.ws_for)
            wsb = L.frame_scan_workspace(cover)
            self.ws = torch.empty(max(wsb, 256), dtype=U8,
                                  device=buf.device)
            self.ws_for = cover
            self.clean_for = -1
        t = self.table
        # a scan leaves its workspace's flags cleared for the next scan over
        # the same capacity (the layout depends on it): no memset then
        with _on(stream):
            L.frame_scan(buf, n_dev, ncap, self.max_packet, self.ws, t.off,
                         t.length, t.result, int(self.window),
                         ncap == self.clean_for,
                         (1 if nospec else 0) | (int(misspec) << 8) |
                         ((self.group - 1) << 4))
        self.clean_for = ncap
        self.last_cap = ncap
        return t

    def chain_stats(self, stream=None):
        """K1 chain counters (host sync) accumulated over this scanner's
        scans since the previous call (a reused workspace skips the memset
        that used to reset them per scan): tiles without a speculated
        entry, tiles re-walked, repair rounds, tiles fs_link's chases
        looked up in fs_tile's candidate exits."""
        if getattr(self, 'last_cap', None) is None:      # no scan yet
            return {'no_spec': 0, 'rewalked': 0, 'rounds': 0, 'looked_up': 0}
        with _on(stream):
            out = _lib.lib().frame_scan_stats(self.ws, self.last_cap,
                                              int(self.window))
        return {'no_spec': out[0], 'rewalked': out[1], 'rounds': out[2],
                'looked_up': out[3]}


def frame_scan(buf, n=None, max_packet=consts.MAX_PACKET, cap=None,
               stream=None, workspace=None, window=2048):
    """K1: split ``buf[:n]`` (uint8 device tensor) into frames.

    ``n``: a host int, or a device int64 tensor holding the stream length
    (e.g. the ``total`` an encoder returned): the scan then reads it on the
    GPU, covers at most ``buf.numel()`` bytes and needs no host sync.
    ``cap`` bounds the frame table (default: a quarter of the bytes, the
    most frames they can hold).  ``window`` is the per-tile fast-path entry
    window (256..2048 bytes, see :func:`frame_window`): a hint for the usual
    frame size, never a limit — longer frames are framed exactly on a
    slower path.  (:class:`FrameScanner` keeps the buffers across calls.)"""
    L = _lib.lib()
    n_dev, ncap = _scan_len(buf, n)
    dev = buf.device
    if cap is None:
        cap = max(ncap // 4, 1)
    wsb = L.frame_scan_workspace(ncap)
    if workspace is None or workspace.numel() < wsb:
        workspace = torch.empty(max(wsb, 256), dtype=U8, device=dev)
    off = torch.empty(cap, dtype=I64, device=dev)
    ln = torch.empty(cap, dtype=I32, device=dev)
    res = torch.empty(4, dtype=I64, device=dev)     # zeroed by the kernels
    with _on(stream):
        L.frame_scan(buf, n_dev, ncap, max_packet, workspace, off, ln, res,
                     int(window))
    return FrameTable(off, ln, res)


# ---------------------------------------------------------------------------
# K2-K8 reply decode
# ---------------------------------------------------------------------------

STAT64 = ('czxid', 'mzxid', 'ctime', 'mtime', 'ephemeralOwner', 'pzxid')
STAT32 = ('version', 'cversion', 'aversion', 'dataLength', 'numChildren')


@dataclass
class ReplyBatch:
    xid: torch.Tensor
    err: torch.Tensor
    opcode: torch.Tensor
    status: torch.Tensor
    zxid: torch.Tensor
    stat64: torch.Tensor     # [6, cap]
    stat32: torch.Tensor     # [5, cap]
    pay_off: torch.Tensor
    pay_len: torch.Tensor
    aux0: torch.Tensor
    aux1: torch.Tensor
    count: torch.Tensor      # device int64 [1]

    def tensors(self):
        """The reply table list torch.ops.zkmi takes (ZkReplyOut order)."""
        return [self.xid, self.err, self.opcode, self.status, self.zxid,
                self.stat64, self.stat32, self.pay_off, self.pay_len,
                self.aux0, self.aux1]


def alloc_replies(cap, device):
    dev = _dev(device)
    return ReplyBatch(
        torch.empty(cap, dtype=I32, device=dev),
        torch.empty(cap, dtype=I32, device=dev),
        torch.empty(cap, dtype=I32, device=dev),
        torch.empty(cap, dtype=I32, device=dev),
        torch.empty(cap, dtype=I64, device=dev),
        torch.zeros(6, cap, dtype=I64, device=dev),
        torch.zeros(5, cap, dtype=I32, device=dev),
        torch.empty(cap, dtype=I64, device=dev),
        torch.empty(cap, dtype=I32, device=dev),
        torch.empty(cap, dtype=I32, device=dev),
        torch.empty(cap, dtype=I32, device=dev),
        None)


def decode_replies(buf, frames, xid_table, out=None, stream=None,
                   check=None, tick=None):
    """K2-K8: decode every frame of ``frames`` as a reply.

    ``check = (idx, xid, data_len, acc[, slab, slot_off])``: also count, in
    the same kernel, the replies that are clean GET_DATA successes for the
    requests sent (request i = node idx[i] with xid[i]; czxid idx + 1 and
    the node's data length) into ``acc`` (int64, 1..64 slots the caller
    sums); with the tree's ``slab`` / ``slot_off`` one reply in 16 (rotating
    with ``tick``) must also carry its node's payload bytes.  ``tick``
    (int64 [2], with ``check``): ``tick[1]`` advances by one in the same
    kernel (the device step counter of a captured pipeline)."""
    L = _lib.lib()
    cap = frames.off.numel()
    if out is None:
        out = alloc_replies(cap, buf.device)
    out.count = frames.count
    with _on(stream):
        if check is None:
            L.decode_replies(buf, frames.off, frames.length, frames.count,
                             xid_table.tab, xid_table.mask, out.tensors())
        else:
            idx, xid, data_len, acc = check[:4]
            slab, slot_off = check[4:6] if len(check) > 4 else (None, None)
            L.decode_replies_check(buf, frames.off, frames.length,
                                   frames.count, xid_table.tab,
                                   xid_table.mask, out.tensors(), idx, xid,
                                   data_len, acc, tick, slab, slot_off)
    return out


def exclusive_scan(x, stream=None):
    """Device-wide exclusive prefix sum of an int32/int64 vector -> (int64
    prefix, int64 total).  The engine (MFMA byte-plane or shuffle) is the
    one selected by :func:`zkmi.ops._lib.set_scan_mode`."""
    L = _lib.lib()
    n = x.numel()
    dev = x.device
    base = torch.empty(max(n, 1), dtype=I64, device=dev)
    total = torch.zeros(1, dtype=I64, device=dev)
    ws = torch.empty(L.scan_workspace(max(n, 1)), dtype=I64, device=dev)
    if x.dtype not in (torch.int32, torch.int64):
        raise TypeError('exclusive_scan: int32 or int64 input')
    with _on(stream):
        L.scan_excl(x, base, total, ws)
    return base[:n], total


def _scan_i32(counts, stream=None):
    L = _lib.lib()
    n = counts.numel()
    dev = counts.device
    base = torch.empty(max(n, 1), dtype=I64, device=dev)
    total = torch.zeros(1, dtype=I64, device=dev)
    ws = torch.empty(L.scan_workspace(max(n, 1)), dtype=I64, device=dev)
    with _on(stream):
        L.scan_excl(counts, base, total, ws)
    return base, total


def expand_strings(buf, region, count, stream=None):
    """Ragged string vectors (children lists) -> (row_base, off, len)."""
    L = _lib.lib()
    n = region.numel()
    base, total = _scan_i32(count, stream)
    m = int(total.item())
    soff = torch.empty(max(m, 1), dtype=I64, device=buf.device)
    slen = torch.empty(max(m, 1), dtype=I32, device=buf.device)
    with _on(stream):
        L.expand_strings(buf, region, count, base[:n], soff, slen)
    return base[:n], soff[:m], slen[:m]


def expand_acl(buf, region, count, stream=None):
    """Ragged ACL vectors -> (row_base, perms, scheme off/len, id off/len)."""
    L = _lib.lib()
    n = region.numel()
    base, total = _scan_i32(count, stream)
    m = int(total.item())
    dev = buf.device
    perms = torch.empty(max(m, 1), dtype=I32, device=dev)
    so = torch.empty(max(m, 1), dtype=I64, device=dev)
    sl = torch.empty(max(m, 1), dtype=I32, device=dev)
    io = torch.empty(max(m, 1), dtype=I64, device=dev)
    il = torch.empty(max(m, 1), dtype=I32, device=dev)
    with _on(stream):
        L.expand_acl(buf, region, count, base[:n], perms, so, sl, io, il)
    return base[:n], perms[:m], so[:m], sl[:m], io[:m], il[:m]


# ---------------------------------------------------------------------------
# K12 / K13 server mode
# ---------------------------------------------------------------------------

@dataclass
class RequestTable:
    xid: torch.Tensor
    opcode: torch.Tensor
    status: torch.Tensor
    path_off: torch.Tensor
    path_len: torch.Tensor
    data_off: torch.Tensor
    data_len: torch.Tensor
    arg: torch.Tensor
    vec_off: torch.Tensor
    vec_count: torch.Tensor
    rel_zxid: torch.Tensor
    count: torch.Tensor

    def tensors(self):
        """The request table list torch.ops.zkmi takes (ZkReqOut order)."""
        return [self.xid, self.opcode, self.status, self.path_off,
                self.path_len, self.data_off, self.data_len, self.arg,
                self.vec_off, self.vec_count, self.rel_zxid]


def alloc_request_table(cap, device):
    dev = _dev(device)
    e32 = lambda: torch.empty(cap, dtype=I32, device=dev)  # noqa: E731
    e64 = lambda: torch.empty(cap, dtype=I64, device=dev)  # noqa: E731
    return RequestTable(e32(), e32(), e32(), e64(), e32(), e64(), e32(),
                        e32(), e64(), e32(), e64(), None)


def decode_requests(buf, frames, out=None, stream=None):
    L = _lib.lib()
    cap = frames.off.numel()
    if out is None:
        out = alloc_request_table(cap, buf.device)
    out.count = frames.count
    with _on(stream):
        L.decode_requests(buf, frames.off, frames.length, frames.count,
                          out.tensors())
    return out


@dataclass
class ResponseBatch:
    opcode: torch.Tensor
    xid: torch.Tensor
    err: torch.Tensor
    node: torch.Tensor
    zxid: torch.Tensor
    path_off: torch.Tensor
    path_len: torch.Tensor
    path_arena: torch.Tensor
    aux: torch.Tensor
    count: torch.Tensor
    slot: torch.Tensor = None   # slot offsets (from the tree lookup) or None

    def tensors(self):
        """The reply descriptor list torch.ops.zkmi takes (ZkRespBatch
        order; ``slot`` goes separately, it is optional)."""
        return [self.opcode, self.xid, self.err, self.node, self.zxid,
                self.path_off, self.path_len, self.path_arena, self.aux]


def response_workspace(cap, device):
    """(sizes, scan workspace) a producer fills for a presized
    :func:`encode_responses` (zk_tree_serve writes both)."""
    L = _lib.lib()
    return (torch.empty(cap, dtype=I64, device=device),
            torch.empty(L.scan_workspace(cap), dtype=I64, device=device))


def encode_responses(resp, store, out_cap, out=None, stream=None,
                     presized=None, terminate=False, stage=0,
                     total_err=None, prescanned=False):
    """K13: server-mode reply encode -> (bytes, rec_off, total, err).
    ``store``: the node store's tensors [slab, slot_off, data_len,
    slot_cap] (:attr:`zkmi.bench.synthetic.GpuTree.store`).
    ``presized``: the (sizes, workspace) pair of :func:`response_workspace`
    already filled by the producer; the sizes pass is then skipped.
    ``stage``: LDS bytes per workgroup (0: the encoder's default; uniform
    GET_DATA replies need only 8 KiB, more workgroups then fit a CU).
    ``total_err``: the (total, err) pair to write (default: new ones);
    ``prescanned``: the presized workspace's block bases and ``total`` were
    already computed (the tree's finish_scan launch)."""
    L = _lib.lib()
    cap = resp.opcode.numel()
    dev = resp.opcode.device
    if presized is not None:
        sizes, ws = presized
    else:
        sizes = torch.empty(cap, dtype=I64, device=dev)
        ws = torch.empty(L.scan_workspace(cap), dtype=I64, device=dev)
    rec_off = torch.empty(cap, dtype=I64, device=dev)
    total, err = total_err if total_err is not None else _total_err(dev)
    if out is None:
        out = torch.empty(out_cap, dtype=U8, device=dev)
    with _on(stream):
        L.encode_responses(resp.tensors(), resp.slot, list(store), resp.count,
                           cap, sizes, rec_off, total, ws, out, err,
                           presized is not None, bool(terminate),
                           int(stage), bool(prescanned))
    return out, rec_off, total, err


# ---------------------------------------------------------------------------
# Host views (tests, the client's batched API)
# ---------------------------------------------------------------------------

def replies_to_packets(buf, replies, n=None, children=None, acls=None):
    """Convert a decoded :class:`ReplyBatch` to the dicts
    :func:`zkmi.jute.decode_response` produces (for parity checks and for
    the client's batched calls)."""
    if n is None:
        n = int(replies.count.item())
    hb = bytes(buf.cpu().numpy().tobytes())
    cols = {k: getattr(replies, k)[:n].cpu().tolist() for k in (
        'xid', 'err', 'opcode', 'status', 'zxid', 'pay_off', 'pay_len',
        'aux0', 'aux1')}
    s64 = replies.stat64[:, :n].cpu().tolist()
    s32 = replies.stat32[:, :n].cpu().tolist()
    out = []
    for i in range(n):
        st = cols['status'][i]
        op = consts.OP_CODE_LOOKUP.get(cols['opcode'][i])
        if st != 0:
            out.append({'xid': cols['xid'][i], 'status': st})
            continue
        err = consts.ERR_LOOKUP.get(cols['err'][i], cols['err'][i])
        pkt = {'xid': cols['xid'][i], 'zxid': cols['zxid'][i], 'err': err,
               'opcode': op}
        if err == 'OK':
            po, pl = cols['pay_off'][i], cols['pay_len'][i]

            def stat():
                return jute.Stat(s64[0][i], s64[1][i], s64[2][i], s64[3][i],
                                 s32[0][i], s32[1][i], s32[2][i], s64[4][i],
                                 s32[3][i], s32[4][i], s64[5][i])
            if op == 'GET_DATA':
                pkt['data'] = hb[po:po + pl]
                pkt['stat'] = stat()
            elif op in ('EXISTS', 'SET_DATA'):
                pkt['stat'] = stat()
            elif op == 'CREATE':
                pkt['path'] = hb[po:po + pl].decode('utf-8')
            elif op in ('GET_CHILDREN', 'GET_CHILDREN2'):
                r = jute.JuteReader(hb, po, po + pl)
                pkt['children'] = [r.read_ustring()
                                   for _ in range(cols['aux0'][i])]
                if op == 'GET_CHILDREN2':
                    pkt['stat'] = stat()
            elif op == 'GET_ACL':
                r = jute.JuteReader(hb, po - 4, po + pl)
                pkt['acl'] = r.read_acl()
                pkt['stat'] = stat()
            elif op == 'NOTIFICATION':
                pkt['type'] = consts.NOTIFICATION_TYPE_LOOKUP.get(
                    cols['aux0'][i], cols['aux0'][i])
                pkt['state'] = consts.STATE_LOOKUP.get(cols['aux1'][i],
                                                       cols['aux1'][i])
                pkt['path'] = hb[po:po + pl].decode('utf-8')
        out.append(pkt)
    return out
