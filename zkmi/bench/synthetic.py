"""GPU-resident synthetic ZooKeeper workload: a 1M-znode tree in HBM and the
full wire pipeline around it.

One :meth:`GetPipeline.step` performs, entirely on the GPU and on the real
ZooKeeper wire format:

  client  K10 encode B GET_DATA requests (paths gathered straight from the
          tree's path arena, xids recorded in the HBM xid->opcode table)
  server  K1 frame-scan the request stream, K12 decode the requests, hash
          lookup in the tree, K13 encode GET_DATA replies (header + data +
          Stat) into the reply stream
  client  K1 frame-scan the reply stream, K2/K3/K4 decode header, opcode
          (via the xid table), data (offset/length) and Stat

plus a device-side check that every reply is OK and carries the node the
request asked for.  Nothing is skipped inside a step, and a step makes no
device-to-host read: K1 reads each stream's length from the device-side
byte count its encoder produced (``total``), so any frame-size mix scans
sync-free and no byte past a stream's end is walked.

:class:`MixPipeline` does the same for the create/set/delete mix with
version CAS and ACL encode (BASELINE config 3).
"""

import os
import time

import numpy as np
import torch

from .. import consts
from ..ops import _lib
from ..ops import batch as B

I64, I32, U8 = torch.int64, torch.int32, torch.uint8

# ZKMI_SERVE_TICKETS=1: the serve launch's last workgroup does the tree
# finish (sign-off tickets) instead of a tree_finish_k launch.  Off by
# default: every workgroup's release fence costs an L2 writeback on a
# multi-XCD part — tree_serve 90 -> 231 us, the GET step 0.651 -> 0.718 ms
# (profiles/r5_regression_ab.md); the extra launch is far cheaper.
_SERVE_TICKETS = os.environ.get('ZKMI_SERVE_TICKETS', '0') == '1'
# ZKMI_GET_STAGE: the LDS bytes per workgroup the GET pipelines' reply
# encode asks for (0: the encoder's 28 KiB).  Uniform GET replies need only
# the writer's 7 KiB header table, but 8 KiB measured no faster for them
# (0.581 vs 0.581 ms) and slowed variable payloads, whose replies go
# through the LDS image (uniform 0-200 B 0.710 -> 0.972 ms,
# profiles/r5_get_stage_ab.log): off.
_GET_STAGE = int(os.environ.get('ZKMI_GET_STAGE', '0'))
# ZKMI_SERVE_RO=0: the GET pipelines serve with the general serve kernel
# instead of its read-only instance
_SERVE_RO = os.environ.get('ZKMI_SERVE_RO', '1') == '1'
# ZKMI_FREE_COMPACT=0: no free-ring compaction after write batches (trees
# built with compact_free=True; GpuTree.free_compact)
_FREE_COMPACT = os.environ.get('ZKMI_FREE_COMPACT', '1') == '1'
# ZKMI_FINISH_SCAN=0: the tree finish and the reply encode's block-sum scan
# as two launches again (tree_finish_scan_k runs them as one)
_FINISH_SCAN = os.environ.get('ZKMI_FINISH_SCAN', '1') == '1'
# the largest batch tree_seq_order numbers
_SEQ_MAX = 1 << 24
# ZKMI_GET_PRESIZED=0: the GET pipelines' request encode runs its own sizes
# pass instead of taking the generator's (bench_gen_get sizes / bsum)
_GET_PRESIZED = os.environ.get('ZKMI_GET_PRESIZED', '1') == '1'
# ZKMI_STORM_STREAMS=1: the one-member storm step on one stream (its
# handshake and expiry no longer beside the encode / the reply decode)
_STORM_STREAMS = os.environ.get('ZKMI_STORM_STREAMS', '2') != '1'
# ZKMI_SRV_GROUP: K1 tiles a wave on the GPU server's request streams, for
# every workload (unset: the defaults below).  Request streams of equal-
# sized frames without length-like words take groups (the groups' walk
# steps over a run of equal frames): GET 4 tiles a wave (0.5255 vs 0.5337
# ms a step at 1), the storm's identical creates 8 (1.298 vs 1.316 at 4,
# 1.344 at 1; profiles/r6_srv_group_ab.log,
# r6_srv_group_storm_mix_ab.log).  The others stay at one: SET_DATA
# versions read as frame lengths make phantom chains, which the per-tile
# maps settle and a group's walked tiles do not (the watch workload's
# version-84 step took 32.6 ms against a 2.4 ms median at 4 tiles a wave,
# tests/test_watch_sustained.py; mix gained 1.2 % at 4).
_SRV_GROUP_ENV = (int(os.environ['ZKMI_SRV_GROUP'])
                  if os.environ.get('ZKMI_SRV_GROUP') else None)
_SRV_GROUP = _SRV_GROUP_ENV
_GET_SRV_GROUP = _SRV_GROUP_ENV or 4
_STORM_SRV_GROUP = _SRV_GROUP_ENV or 8


def _len(total):
    """A stream length for K1: the encoder's device total (no host read)."""
    return total



def _next_pow2(x):
    p = 1
    while p < x:
        p <<= 1
    return p


NODE_FREE = -2           # node_parent of an unused node (tree.hip)


def path_owner(paths, world):
    """Owner rank of every path: FNV-1a 32 of the bytes mod ``world`` —
    the host mirror of csrc/kernels/route.hip's router."""
    out = np.empty(len(paths), np.int64)
    by_len = {}
    for i, p in enumerate(paths):
        by_len.setdefault(len(p), []).append(i)
    for ln, ids in by_len.items():
        m = np.frombuffer(b''.join(paths[i] for i in ids),
                          np.uint8).reshape(len(ids), ln) if ln else \
            np.zeros((len(ids), 0), np.uint8)
        h = np.full(len(ids), 2166136261, np.uint64)
        for k in range(ln):
            h = ((h ^ m[:, k]) * np.uint64(16777619)) & np.uint64(0xffffffff)
        out[ids] = (h % np.uint64(world)).astype(np.int64)
    return out


def _i64(u):
    """A 64-bit unsigned seed as the signed int a torch op schema takes."""
    u &= (1 << 64) - 1
    return u - (1 << 64) if u >= (1 << 63) else u


def slot_bytes(data_cap):
    """Bytes of one wire-format node slot (zk_batch.h ZkNodeStore)."""
    return _lib.SLOT_DATA + ((data_cap + 15) & ~15) + 4


class GpuTree(object):
    """``n_nodes`` znodes ``/bench/dDDDDD/nNNNNNNNN`` (``fanout`` children per
    directory) with ``data_bytes`` of random data each.  Node ``v`` has
    ``czxid == v + 1``."""

    def __init__(self, n_nodes=1_000_000, data_bytes=100, fanout=1000,
                 device=None, spare=0.25, seed=0, shard=None, ctime_ms=None,
                 data_dist=None, name_pad=None, scratch=0, watch_cap=0,
                 hash_factor=2, compact_free=False):
        dev = torch.device(device) if device is not None else \
            torch.device('cuda', torch.cuda.current_device())
        self.device = dev
        L = _lib.lib()
        ndirs = (n_nodes + fanout - 1) // fanout
        # node order: 0 = /bench, 1..ndirs = dirs, then leaves
        paths = ['/bench'] + ['/bench/d%06d' % d for d in range(ndirs)]
        leaf0 = len(paths)
        # name_pad = (lo, hi): leaf names padded with a uniform lo..hi
        # characters (variable path lengths)
        rng = np.random.default_rng(seed + 17)
        if name_pad is not None:
            pad = rng.integers(name_pad[0], name_pad[1] + 1, n_nodes)
            paths += ['/bench/d%06d/n%09d%s' % (i // fanout, i, 'p' * pad[i])
                      for i in range(n_nodes)]
        else:
            paths += ['/bench/d%06d/n%09d' % (i // fanout, i)
                      for i in range(n_nodes)]
        nst = len(paths)
        parents = np.empty(nst, np.int64)
        parents[0] = -1
        parents[1:leaf0] = 0
        parents[leaf0:] = 1 + np.arange(n_nodes) // fanout
        self.n_static = nst
        self.leaf0 = leaf0
        self.n_leaves = n_nodes
        # data_dist = (lo, hi): leaf data lengths uniform in lo..hi bytes
        # (variable payloads); data_bytes is then the largest
        if data_dist is not None:
            leaf_dl = rng.integers(data_dist[0], data_dist[1] + 1,
                                   n_nodes).astype(np.int32)
            data_bytes = int(data_dist[1])
        self.data_bytes = data_bytes
        self.data_dist = data_dist
        cap = int(nst * (1 + spare)) + 1024
        self.cap = cap
        enc = [p.encode() for p in paths]
        plen = np.fromiter((len(e) for e in enc), np.int32, nst)
        poff = np.zeros(nst, np.int64)
        np.cumsum(plen[:-1], out=poff[1:])
        arena = b''.join(enc)
        # every spare node may need a fresh path (up to 64 bytes each, in
        # 16-byte multiples)
        self.path_cap = len(arena) + (cap - nst) * 80 + (1 << 16)
        self.path_arena = torch.zeros(self.path_cap, dtype=U8, device=dev)
        self.path_arena[:len(arena)] = torch.frombuffer(
            bytearray(arena), dtype=U8).to(dev)
        self.node_path_off = torch.zeros(cap, dtype=I64, device=dev)
        self.node_path_len = torch.zeros(cap, dtype=I32, device=dev)
        self.node_path_off[:nst] = torch.from_numpy(poff).to(dev)
        self.node_path_len[:nst] = torch.from_numpy(plen).to(dev)
        # bytes of each node's path storage (the static paths are packed)
        self.node_path_cap = torch.zeros(cap, dtype=I32, device=dev)
        self.node_path_cap[:nst] = self.node_path_len[:nst]
        # path word (offset << 24 | length) the hash lookups verify against
        self.node_pw = torch.zeros(cap, dtype=I64, device=dev)
        self.node_pw[:nst] = torch.from_numpy(
            (poff << 24) | plen.astype(np.int64)).to(dev)
        self.node_parent = torch.full((cap,), -1, dtype=I64, device=dev)
        self.node_parent[:nst] = torch.from_numpy(parents).to(dev)
        # wire-format slots; data capacity >= 128 so sets can grow
        dcap = max(data_bytes, 128)
        sb = slot_bytes(dcap)
        self.slot = sb
        self.slab_cap = cap * sb
        # hash vals pack node (32 bits) and slot offset / 16 (31 bits)
        assert cap < (1 << 31) and self.slab_cap < (1 << 35), 'tree too big'
        g = torch.Generator(device=dev)
        g.manual_seed(seed)
        # scratch: bytes past the tree's slab for the snapshots of ordered
        # serving (GpuServer.serve(ordered=True)); the tree's descriptor
        # sees slab[:slab_cap], the reply encoder the whole allocation
        scratch = (int(scratch) + 15) & ~15
        self.slab_all = torch.randint(0, 256, (self.slab_cap + scratch,),
                                      dtype=U8, device=dev, generator=g)
        self.slab = self.slab_all[:self.slab_cap]
        self.scratch = self.slab_all[self.slab_cap:] if scratch else None
        self.slot_off = torch.arange(cap, dtype=I64, device=dev) * sb
        self.data_len = torch.zeros(cap, dtype=I32, device=dev)
        if data_dist is not None:
            self.data_len[leaf0:nst] = torch.from_numpy(leaf_dl).to(dev)
        else:
            self.data_len[leaf0:nst] = data_bytes
        self.slot_cap = torch.full((cap,), dcap, dtype=I32, device=dev)
        nkids = np.zeros(nst, np.int32)
        nkids[0] = ndirs
        nkids[1:leaf0] = np.bincount(np.arange(n_nodes) // fanout,
                                     minlength=ndirs)[:ndirs]
        nk = torch.from_numpy(nkids).to(dev)
        # hash entries per node slot (a power of two above it): 2 keeps a
        # read-mostly tree's table under half full; a write-heavy one
        # (SEQUENTIAL names never reused) fills with tombstones between
        # rebuilds, and a wider table rebuilds less often
        # (capped at 2^28 entries, 16 GB, unless 2 a slot needs more: the
        # storm's replicated tree at 8 ranks holds ~25M node slots)
        hcap = max(min(_next_pow2(hash_factor * cap), 1 << 28),
                   _next_pow2(2 * cap))
        # 64-byte entries, empty = all zero bytes (csrc/kernels/tree.hip)
        self.ht = torch.zeros(_lib.HT_WORDS * hcap, dtype=I64, device=dev)
        cnt = [0] * _lib.TC_N
        cnt[_lib.TC_NODES], cnt[_lib.TC_ZXID] = nst, nst
        cnt[_lib.TC_PATH_TOP], cnt[_lib.TC_SLAB_TOP] = len(arena), nst * sb
        self.counters = torch.tensor(cnt, dtype=I64, device=dev)
        self.free_list = torch.empty(cap, dtype=I64, device=dev)
        # host-endian cversion / numChildren / pzxid shadows + dirty list
        # cversion << 32 | numChildren per node (one atomic per child write)
        self.cn = torch.zeros(cap, dtype=I64, device=dev)
        # ephemeralOwner per node, host-endian (session expiry scans it)
        self.eph = torch.zeros(cap, dtype=I64, device=dev)
        self.pzxid = torch.zeros(cap, dtype=I64, device=dev)
        self.dirty = torch.zeros(cap, dtype=I32, device=dev)
        self.dirty_list = torch.empty(cap, dtype=I64, device=dev)
        self.hcap = hcap
        # write workloads: the free ring's pending entries re-sorted after
        # every served batch (free_compact; ZKMI_FREE_COMPACT=0 turns it off)
        self.compact_free = compact_free and _FREE_COMPACT
        self.free_ws = None
        # the tree / node-store descriptor lists torch.ops.zkmi takes
        # (csrc/torch/zkmi_ops.cpp tree() / node_store() field order)
        self.store = [self.slab_all, self.slot_off, self.data_len,
                      self.slot_cap]
        self._tensors = [self.ht, self.node_path_off, self.node_path_len,
                         self.node_parent, self.path_arena, self.counters,
                         self.slab, self.slot_off, self.data_len,
                         self.slot_cap, self.free_list, self.cn,
                         self.pzxid, self.dirty, self.dirty_list,
                         self.node_pw, self.node_path_cap, self.eph]
        # watch table (watch_cap > 0): path-keyed one-shot watches of up to
        # 64 watcher slots (csrc/kernels/tree.hip wt_*); every serve of a
        # tree with one fires the watches its writes hit
        self.watch = None
        if watch_cap > 0:
            wh = _next_pow2(2 * int(watch_cap))
            self.watch = (torch.zeros(wh, dtype=I64, device=dev),
                          torch.zeros(2 * wh, dtype=I64, device=dev))
            self._tensors = self._tensors + list(self.watch)
        now = int(time.time() * 1000) if ctime_ms is None else ctime_ms
        L.tree_fill(self._tensors, 0, nst, nk, now)
        # shard = (rank, world): this replica indexes only the leaves whose
        # path hashes to `rank` (zkmi/parallel/sharded.py routes every read
        # there); the rest stay in the layout, unreachable by lookup
        self.shard = shard
        if shard is not None and shard[1] > 1:
            own = path_owner(enc[leaf0:], shard[1])
            gone = np.nonzero(own != shard[0])[0] + leaf0
            self.node_parent[torch.from_numpy(gone).to(dev)] = NODE_FREE
        L.tree_build(self._tensors, 0, nst)
        torch.cuda.synchronize(dev)

    @property
    def tensors(self):
        """The descriptor list of the tree for torch.ops.zkmi."""
        return self._tensors

    def expire(self, session, removed=None):
        """Delete every ephemeral node owned by ``session`` (server side of
        session expiry).  ``removed`` (device int64 [1]) accumulates the
        number of nodes removed."""
        if removed is None:
            removed = torch.zeros(1, dtype=I64, device=self.device)
        _lib.lib().tree_expire(self._tensors, session, self.cap, removed)
        return removed

    def rehash(self):
        """Rebuild the hash index from the live nodes (drops tombstones left
        by deleted paths that are never re-created, e.g. SEQUENTIAL names).
        One host read of the node high-water mark."""
        n = int(self.counters[_lib.TC_NODES].item())
        _lib.lib().tree_ht_reset(self._tensors)
        _lib.lib().tree_build(self._tensors, 0, min(n, self.cap))

    def digest(self):
        """(digest, live nodes, hash entries in use, tombstones): the digest
        is an order-independent hash of every live znode's path, czxid,
        mzxid, version, cversion / numChildren, pzxid, ephemeralOwner and
        data (times aside): two replicas of one tree agree on it whatever
        slots and hash entries their nodes sit in.  One host read."""
        out = torch.zeros(4, dtype=I64, device=self.device)
        _lib.lib().tree_digest(self._tensors, out)
        d, live, used, tomb = out.cpu().tolist()
        return d & ((1 << 64) - 1), live, used, tomb

    def free_compact(self):
        """Rebuild the free ring's pending entries as the free nodes in node
        order, on the device (csrc/kernels/tree.hip free_count_k): the next
        batch's creates take nodes from dense runs.  Capturable."""
        L = _lib.lib()
        if self.free_ws is None:
            self.free_ws = torch.empty(L.tree_free_workspace(self.cap),
                                       dtype=I64, device=self.device)
        L.tree_free_compact(self._tensors, self.free_ws)

    def free_order(self):
        """(pending free-ring entries, fraction of neighbours one apart):
        how much of the locality of the nodes the next creates get is left
        (one host read; probes)."""
        c = self.counters.cpu().tolist()
        h, pub = c[_lib.TC_FREE_HEAD], c[_lib.TC_FREE_PUB]
        if pub - h <= 1:
            return pub - h, 1.0
        idx = torch.arange(h, pub, device=self.device) % \
            self.free_list.numel()
        seg = self.free_list[idx]
        near = ((seg[1:] - seg[:-1]).abs() == 1).float().mean().item()
        return pub - h, near

    def sort_free(self):
        """Sort the pending entries of the free ring (the nodes the next
        creates take, in ring order): each workgroup's creates then get
        nodes from one dense run again, however the blocks of earlier
        batches interleaved their frees.  One host read of the ring
        bounds; returns the entries sorted."""
        c = self.counters.cpu().tolist()
        h, pub = c[_lib.TC_FREE_HEAD], c[_lib.TC_FREE_PUB]
        if pub - h <= 1:
            return 0
        idx = torch.arange(h, pub, device=self.device) % \
            self.free_list.numel()
        self.free_list[idx] = torch.sort(self.free_list[idx]).values
        return pub - h

    def find_host(self, path):
        """Node index of ``path`` (host scan of the path table; tests)."""
        n = min(int(self.counters[_lib.TC_NODES].item()), self.cap)
        want = path.encode()
        po = self.node_path_off[:n].cpu().numpy()
        pl = self.node_path_len[:n].cpu().numpy()
        par = self.node_parent[:n].cpu().numpy()
        arena = self.path_arena.cpu().numpy().tobytes()
        for v in range(n):
            if par[v] != -2 and pl[v] == len(want) and \
                    arena[po[v]:po[v] + pl[v]] == want:
                return v
        return -1

    def node_slot_host(self, v):
        """(data bytes, Stat) of node ``v`` read back from HBM (tests)."""
        from .. import jute
        off = int(self.slot_off[v].item())
        raw = bytes(self.slab[off:off + self.slot].cpu().numpy().tobytes())
        r = jute.JuteReader(raw, 0)
        st = r.read_stat()
        r.off = _lib.SLOT_LEN
        return r.read_buffer(), st


class GpuServer(object):
    """Server half of the pipeline: frame-scan + decode requests, apply them
    to a :class:`GpuTree`, encode replies."""

    def __init__(self, tree, cap_frames, out_cap, window=2048,
                 seq_order=True, group=_SRV_GROUP):
        self.tree = tree
        self.window = window              # K1 entry window of the requests
        # SEQUENTIAL creates numbered in stream order before each serve
        # (csrc/kernels/tree.hip seq_*: five launches); a server whose
        # batches never carry one (the GET pipeline, the write mixes
        # without SEQUENTIAL) skips them.  Off, a SEQUENTIAL create still
        # gets a unique number, in arrival order.
        self.seq_order = seq_order and cap_frames <= _SEQ_MAX
        self.seq_ws = None
        self.seqno = None
        # batches of GET_DATA / EXISTS only (the GET pipeline): the serve's
        # read-only instance (no claim / free / dirty-parent barriers; any
        # other op is refused UNIMPLEMENTED)
        self.read_only = False
        dev = tree.device
        self.rt = B.alloc_request_table(cap_frames, dev)
        # CREATE replies carry the created path from the tree's arena
        # (a SEQUENTIAL name differs from the requested one)
        self.resp = B.ResponseBatch(
            torch.empty(cap_frames, dtype=I32, device=dev),
            torch.empty(cap_frames, dtype=I32, device=dev),
            torch.empty(cap_frames, dtype=I32, device=dev),
            torch.empty(cap_frames, dtype=I64, device=dev),
            torch.empty(cap_frames, dtype=I64, device=dev),
            torch.zeros(cap_frames, dtype=I64, device=dev),
            torch.zeros(cap_frames, dtype=I32, device=dev),
            tree.path_arena,
            torch.zeros(cap_frames, dtype=I32, device=dev), None,
            torch.empty(cap_frames, dtype=I64, device=dev))
        # the serve kernel sizes the replies itself (presized K13 encode)
        self.presized = B.response_workspace(cap_frames, dev)
        self.out = torch.empty(out_cap, dtype=U8, device=dev)
        self.cap_frames = cap_frames
        self.scanner = B.FrameScanner(cap_frames, dev, window=window,
                                      group=group)
        self.ows = None                   # ordered-serve workspace (lazy)
        self.enc_stage = 0                # K13 LDS per workgroup (0: default)
        self.total_err = B._total_err(dev)  # the reply encode's scalars
        # the serve launch's sign-off counters (its last workgroup does the
        # tree's finish: no separate launch); this server's own, zero
        self.tickets = torch.zeros(_lib.lib().serve_tickets(cap_frames),
                                   dtype=I32, device=dev)
        self.notif = None
        if tree.watch is not None:
            self._init_watch(cap_frames, dev)

    # -- watches --------------------------------------------------------------

    def _init_watch(self, cap, dev):
        """Buffers of the watch events of one batch: the masks each write
        fired (5 words per request), then per event the watcher slot,
        notification type and path, and their K13 encode as xid -1
        notification frames (``NOTIFICATION``, state SyncConnected)."""
        ecap = 3 * cap + 64
        self.ecap = ecap
        self.fired = torch.zeros(5 * cap, dtype=I64, device=dev)
        self.wbsum = torch.empty((cap + 255) // 256, dtype=I64, device=dev)
        self.ev_slot = torch.empty(ecap, dtype=I32, device=dev)
        self.ev_type = torch.empty(ecap, dtype=I32, device=dev)
        self.ev_poff = torch.empty(ecap, dtype=I64, device=dev)
        self.ev_plen = torch.empty(ecap, dtype=I32, device=dev)
        # [events written (<= ecap), events fired]
        self.ev_total = torch.zeros(2, dtype=I64, device=dev)
        self.rs_out = torch.zeros(3, dtype=I64, device=dev)
        # notification frame: 4 + 16 header + type + state + path
        self.maxpath = int(self.tree.node_path_len.max().item()) + 16
        self.notif_buf = torch.empty(ecap * (28 + 4 + self.maxpath) + 64,
                                     dtype=U8, device=dev)
        self._nresp = self._notif_batch(self.ev_poff, self.ev_plen,
                                        self.tree.path_arena, self.ev_type,
                                        self.ev_total[0:1], ecap, dev)

    @staticmethod
    def _notif_batch(poff, plen, arena, ntype, count, cap, dev):
        """ResponseBatch of `cap` notification records (xid -1, zxid -1)."""
        return B.ResponseBatch(
            torch.full((cap,), consts.OP_CODES['NOTIFICATION'], dtype=I32,
                       device=dev),
            torch.full((cap,), consts.XID_NOTIFICATION, dtype=I32,
                       device=dev),
            torch.zeros(cap, dtype=I32, device=dev),
            torch.full((cap,), -1, dtype=I64, device=dev),
            torch.full((cap,), -1, dtype=I64, device=dev),
            poff, plen, arena, ntype, count)

    def _notify(self):
        """Expand the fired masks of the last serve into events (request
        order) and encode them: ``self.notif = (stream, bytes, slot per
        frame, events)`` — the watchers' notification frames, all on the
        device."""
        L = _lib.lib()
        r = self.resp
        L.watch_events(r.opcode, r.err, r.count, self.cap_frames, self.fired,
                       self.wbsum, self.ev_slot, self.ev_type, self.ev_poff,
                       self.ev_plen, self.ev_total)
        out, rec_off, total, _ = B.encode_responses(
            self._nresp, self.tree.store, self.notif_buf.numel(),
            out=self.notif_buf)
        self.notif_rec_off = rec_off
        self.notif = (out, total, self.ev_slot, self.ev_total[0:1])

    def _resume(self, rx, ft, wslot):
        """SET_WATCHES catch-up of the batch's SET_WATCHES frames for
        watcher ``wslot`` (csrc/kernels/tree.hip wt_resume_k): events for
        what changed after relZxid, encoded with the request bytes as path
        arena; the other watches are re-armed."""
        L = _lib.lib()
        dev = self.tree.device
        cap = self.ecap
        ev_type = torch.empty(cap, dtype=I32, device=dev)
        ev_poff = torch.empty(cap, dtype=I64, device=dev)
        ev_plen = torch.empty(cap, dtype=I32, device=dev)
        ent = torch.empty(cap, dtype=I64, device=dev)
        L.watch_resume(self.tree.tensors, rx, ft.off, ft.length, ft.count,
                       self.cap_frames, wslot, ent, ev_type, ev_poff, ev_plen,
                       self.rs_out)
        nb = self._notif_batch(ev_poff, ev_plen, rx, ev_type,
                               self.rs_out[0:1], cap, dev)
        # paths of a SET_WATCHES are bounded by its frame: ZooKeeper paths
        buf = torch.empty(cap * 32 + int(rx.numel()) + 64, dtype=U8,
                          device=dev)
        out, _, total, _ = B.encode_responses(nb, self.tree.store,
                                              buf.numel(), out=buf)
        self.resume_notif = (out, total, self.rs_out)

    def serve(self, rx, n, session=0, terminate=False, ordered=False,
              passes=4, wslot=-1, resume=False):
        """Serve the request stream ``rx[:n]`` for ``session`` (the owner of
        any EPHEMERAL node it creates).  ``n`` is a host length or the
        request encoder's device total (no host read).  Returns the reply
        stream buffer, its device total, the encoder error flag and the
        request frame table.

        ``ordered``: requests on one path are applied in stream order when
        one of them writes it (``passes`` launches; a path with more than
        ``passes`` requests in the batch has the excess answered
        SYSTEMERROR, see :meth:`order_stats`).  Reads and sets followed by
        a write to their path snapshot their reply into the tree's
        ``scratch``.  Without it requests of a batch are concurrent."""
        for _ in self.serve_steps(rx, n, session, terminate, ordered, passes,
                                  wslot, resume):
            pass
        return self.result

    def serve_steps(self, rx, n, session=0, terminate=False, ordered=False,
                    passes=4, wslot=-1, resume=False):
        """:meth:`serve` as a generator yielding once, between the request
        decode and the tree; the return tuple lands in ``self.result`` (a
        pipelined caller interleaves another connection's work there).

"""
        L = _lib.lib()
        ft = self.scanner.scan(rx, n)
        # ordered serving ranks the batch from K12's request table; the
        # plain serve parses each frame in registers instead
        rt = B.decode_requests(rx, ft, out=self.rt) if ordered else None
        yield
        r = self.resp
        r.count = ft.count
        out = [r.opcode, r.xid, r.err, r.node, r.zxid, r.path_off,
               r.path_len, r.slot, self.presized[0], self.presized[1]]
        now = int(time.time() * 1000)
        fuse = False
        seqno = self._seq_order(rx, ft) if self.seq_order else None
        if ordered:
            if self.ows is None:
                self.ows = torch.empty(
                    L.tree_order_workspace(self.cap_frames), dtype=U8,
                    device=self.tree.device)
            L.tree_serve_ordered(self.tree.tensors, rx, rt.tensors(),
                                 ft.count, self.cap_frames, out, session,
                                 now, self.ows, passes, self.tree.scratch,
                                 wslot, self.fired if self.tree.watch
                                 is not None else None, seqno)
        else:
            fuse = _FINISH_SCAN and not _SERVE_TICKETS
            L.tree_serve_frames(self.tree.tensors, rx, ft.off, ft.length,
                                ft.count, self.cap_frames, out, session, now,
                                wslot, self.fired if self.tree.watch
                                is not None else None,
                                self.tickets if _SERVE_TICKETS else None,
                                not fuse, seqno, self.read_only)
            if fuse:
                # the finish and K13's block-sum scan: one launch
                L.tree_finish_scan(self.tree.tensors, ft.count, 0, True,
                                   self.cap_frames, self.presized[1],
                                   self.total_err[0])
        out, rec_off, total, err = B.encode_responses(
            r, self.tree.store, self.out.numel(), out=self.out,
            presized=self.presized, terminate=terminate,
            stage=self.enc_stage, total_err=self.total_err,
            prescanned=fuse)
        if self.tree.compact_free:
            self.tree.free_compact()
        self.last_rec_off = rec_off         # reply frame starts (R2 splits)
        self.result = (out, total, err, ft)
        if self.tree.watch is not None:
            self._notify()
            if resume:
                if wslot < 0:
                    raise ValueError('resume needs the watcher slot')
                self._resume(rx, ft, wslot)

    def _seq_order(self, rx, ft):
        """Number the batch's SEQUENTIAL creates in stream order (parent's
        cversion before the batch + rank among its sequential creates
        here): returns the int64 [cap_frames] words for the serve (parent
        node << 32 | number; -1 none)."""
        L = _lib.lib()
        dev = self.tree.device
        if self.seq_ws is None:
            n = self.cap_frames
            self.seq_ws = torch.empty(L.tree_seq_workspace(n), dtype=U8,
                                      device=dev)
            self.seq_ws[:L.tree_seq_zeroed(n)].zero_()
            self.seqno = torch.empty(n, dtype=I64, device=dev)
        L.tree_seq_order(self.tree.tensors, rx, ft.off, ft.length, ft.count,
                         self.cap_frames, self.seq_ws, self.seqno)
        return self.seqno

    def order_stats(self):
        """(largest same-path rank, scratch bytes used) of the last ordered
        serve (host read).  A rank >= the passes used means refusals."""
        o = _lib.lib().tree_order_stats_offset(self.cap_frames)
        v = self.ows[o:o + 16].cpu().view(torch.int64).tolist()
        return v[0], v[1]


class GetPipeline(object):
    """Batched get() over the synthetic tree (BASELINE config 2)."""

    # client encode | server decode | tree + encode | client decode
    PHASES = 4

    def __init__(self, tree, batch, seed=0, streams=1, stagger=False,
                 priority=False):
        self.tree = tree
        self.batch = batch
        dev = tree.device
        self.dev = dev
        self.subs = []
        if streams > 1:
            # `streams` independent pipelined connections, each with its own
            # HIP stream, buffers and xid table, sharing the (read-only)
            # tree.  Their phases are issued round-robin (see step), so one
            # connection's latency-bound kernels (frame-scan walks, scans)
            # overlap another's bandwidth-bound ones.  `stagger`: connection
            # k runs k * PHASES / streams phases behind connection 0 (the
            # steady state of pipelined connections), so the frame scans of
            # one meet the encoders and tree of another instead of their own
            # copies; a step still issues PHASES phases of every connection,
            # and a connection's reply check lands in the step() call that
            # runs its last phase.
            per = [batch // streams + (1 if k < batch % streams else 0)
                   for k in range(streams)]
            self.subs = [GetPipeline(tree, m, seed=seed * streams + k)
                         for k, m in enumerate(per)]
            # priority: connection 0's stream is a high-priority one (its
            # small kernels take the next free slots, the others fill in)
            self.streams = [torch.cuda.Stream(
                dev, priority=-1 if priority and k == 0 else 0)
                for k in range(len(per))]
            self.stagger = stagger
            self._gens = None
            self.last = None
            return
        self.xt = B.XidTable(bits=max(20, (batch - 1).bit_length() + 1),
                             device=dev)
        n = batch
        # request descriptors (reused every step)
        self.opcode = torch.full((n,), consts.OP_CODES['GET_DATA'],
                                 dtype=I32, device=dev)
        self.arg = torch.zeros(n, dtype=I32, device=dev)
        self.zero64 = torch.zeros(n, dtype=I64, device=dev)
        self.zero32 = torch.zeros(n, dtype=I32, device=dev)
        self.acl_off = torch.zeros(1, dtype=I64, device=dev)
        self.acl_len = torch.zeros(1, dtype=I32, device=dev)
        self.acl_arena = torch.zeros(16, dtype=U8, device=dev)
        maxpath = int(tree.node_path_len.max().item())
        self.tx = torch.empty(n * (17 + maxpath) + 64, dtype=U8, device=dev)
        dmax = max(tree.data_bytes, 128)
        # K1 windows: the largest request / reply frame of this workload
        self.server = GpuServer(tree, n, n * (4 + 16 + 4 + dmax + 68) + 64,
                                window=B.frame_window(17 + maxpath),
                                seq_order=False, group=_GET_SRV_GROUP)
        self.server.read_only = _SERVE_RO
        self.server.enc_stage = _GET_STAGE
        self.rwindow = B.frame_window(4 + 16 + 4 + dmax + 68)
        lo, hi = tree.data_dist or (tree.data_bytes, tree.data_bytes)
        self.rscanner = B.FrameScanner(n, dev, window=self.rwindow,
                                       frame_hint=4 + 16 + 4 + 68 +
                                       (lo + hi) // 2)
        self.reply = B.alloc_replies(n, dev)
        self.xid_base = 0
        self.last = None
        self.seed = seed
        self.step_no = 0
        self.idx = torch.empty(n, dtype=I64, device=dev)
        self.xid = torch.empty(n, dtype=I32, device=dev)
        self.poff = torch.empty(n, dtype=I64, device=dev)
        self.plen = torch.empty(n, dtype=I32, device=dev)
        # the encode's sizes pass, written by the generator
        self.sizes = torch.empty(n, dtype=I64, device=dev) \
            if _GET_PRESIZED else None
        self.bsum = torch.empty((n + 255) // 256, dtype=I64, device=dev) \
            if _GET_PRESIZED else None
        self.gstate = None      # device {seed, step} (see capture)

    def _device_seed(self):
        """Draw each step's requests from a device-resident {seed, step}
        pair advanced on the device, so a captured graph replays NEW
        batches (a host seed would be frozen into the graph)."""
        for p in self.subs or [self]:
            if p.gstate is None:
                p.gstate = torch.tensor([p.seed, p.step_no], dtype=I64,
                                        device=self.dev)

    def capture(self, acc):
        """Capture one step (validated into ``acc``, which every replay adds
        to) as a HIP graph: a step's ~50 launches over two streams replay
        with one host call.  Run at least one eager step first (buffers
        are sized then).  Returns the graph; ``graph.replay()`` is a step.
        """
        self._device_seed()
        torch.cuda.synchronize(self.dev)
        g = torch.cuda.CUDAGraph()
        # thread-local: another thread's HIP calls (a process group's
        # watchdog) do not invalidate this capture
        with torch.cuda.graph(g, capture_error_mode='thread_local'):
            self.step(acc=acc)
        self.graph = g
        return g

    def step(self, validate=True, acc=None):
        """One batch.  With ``validate`` the number of correct replies is
        added to ``acc`` (device int64 [1]; a fresh one when None), which is
        returned.  Request generation and the reply check are one fused
        kernel each (csrc/kernels/bench.hip)."""
        if validate and acc is None:
            acc = torch.zeros(1, dtype=I64, device=self.dev)
        if not self.subs:
            for _ in self._phases(validate, acc):
                pass
            return acc if validate else None
        cur = torch.cuda.current_stream(self.dev)
        if self.stagger:
            for s in self.streams:
                s.wait_stream(cur)
            self._validate, self._acc = validate, acc
            if self._gens is None:
                ns = len(self.subs)
                self._gens = [p._forever(self, k * self.PHASES // ns)
                              for k, p in enumerate(self.subs)]
            for _ in range(self.PHASES):
                for s, g in zip(self.streams, self._gens):
                    with torch.cuda.stream(s):
                        next(g)
            for s in self.streams:
                cur.wait_stream(s)
            return acc if validate else None
        live = []
        for p, s in zip(self.subs, self.streams):
            s.wait_stream(cur)
            live.append((s, p._phases(validate, acc)))
        while live:
            nxt = []
            for s, g in live:
                with torch.cuda.stream(s):
                    if next(g, StopIteration) is not StopIteration:
                        nxt.append((s, g))
            live = nxt
        for s in self.streams:
            cur.wait_stream(s)
        return acc if validate else None

    def _forever(self, parent, lag):
        """Phases of step after step, one per next(), starting ``lag`` idle
        phases late; the validation flag and counter are the parent's at
        the time of the check."""
        for _ in range(lag):
            yield
        while True:
            for _ in self._phases(None, None, parent):
                yield           # after each of the first PHASES - 1 phases
            yield               # after the last

    def _phases(self, validate, acc, parent=None):
        """The step as a generator on the caller's current stream, yielding
        between its PHASES phases (client encode, server frame scan and
        decode, tree and reply encode, client decode and check); a
        multi-stream step interleaves the connections' phases."""
        t = self.tree
        n = self.batch
        L = _lib.lib()
        seed = (self.seed * 0x9E3779B97F4A7C15 + self.step_no) & (2**64 - 1)
        self.step_no += 1
        L.bench_gen_get(n, _i64(seed), t.leaf0, t.n_leaves, self.xid_base,
                        t.node_pw, self.idx, self.xid, self.poff, self.plen,
                        self.gstate, self.sizes, self.bsum)
        xid = self.xid
        self.xid_base = (self.xid_base + n) & 0x7fffffff
        rb = B.RequestBatch(n, self.opcode, xid, self.arg, self.poff,
                            self.plen, self.zero64, self.zero32, self.zero32,
                            t.path_arena, t.slab, self.acl_off,
                            self.acl_len, self.acl_arena)
        tx, rec_off, total, err = B.encode_requests(
            rb, self.xt, out=self.tx,
            presized=(self.sizes, self.bsum) if self.sizes is not None
            else None)
        yield
        srv = self.server.serve_steps(tx, _len(total))
        next(srv)
        yield
        for _ in srv:
            pass
        rx, rtotal, rerr, _ = self.server.result
        yield
        ft = self.rscanner.scan(rx, _len(rtotal))
        if parent is not None:
            validate, acc = parent._validate, parent._acc
        # the reply check rides in the decode kernel (acc: 1..64 slots)
        chk = (self.idx, xid, t.data_len, acc, t.slab_all,
               t.slot_off) if validate else None
        # the device step counter advances in the checking decode (one
        # launch less per step), else on its own
        rep = B.decode_replies(rx, ft, self.xt, out=self.reply, check=chk,
                               tick=self.gstate if validate else None)
        if self.gstate is not None and not validate:
            self.gstate[1:].add_(1)
        self.last = (self.idx, rep, rx, ft)


def _arena(strings, dev):
    """Pack host strings into (arena u8, off i64, len i32) device tensors."""
    enc = [x.encode() for x in strings]
    ln = np.fromiter((len(e) for e in enc), np.int32, len(enc))
    off = np.zeros(len(enc), np.int64)
    if len(enc) > 1:
        np.cumsum(ln[:-1], out=off[1:])
    blob = b''.join(enc) or b'\0'
    arena = torch.frombuffer(bytearray(blob), dtype=U8).to(dev)
    return arena, torch.from_numpy(off).to(dev), torch.from_numpy(ln).to(dev)


def _acl_table(acls, dev):
    blobs = [B._acl_bytes(a) for a in acls]
    raw = b''.join(blobs)
    lens = np.array([len(b) for b in blobs], np.int32)
    offs = np.zeros(len(blobs), np.int64)
    np.cumsum(lens[:-1], out=offs[1:])
    arena = torch.frombuffer(bytearray(raw), dtype=U8).to(dev)
    return (arena, torch.from_numpy(offs).to(dev),
            torch.from_numpy(lens).to(dev))


# ACLs the mix alternates between (K10 encodes them from the pre-encoded
# vectors; the server rejects an empty one with INVALID_ACL)
MIX_ACLS = (
    [{'perms': consts.PERM_ALL, 'id': {'scheme': 'world', 'id': 'anyone'}}],
    [{'perms': ['READ'], 'id': {'scheme': 'world', 'id': 'anyone'}},
     {'perms': consts.PERM_ALL, 'id': {'scheme': 'digest',
                               'id': 'bench:kQq8nOxk1NC8y2GdzFjp0v4ZbVY='}}],
)


class _GraphCycle(object):
    """HIP graphs replayed in turn (a workload whose steps rotate through a
    few shapes: one captured graph per shape).  ``counter``: the name of the
    pipeline's host step counter; capturing advanced it without running a
    step, so it is put back and then advanced by each replay — an eager step
    after replays continues where they left the device state."""

    def __init__(self, graphs, pipe=None, counter=None):
        self.graphs = graphs
        self.i = 0
        self.pipe = pipe
        self.counter = counter

    def replay(self):
        self.graphs[self.i].replay()
        self.i = (self.i + 1) % len(self.graphs)
        if self.counter:
            setattr(self.pipe, self.counter,
                    getattr(self.pipe, self.counter) + 1)


def _capture_steps(pipe, acc, k=1, counter=None):
    """Capture ``k`` consecutive steps of ``pipe`` as HIP graphs (run one
    eager step first: buffers are sized then).  A replay is a step."""
    dev = pipe.tree.device
    torch.cuda.synchronize(dev)
    s0 = getattr(pipe, counter) if counter else None
    graphs = []
    for _ in range(k):
        g = torch.cuda.CUDAGraph()
        # thread-local: another thread's HIP calls do not invalidate it
        with torch.cuda.graph(g, capture_error_mode='thread_local'):
            pipe.step(acc=acc)
        graphs.append(g)
    if counter:
        setattr(pipe, counter, s0)
    if k == 1 and not counter:
        return graphs[0]
    return _GraphCycle(graphs, pipe, counter)


class _Driver(object):
    """Client half shared by the write pipelines: K10 encode of a request
    batch (xids recorded in the HBM xid table), the GPU server, then K1 +
    K2-K8 decode of the reply stream."""

    def __init__(self, tree, batch, max_path, data_bytes, seed,
                 seq_order=False, group=_SRV_GROUP):
        self.tree = tree
        self.batch = batch
        self.dev = dev = tree.device
        self.xt = B.XidTable(bits=max(20, (batch - 1).bit_length() + 1),
                             device=dev)
        self.tx = torch.empty(batch * (33 + max_path + data_bytes + 128) + 64,
                              dtype=U8, device=dev)
        dmax = max(tree.data_bytes, 128, data_bytes)
        # K1 windows from the largest frames (CREATE with data and a
        # two-entry ACL; a GET_DATA-sized reply)
        self.server = GpuServer(
            tree, batch, batch * (4 + 16 + 4 + max(dmax, max_path + 16) + 68)
            + 64, window=B.frame_window(33 + max_path + data_bytes + 128),
            seq_order=seq_order, group=group)
        self.rwindow = B.frame_window(4 + 16 + 4 + max(dmax, max_path + 16)
                                      + 68)
        self.reply = B.alloc_replies(batch, dev)
        self.rscanner = None
        # the session's next xid, on the device: a captured step replays
        # with new xids
        self.xid_dev = torch.zeros(1, dtype=I64, device=dev)
        self.iota = torch.arange(batch, dtype=I64, device=dev)
        self.passes = 0          # > 0: ordered serving in that many passes

    def xids(self, n):
        x = torch.empty(n, dtype=I32, device=self.dev)
        _lib.lib().bench_xids(n, self.xid_dev, x)     # (one fused launch)
        self.xid_dev.add_(n)
        return x

    def create_dirs(self, levels, acl):
        """CREATE persistent directories, one batch per level (a parent must
        exist before its children's batch runs).  ``acl`` = (arena, off,
        len) pre-encoded ACL table."""
        dev = self.dev
        aarena, aoff, alen = acl
        for level in levels:
            n = len(level)
            arena, off, ln = _arena(level, dev)
            z32 = torch.zeros(n, dtype=I32, device=dev)
            rb = B.RequestBatch(
                n, torch.full((n,), consts.OP_CODES['CREATE'], dtype=I32,
                              device=dev),
                self.xids(n), z32, off, ln,
                torch.zeros(n, dtype=I64, device=dev), z32, z32, arena,
                arena, aoff, alen, aarena)
            rep, _ = self.run(rb)
            errs = rep.err[:n]
            if not bool(((errs == 0) |
                         (errs == consts.ERR_CODES['NODE_EXISTS'])).all()):
                raise RuntimeError('directory create failed: %r' % (
                    errs.unique().cpu().tolist(),))

    def run(self, rb, session=0):
        """One batch through encode -> server -> decode.  Both streams are
        scanned over their encoders' device totals: no device-to-host read."""
        tx, _, total, _ = B.encode_requests(rb, self.xt, out=self.tx)
        rx, rtotal, _, _ = self.server.serve(tx, _len(total),
                                             session=session,
                                             ordered=self.passes > 0,
                                             passes=max(self.passes, 1))
        if self.rscanner is None:
            self.rscanner = B.FrameScanner(self.batch, self.dev,
                                           window=self.rwindow)
        ft = self.rscanner.scan(rx, _len(rtotal))
        rep = B.decode_replies(rx, ft, self.xt, out=self.reply)
        return rep, rx


class MixPipeline(object):
    """create / set(version CAS) / delete mix with ACL encode (BASELINE
    config 3) over the synthetic tree.

    Every step issues ``m = batch // 3`` of each op on three rotating
    generations of ``m`` nodes ``/mix/dDDDD/gG_KKKKKKKKK``: step ``s``
    CREATEs generation ``s % 3`` (alternating two ACL vectors), SET_DATAs
    generation ``s-1`` with expected version 0 (every 16th with a stale
    version, which must fail with BAD_VERSION) and DELETEs generation ``s-2``
    with its exact current version.  Node slots, paths and hash entries are
    recycled through the tree's free ring, so the tree size is steady.
    Every reply is checked on the device against its expected error code,
    xid and opcode (and version 1 for successful sets)."""

    def __init__(self, tree, batch, data_bytes=100, ndirs=1024, seed=0):
        m = max(batch // 3, 1)
        self.m = m
        self.n = 3 * m
        dev = tree.device
        self.tree = tree
        self.ndirs = ndirs
        paths = ['/mix/d%05d/g%d_%09d' % (k % ndirs, g, k)
                 for g in range(3) for k in range(m)]
        maxp = max(len(p) for p in paths)
        self.drv = _Driver(tree, self.n, maxp, data_bytes, seed)
        self.path_arena, poff, plen = _arena(paths, dev)
        g = torch.Generator(device=dev)
        g.manual_seed(seed + 7)
        nblk = 1024
        self.data_arena = torch.randint(0, 256, (nblk * data_bytes + 16,),
                                        dtype=U8, device=dev, generator=g)
        self.acl_arena, self.acl_off, self.acl_len = _acl_table(MIX_ACLS, dev)
        k = torch.arange(m, dtype=I64, device=dev)
        stale = (k % 16) == 15
        ops = consts.OP_CODES
        self.opcode = torch.cat([
            torch.full((m,), ops['CREATE'], dtype=I32, device=dev),
            torch.full((m,), ops['SET_DATA'], dtype=I32, device=dev),
            torch.full((m,), ops['DELETE'], dtype=I32, device=dev)])
        self.arg = torch.cat([torch.zeros(m, dtype=I64, device=dev),
                              torch.where(stale, 7, 0),
                              torch.where(stale, 0, 1)]).to(I32)
        self.data_off = torch.cat([(k % nblk) * data_bytes,
                                   ((k + 7) % nblk) * data_bytes,
                                   torch.zeros(m, dtype=I64, device=dev)])
        self.data_len = torch.cat([
            torch.full((2 * m,), data_bytes, dtype=I32, device=dev),
            torch.zeros(m, dtype=I32, device=dev)])
        self.acl_id = torch.cat([(k % 2).to(I32),
                                 torch.zeros(2 * m, dtype=I32, device=dev)])
        bad = consts.ERR_CODES['BAD_VERSION']
        self.want_err = torch.cat([
            torch.zeros(m, dtype=I32, device=dev),
            torch.where(stale, bad, 0).to(I32),
            torch.zeros(m, dtype=I32, device=dev)])
        self.is_set_ok = torch.cat([
            torch.zeros(m, dtype=torch.bool, device=dev), ~stale,
            torch.zeros(m, dtype=torch.bool, device=dev)])
        # path offsets per rotation r = s % 3: (create, set, delete) gens
        po = poff.view(3, m)
        self.path_off = [torch.cat([po[r], po[(r - 1) % 3], po[(r - 2) % 3]])
                         for r in range(3)]
        self.path_len = plen[:m].repeat(3)
        self.s = -2
        self.drv.create_dirs(
            [['/mix'], ['/mix/d%05d' % d for d in range(ndirs)]],
            (self.acl_arena, self.acl_off, self.acl_len))
        # prime: s = -2 creates generation 1, s = -1 creates 2 and sets 1
        self.step(validate=False, n=m)
        self.step(validate=False, n=2 * m)

    def capture(self, acc):
        """Three HIP graphs, one per rotation of the generations (step s
        creates s % 3, sets s - 1, deletes s - 2), replayed in turn."""
        return _capture_steps(self, acc, 3, counter='s')

    def _batch(self, n, r):
        d = self.drv
        return B.RequestBatch(n, self.opcode[:n], d.xids(n), self.arg[:n],
                              self.path_off[r][:n], self.path_len[:n],
                              self.data_off[:n], self.data_len[:n],
                              self.acl_id[:n], self.path_arena,
                              self.data_arena, self.acl_off, self.acl_len,
                              self.acl_arena)

    def step(self, validate=True, n=None, acc=None):
        n = self.n if n is None else n
        rb = self._batch(n, self.s % 3)
        rep, _ = self.drv.run(rb)
        self.last = (rb, rep)
        self.s += 1
        if not validate:
            return None
        ok = ((rep.status[:n] == 0) & (rep.err[:n] == self.want_err[:n]) &
              (rep.xid[:n] == rb.xid) & (rep.opcode[:n] == rb.opcode) &
              (~self.is_set_ok[:n] | (rep.stat32[0, :n] == 1)))
        if acc is None:
            return ok.sum()
        acc[:1] += ok.sum()
        return acc

    def diagnose(self):
        rb, rep = self.last
        n = rb.n
        bad = rep.err[:n] != self.want_err[:n]
        e, c = torch.unique(rep.err[:n][bad], return_counts=True)
        return {'wrong_err': dict(zip(e.cpu().tolist(), c.cpu().tolist())),
                'status_bad': int((rep.status[:n] != 0).sum().item()),
                'counters': self.tree.counters.cpu().tolist()}


class ChainPipeline(object):
    """In-batch ordering workload: every step sends, for each of ``m`` paths
    ``/chain/dDDDD/cKKKKKKKKK``, the chain CREATE (``data_bytes // 2``
    bytes) -> SET_DATA (version 0, ``data_bytes``) -> GET_DATA -> DELETE
    (version 1) back to back in one batch, as one session pipelining them
    would.  The server must apply each chain in order (ordered serving, 4
    passes): every reply is checked on the device — all OK, the set and the
    get see version 1, and the get returns the set's data length.  Nodes
    are recycled through the free ring (each step deletes what it created).
    """

    def __init__(self, tree, batch, data_bytes=100, ndirs=1024, seed=0):
        m = max(batch // 4, 1)
        self.m = m
        self.n = n = 4 * m
        dev = tree.device
        self.tree = tree
        self.data_bytes = data_bytes
        need = 2 * m * (80 + ((data_bytes + 15) & ~15))
        if tree.scratch is None or tree.scratch.numel() < need:
            raise ValueError('ChainPipeline needs GpuTree(scratch >= %d)'
                             % need)
        paths = ['/chain/d%05d/c%09d' % (k % ndirs, k) for k in range(m)]
        maxp = max(len(p) for p in paths)
        self.drv = _Driver(tree, n, maxp, data_bytes, seed)
        self.drv.passes = 4
        self.path_arena, poff, plen = _arena(paths, dev)
        g = torch.Generator(device=dev)
        g.manual_seed(seed + 11)
        nblk = 1024
        self.data_arena = torch.randint(0, 256, (nblk * data_bytes + 16,),
                                        dtype=U8, device=dev, generator=g)
        self.acl_arena, self.acl_off, self.acl_len = _acl_table(MIX_ACLS, dev)
        ops = consts.OP_CODES

        def il(a, b, c, d):      # interleave per path: [a0 b0 c0 d0 a1 ...]
            return torch.stack([a, b, c, d], 1).reshape(-1)
        k = torch.arange(m, dtype=I64, device=dev)
        full = lambda v, dt: torch.full((m,), v, dtype=dt, device=dev)  # noqa
        self.opcode = il(full(ops['CREATE'], I32), full(ops['SET_DATA'], I32),
                         full(ops['GET_DATA'], I32), full(ops['DELETE'], I32))
        self.arg = il(full(0, I32), full(0, I32), full(0, I32), full(1, I32))
        self.path_off = il(poff, poff, poff, poff)
        self.path_len = il(plen, plen, plen, plen)
        self.data_off = il((k % nblk) * data_bytes,
                           ((k + 7) % nblk) * data_bytes, full(0, I64),
                           full(0, I64))
        self.data_len = il(full(data_bytes // 2, I32), full(data_bytes, I32),
                           full(0, I32), full(0, I32))
        self.acl_id = il((k % 2).to(I32), full(0, I32), full(0, I32),
                         full(0, I32))
        self.is_set = self.opcode == ops['SET_DATA']
        self.is_get = self.opcode == ops['GET_DATA']
        self.drv.create_dirs(
            [['/chain'], ['/chain/d%05d' % d for d in range(ndirs)]],
            (self.acl_arena, self.acl_off, self.acl_len))
        self.last = None

    def capture(self, acc):
        """One step as a HIP graph (every step has the same shape)."""
        return _capture_steps(self, acc)

    def step(self, validate=True, acc=None):
        n = self.n
        d = self.drv
        rb = B.RequestBatch(n, self.opcode, d.xids(n), self.arg,
                            self.path_off, self.path_len, self.data_off,
                            self.data_len, self.acl_id, self.path_arena,
                            self.data_arena, self.acl_off, self.acl_len,
                            self.acl_arena)
        rep, _ = d.run(rb)
        self.last = (rb, rep)
        if not validate:
            return None
        ver1 = rep.stat32[0, :n] == 1
        ok = ((rep.status[:n] == 0) & (rep.err[:n] == 0) &
              (rep.xid[:n] == rb.xid) & (rep.opcode[:n] == rb.opcode) &
              (~(self.is_set | self.is_get) | ver1) &
              (~self.is_get | ((rep.stat32[3, :n] == self.data_bytes) &
                               (rep.pay_len[:n] == self.data_bytes))))
        if acc is None:
            return ok.sum()
        acc[:1] += ok.sum()
        return acc

    def diagnose(self):
        rb, rep = self.last
        n = rb.n
        bad = rep.err[:n] != 0
        e, c = torch.unique(rep.err[:n][bad], return_counts=True)
        return {'wrong_err': dict(zip(e.cpu().tolist(), c.cpu().tolist())),
                'order_stats': self.drv.server.order_stats()}


class NestPipeline(object):
    """createWithEmptyParents in one batch (lib/client.js:412-481): every
    step sends, for each of ``m`` trees ``/nest/dDDDD/pKKKKKKKKK``, the
    depth-3 chain CREATE p -> CREATE p/c -> CREATE p/c/g -> EXISTS p ->
    DELETE p/c/g -> DELETE p/c -> DELETE p (7 requests) back to back in ONE
    batch, as one session pipelining them would.  The creates depend on
    their parents, the EXISTS on its children's writes and the deletes on
    their children being gone: the ordered GPU server must honour
    parent / child order (passes by the longest conflict chain, 6 here).
    Every reply is checked on the device: all OK, and the parent's EXISTS
    sees exactly one child (numChildren 1, cversion 1).  The tree is left
    as it was (every step deletes what it created)."""

    PER = 7

    def __init__(self, tree, batch, ndirs=1024, seed=0):
        m = max(batch // self.PER, 1)
        self.m = m
        self.n = n = self.PER * m
        dev = tree.device
        self.tree = tree
        need = 2 * m * (80 + 16)
        if tree.scratch is None or tree.scratch.numel() < need:
            raise ValueError('NestPipeline needs GpuTree(scratch >= %d)'
                             % need)
        base = ['/nest/d%05d/p%09d' % (k % ndirs, k) for k in range(m)]
        paths = [b + sfx for b in base for sfx in ('', '/c', '/c/g')]
        maxp = max(len(p) for p in paths)
        self.drv = _Driver(tree, n, maxp, 16, seed)
        self.drv.passes = 8
        self.path_arena, poff, plen = _arena(paths, dev)
        poff = poff.view(m, 3)
        plen = plen.view(m, 3)
        self.data_arena = torch.full((16,), 0x6e, dtype=U8, device=dev)
        self.acl_arena, self.acl_off, self.acl_len = _acl_table(MIX_ACLS[:1],
                                                                dev)
        ops = consts.OP_CODES
        col = lambda *c: torch.stack(c, 1).reshape(-1)     # noqa: E731
        full = lambda v, dt: torch.full((m,), v, dtype=dt, device=dev)  # noqa
        self.opcode = col(*(full(ops[o], I32) for o in (
            'CREATE', 'CREATE', 'CREATE', 'EXISTS', 'DELETE', 'DELETE',
            'DELETE')))
        # path per request: p, c, g, p, g, c, p
        self.path_off = col(poff[:, 0], poff[:, 1], poff[:, 2], poff[:, 0],
                            poff[:, 2], poff[:, 1], poff[:, 0])
        self.path_len = col(plen[:, 0], plen[:, 1], plen[:, 2], plen[:, 0],
                            plen[:, 2], plen[:, 1], plen[:, 0])
        self.arg = col(full(0, I32), full(0, I32), full(0, I32),
                       full(0, I32), full(-1, I32), full(-1, I32),
                       full(-1, I32))
        self.data_off = torch.zeros(n, dtype=I64, device=dev)
        self.data_len = col(full(4, I32), full(4, I32), full(4, I32),
                            *(full(0, I32) for _ in range(4)))
        self.acl_id = torch.zeros(n, dtype=I32, device=dev)
        self.is_exists = self.opcode == ops['EXISTS']
        self.drv.create_dirs(
            [['/nest'], ['/nest/d%05d' % d for d in range(ndirs)]],
            (self.acl_arena, self.acl_off, self.acl_len))
        self.last = None

    def capture(self, acc):
        """One step as a HIP graph (every step has the same shape)."""
        return _capture_steps(self, acc)

    def step(self, validate=True, acc=None):
        n = self.n
        d = self.drv
        rb = B.RequestBatch(n, self.opcode, d.xids(n), self.arg,
                            self.path_off, self.path_len, self.data_off,
                            self.data_len, self.acl_id, self.path_arena,
                            self.data_arena, self.acl_off, self.acl_len,
                            self.acl_arena)
        rep, _ = d.run(rb)
        self.last = (rb, rep)
        if not validate:
            return None
        one_child = (rep.stat32[4, :n] == 1) & (rep.stat32[1, :n] == 1)
        ok = ((rep.status[:n] == 0) & (rep.err[:n] == 0) &
              (rep.xid[:n] == rb.xid) & (rep.opcode[:n] == rb.opcode) &
              (~self.is_exists | one_child))
        if acc is None:
            return ok.sum()
        acc[:1] += ok.sum()
        return acc

    def diagnose(self):
        rb, rep = self.last
        n = rb.n
        bad = rep.err[:n] != 0
        e, c = torch.unique(rep.err[:n][bad], return_counts=True)
        return {'wrong_err': dict(zip(e.cpu().tolist(), c.cpu().tolist())),
                'order_stats': self.drv.server.order_stats()}


class GpuSessionTable(object):
    """The GPU server's session table in HBM and its handshake (K9 server
    side, csrc/kernels/session.hip): ConnectRequest frames in,
    ConnectResponse frames out, new / resumed / expired decided on the
    device.  Session ids are ``server_id << 56 | (index + 1)`` in allocation
    order, so the server's host side knows the id it handed out without a
    read-back."""

    MIN_TO, MAX_TO = 4000, 40000        # 2 and 20 ticks of 2 s

    def __init__(self, tree, cap=1 << 16, server_id=1, secret=0x5A4B1D,
                 members=1):
        dev = tree.device
        self.tree = tree
        self.dev = dev
        self.cap = cap
        self.server_id = server_id
        self.secret = secret
        # an ensemble of `members` servers replicates its session table:
        # member m's sessions live in slots (m - 1) * span ... (see
        # session.hip); one server's table has no partition
        self.span = cap // members if members > 1 else 0
        self.sid = torch.zeros(cap, dtype=I64, device=dev)
        self.passwd = torch.zeros(cap * 16, dtype=U8, device=dev)
        self.timeout = torch.zeros(cap, dtype=I32, device=dev)
        self.state = torch.zeros(cap, dtype=I32, device=dev)
        self.next = torch.zeros(1, dtype=I64, device=dev)
        self.allocated = 0              # host mirror of `next`
        self._tensors = [self.sid, self.passwd, self.timeout, self.state,
                         self.next]
        self.scanner = B.FrameScanner(64, dev, window=256)
        self.resp = torch.empty(64 * _lib.CR_RESP_BYTES, dtype=U8, device=dev)
        self.resp_sid = torch.empty(64, dtype=I64, device=dev)
        self.outcome = torch.empty(64, dtype=I32, device=dev)

    def sid_of(self, index):
        return (self.server_id << 56) | (index + 1)

    def connect(self, rx, nbytes, n_new):
        """Serve the ConnectRequest stream ``rx[:nbytes]`` (at most 64
        frames); ``n_new`` = how many of them ask for a new session (host
        bookkeeping of the allocation counter).  Returns (response stream
        [41 * frames], bound session ids, outcome codes)."""
        ft = self.scanner.scan(rx, nbytes)
        _lib.lib().session_connect(
            rx, ft.off, ft.length, ft.count, 64, self._tensors,
            self.server_id, _i64(self.secret), self.MIN_TO, self.MAX_TO,
            self.tree.counters[_lib.TC_ZXID:], self.resp, self.resp_sid,
            self.outcome, self.span)
        self.allocated += n_new
        return self.resp, self.resp_sid, self.outcome

    def close(self, sids):
        """Expire / close sessions (device int64 tensor of ids)."""
        _lib.lib().session_close(self._tensors, sids, self.server_id,
                                 self.span)

    def install(self, records):
        """Replicate other members' sessions into this table (device int64
        [k, 4]: sid, timeout, password bytes 0-7 and 8-15; this member's own
        records are skipped) — the receiving end of R3."""
        _lib.lib().session_install(self._tensors, records, self.server_id,
                                   self.span)


class StormPipeline(object):
    """EPHEMERAL|SEQUENTIAL create storm with session expire AND resume
    (BASELINE config 5; lib/zk-session.js:147-205, :265-339,
    test/nasty.test.js:40-103).

    Session ``k`` lives three steps:

      step 2k    born: the client K9-encodes a ConnectRequest with
                 sessionId 0, the GPU server's handshake kernel allocates
                 the session (K9 server side), the client K9-decodes the
                 ConnectResponse; the session creates ``batch`` ephemeral
                 sequential nodes ``/storm/dDDDDD/e-<seq>``; session ``k-1``
                 expires and the server removes its ephemerals, which must
                 be exactly its TWO batches (the one made before its resume
                 survived it)
      step 2k+1  its connection drops; a new one resumes it: ConnectRequest
                 with the id and password from the last ConnectResponse,
                 all on the device; the server answers RESUMED with the same
                 id and password.  In the same handshake batch the client
                 also tries the session that expired at step 2k, which must
                 get the expired answer (id 0).  The resumed session creates
                 its second batch.

    Every check (replies, handshake outcome, ids, password, removed count)
    runs on the device; a step makes no device-to-host read.  The hash
    index needs no rebuild: the expiry moves live entries back over the
    holes it leaves and empties the rest (csrc/kernels/tree.hip ht_shift),
    and the next batch's names take over the tombstones their probes pass,
    so never-reused SEQUENTIAL names leave a bounded number of tombstones
    (~0.6 % of the index at the bench's size,
    tools/microbench/storm_census.py).

    Across GPUs (a process group of ``world`` > 1 ranks: the members of one
    ensemble, each rank's GPU server a member) the session MOVES, as
    ``lib/zk-session.js:265-339`` reattaches it to another backend and
    ``test/multi-node.test.js:233-350`` checks that its ephemeral survives:
    session k of rank r is born on member r, and its records {id, timeout,
    password} go to every member (R3: one ``all_gather_into_tensor`` of
    the step's new sessions, installed into each member's replicated
    table).  At step 2k+1 rank r's client resumes it on member (r+1) %
    world: its ConnectRequests travel there and the ConnectResponses back
    through two small all-gathers, member r+1 answers RESUMED with the same
    id and password, and the session's second batch is created on member
    r+1.  Its first batch survives the move on member r; at its expiry
    every member drops what the session created there (so each removes two
    sessions' batches: its own session's first and its neighbour's second)
    and closes it in its table, so the expired resume tried at the next
    move is refused on any member.

    The members hold ONE replicated tree (every rank builds the same tree,
    seed 0, and applies every committed write): a step's write batches of
    all members are all-gathered as encoded CREATE frames and every member
    applies them in rank order — the step's commit order, the zxid order a
    ZooKeeper leader imposes — so sequential names, zxids and ephemeral
    owners come out the same on every member.  The member a client is
    attached to answers it (its reply stream comes back through an
    all-gather after a move).  A znode created through member r is then
    readable and deletable on member r+1 (:meth:`cross_read`; the
    reference's test/multi-node.test.js:107-165 write visibility and
    :233-350 ephemeral-survives-failover), and an expiry removes the
    session's nodes on every member.  The work of a write grows with the
    members (each applies W batches a step): ``stats['replicated_writes']``
    counts what this member applied."""

    TIMEOUT = 30000
    HS_SLOT = 128            # handshake bytes a rank sends per all-gather

    def __init__(self, tree, batch, ndirs=1024, data_bytes=16, seed=0,
                 group=None, coll_device=None):
        import torch.distributed as dist
        dev = tree.device
        self.tree = tree
        self.dev = dev
        self.n = batch
        self.ndirs = ndirs
        on = dist.is_available() and dist.is_initialized()
        self.dist = dist
        self.group = group
        self.world = W = dist.get_world_size(group) if on else 1
        self.rank = dist.get_rank(group) if on else 0
        self.coll = torch.device(coll_device) if coll_device else dev
        self.drv = _Driver(tree, batch, 32, data_bytes, seed,
                           seq_order=True, group=_STORM_SRV_GROUP)
        self.sessions = GpuSessionTable(tree, server_id=self.rank + 1,
                                        members=W)
        if W > 1:
            # the current session of every member on the device (member m's
            # k-th session is (m + 1) << 56 | k + 1, k = kdev): serve and
            # expiry take theirs through the tree's TC_SESS word, so a
            # captured step replays with the next generation's ids
            self.sid_base = torch.tensor([(m + 1) << 56 for m in range(W)],
                                         dtype=I64, device=dev)
            self.sess_tab = torch.zeros(W, dtype=I64, device=dev)
            # this step's new sessions of every member ([W, 4] records),
            # the generation before's (expired at the next birth), and the
            # handshake slots
            self.recs = torch.zeros(W, 4, dtype=I64, device=dev)
            self.prev_recs = torch.zeros(W, 4, dtype=I64, device=dev)
            self.hs_out = torch.zeros(self.HS_SLOT, dtype=U8, device=dev)
            self.hs_all = torch.zeros(W * self.HS_SLOT, dtype=U8, device=dev)
        prefixes = ['/storm/d%05d/e-' % (k % ndirs) for k in range(batch)]
        self.path_arena, self.path_off, self.path_len = _arena(prefixes, dev)
        self.data_arena = torch.full((data_bytes + 16,), 0x5a, dtype=U8,
                                     device=dev)
        self.acl_arena, self.acl_off, self.acl_len = _acl_table(MIX_ACLS[:1],
                                                                dev)
        flags = consts.CREATE_FLAGS['EPHEMERAL'] | \
            consts.CREATE_FLAGS['SEQUENTIAL']
        self.opcode = torch.full((batch,), consts.OP_CODES['CREATE'],
                                 dtype=I32, device=dev)
        self.arg = torch.full((batch,), flags, dtype=I32, device=dev)
        self.data_off = torch.zeros(batch, dtype=I64, device=dev)
        self.data_len = torch.full((batch,), data_bytes, dtype=I32,
                                   device=dev)
        self.acl_id = torch.zeros(batch, dtype=I32, device=dev)
        self.want_len = self.path_len + 10
        self.removed = torch.zeros(1, dtype=I64, device=dev)
        # client-side credentials, device only: [cur, prev] session ids and
        # passwords (what the last ConnectResponses carried)
        self.cred_sid = torch.zeros(2, dtype=I64, device=dev)
        self.cred_pw = torch.zeros(32, dtype=U8, device=dev)
        self.last_zxid = torch.zeros(1, dtype=I64, device=dev)
        self.chk = torch.zeros(1, dtype=I64, device=dev)
        self.hs_ok = torch.ones(1, dtype=torch.bool, device=dev)
        # one member: the handshake beside the request encode, the expiry
        # beside the reply decode, on this second stream (ZKMI_STORM_STREAMS=1:
        # everything on the caller's)
        self.side = torch.cuda.Stream(dev) if _STORM_STREAMS else None
        self.cr_tx = torch.empty(256, dtype=U8, device=dev)
        self.cr_ws = torch.empty(_lib.lib().scan_workspace(2),
                                 dtype=I64, device=dev)
        self.rscan = B.FrameScanner(4, dev, window=256)
        # K9 encode arguments per handshake shape (m requests, pwl bytes)
        self.zero_sid = torch.zeros(1, dtype=I64, device=dev)
        self.zero_pw = torch.zeros(8, dtype=U8, device=dev)
        self.cr_args = {}
        for m, pwl in ((1, 8), (1, 16), (2, 16)):
            self.cr_args[(m, pwl)] = (
                torch.zeros(m, dtype=I32, device=dev),
                torch.full((m,), self.TIMEOUT, dtype=I32, device=dev),
                torch.arange(m, dtype=I64, device=dev) * pwl,
                torch.full((m,), pwl, dtype=I32, device=dev),
                torch.empty(m, dtype=I64, device=dev),
                torch.empty(m, dtype=I64, device=dev),
                torch.zeros(1, dtype=I64, device=dev))
        self.k = -1                       # index of the current session
        # ... and on the device (a captured step replays with the next
        # session's ids: serve / expire take them from the tree's TC_SESS)
        self.kdev = torch.full((1,), -1, dtype=I64, device=dev)
        self.sid0 = self.sessions.sid_of(0)
        self._capturing = False
        self.step_no = 0
        self.stats = {'born': 0, 'resumed': 0, 'expired': 0,
                      'expired_resume_refused': 0, 'cross_rank_resumes': 0}
        # replicated tree (see the class docs): the step's stream slots
        self.req_bytes = None       # a batch's encoded bytes (constant)
        self.rep_bytes = None
        self.len_ok = torch.ones(1, dtype=torch.bool, device=dev)
        if W > 1:
            self.stats['replicated_writes'] = 0
        self.first = None           # the current session's first batch
        self.drv.create_dirs(
            [['/storm'], ['/storm/d%05d' % d for d in range(ndirs)]],
            (self.acl_arena, self.acl_off, self.acl_len))
        self.step(validate=False)            # session 0 born, first batch

    # -- the client / server handshake, all on the device ---------------------

    def _gather(self, out, inp):
        """``all_gather_into_tensor`` on the collective device."""
        if self.coll == self.dev:
            self.dist.all_gather_into_tensor(out, inp, group=self.group)
            return out
        o = torch.empty(out.shape, dtype=out.dtype, device=self.coll)
        self.dist.all_gather_into_tensor(o, inp.to(self.coll),
                                         group=self.group)
        out.copy_(o)
        return out

    def sid(self, member, k):
        """Session id of member ``member``'s k-th session (every member
        allocates one a birth step, so ids are known on every rank)."""
        return ((member + 1) << 56) | (k + 1)

    def _handshake(self, resume):
        """K9 client encode -> K9 server handshake -> K9 client decode.
        Birth: one request (id 0, 8 zero password bytes as zkstream sends,
        lib/zk-session.js:59).  Resume: [current session, the session that
        expired last step] with their ids and passwords — on the next
        member when the ensemble spans GPUs (the frames go there and the
        answers come back through all-gathers)."""
        L = _lib.lib()
        # the first session has no expired predecessor to try
        m = 2 if resume and self.k >= 1 else 1
        pwl = 16 if resume else 8
        if resume:
            sid = self.cred_sid[:m]
            arena = self.cred_pw[:16 * m]
        else:
            sid = self.zero_sid
            arena = self.zero_pw
        proto, tmo, pwo, pwlt, sizes, off, total = self.cr_args[(m, pwl)]
        zx = self.last_zxid.expand(m).contiguous()
        L.encode_connect_requests(proto, zx, tmo, sid, pwo, pwlt, arena, m,
                                  sizes, off, total, self.cr_ws, self.cr_tx)
        nbytes = m * (32 + pwl)
        rb = m * _lib.CR_RESP_BYTES
        W = self.world
        if resume and W > 1:
            # to member r + 1: every rank's frames gathered, each serves
            # the previous rank's, the answers gathered back
            S = self.HS_SLOT
            self.hs_out[:nbytes].copy_(self.cr_tx[:nbytes])
            self._gather(self.hs_all, self.hs_out)
            src = (self.rank - 1) % W
            rx = self.hs_all[src * S:src * S + nbytes].clone()
            resp, bound, outcome = self.sessions.connect(rx, nbytes, 0)
            self.hs_out[:rb].copy_(resp[:rb])
            self._gather(self.hs_all, self.hs_out)
            dst = (self.rank + 1) % W
            resp = self.hs_all[dst * S:dst * S + rb].clone()
            ft = self.rscan.scan(resp, rb)
            o = B.decode_connect_responses(resp, ft, m)
            # (`outcome`: how this member answered the previous rank's
            # client — every member checks the one it served, the client
            # checks the answer it got)
            return o, bound, outcome, resp
        resp, bound, outcome = self.sessions.connect(
            self.cr_tx[:nbytes], nbytes, 0)
        ft = self.rscan.scan(resp[:rb], rb)
        o = B.decode_connect_responses(resp, ft, m)
        return o, bound, outcome, resp

    @property
    def capturable(self):
        """One member, or an ensemble whose all-gathers run on RCCL on the
        pipeline's device (a host backend cannot be captured)."""
        if self.world == 1:
            return True
        return self.coll == self.dev and \
            self.dist.get_backend(self.group) == 'nccl'

    def capture(self, acc):
        """Capture the steady state's two step shapes (a birth that expires
        the session before, a resume that also tries the expired one) as
        HIP graphs; ``replay()`` runs the next step.  Session ids live on
        the device (``kdev`` -> the tree's TC_SESS word; across members the
        table of every member's current id), so a replay serves, expires
        and checks the next session; the host keeps only its bookkeeping
        (counts).  Across members the all-gathers are captured with the
        rest (RCCL; see ``capturable``)."""
        if not self.capturable:
            raise RuntimeError('storm capture: the process group cannot be '
                               'captured (host backend)')
        while self.step_no < 2 or self.step_no % 2:
            self.step(acc=acc)
        torch.cuda.synchronize(self.dev)
        keep = (self.step_no, self.k, dict(self.stats),
                self.sessions.allocated)
        graphs = []
        self._capturing = True
        try:
            for _ in range(2):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, capture_error_mode='thread_local'):
                    self.step(acc=acc)
                graphs.append(g)
        finally:
            self._capturing = False
        (self.step_no, self.k, self.stats,
         self.sessions.allocated) = keep
        return _StormCycle(self, graphs)

    def _advance(self):
        """The host side of a step (eager and replayed alike): step and
        session counters, stats.  Returns resume."""
        s = self.step_no
        self.step_no += 1
        resume = s % 2 == 1
        if self.world > 1:
            self.stats['replicated_writes'] += self.world * self.n
            self.stats['cross_rank_resumes'] += int(resume)
        if resume:
            self.stats['resumed'] += 1
            self.stats['expired_resume_refused'] += int(self.k >= 1)
        else:
            self.k += 1
            self.sessions.allocated += 1
            self.stats['born'] += 1
            if self.k >= 1:
                self.stats['expired'] += 1
        return resume

    def step(self, validate=True, acc=None):
        t = self.tree
        n = self.n
        resume = self._advance()
        if not resume:
            self.kdev.add_(1)
        # this step's session on the device (one member: its own; the
        # ensemble passes host ids, see _replicated_run)
        sess_dev = t.counters[_lib.TC_SESS:_lib.TC_SESS + 1]
        torch.add(self.kdev, self.sid0, out=sess_dev)
        if self.world > 1:
            torch.add(self.sid_base, self.kdev + 1, out=self.sess_tab)
        if self.world == 1 and self.side is not None:
            return self._step_two_streams(resume, sess_dev, validate, acc)
        o, bound, outcome, resp = self._handshake(resume)
        self._check_handshake(resume, sess_dev, o, bound, outcome, resp)
        rb = self._batch()
        if self.world > 1:
            rep = self._replicated_run(rb, resume)
        else:
            rep, _ = self.drv.run(rb, session=_lib.SESS_DEV)
        self.last = (rb, rep)
        if not resume and self.world > 1:
            # the new session's first batch: the created paths (offsets into
            # the reply stream kept with them), for cross_read
            self.first = (self.my_rx.clone(), rep.pay_off[:n].clone(),
                          rep.pay_len[:n].clone())
        self._check_replies(rb, rep)
        expire_ok = True
        if not resume and self.k >= 1 and self.world > 1:
            # the generation before expires on every member, which holds
            # all members' sessions' nodes (the replicated tree): each of
            # them created two batches — here its first batch (our
            # session) and its second (the previous member's, which moved
            # here); every member closes all of them
            self.removed.zero_()
            for m in range(self.world):
                # member m's session of the generation before
                torch.sub(self.sess_tab[m:m + 1], 1, out=sess_dev)
                t.expire(_lib.SESS_DEV, self.removed)
            self.sessions.close(self.prev_recs[:, 0].contiguous())
            expire_ok = self.removed[0] == 2 * n * self.world
        elif not resume and self.k >= 1:
            self._expire_prev(sess_dev)
            expire_ok = self.removed[0] == 2 * n
        return self._tally(validate, acc, expire_ok)

    def _check_handshake(self, resume, sess_dev, o, bound, outcome, resp):
        """The outcome check (and, at a birth, the credentials' update) in
        one launch: a resume comes back RESUMED with the same id, password
        and timeout, the expired one beside it refused; a birth is NEW with
        member r's k-th session id (csrc/kernels/bench.hip)."""
        want = sess_dev if self.world == 1 else \
            self.sess_tab[self.rank:self.rank + 1]
        _lib.lib().bench_storm_hs(
            resume, resume and self.k >= 1, self.TIMEOUT, o['status'],
            o['sessionId'], o['timeOut'], outcome, bound, resp, want,
            self.cred_sid, self.cred_pw, self.hs_ok)
        if not resume and self.world > 1:
            # R3: every member's new session to every member
            self.prev_recs.copy_(self.recs)
            mine = torch.cat([o['sessionId'][0:1],
                              o['timeOut'][0:1].to(I64),
                              resp[24:40].view(I64)])
            self._gather(self.recs.view(-1), mine)
            self.sessions.install(self.recs)

    def _batch(self):
        n = self.n
        return B.RequestBatch(n, self.opcode, self.drv.xids(n), self.arg,
                              self.path_off, self.path_len, self.data_off,
                              self.data_len, self.acl_id, self.path_arena,
                              self.data_arena, self.acl_off, self.acl_len,
                              self.acl_arena)

    def _check_replies(self, rb, rep):
        """The replies' check (counted into chk) and the batch's largest
        zxid (into last_zxid), one fused pass (csrc/kernels/bench.hip)."""
        self.chk.zero_()
        _lib.lib().bench_check_writes(self.n, rep.status, rep.err, rep.xid,
                                      rb.xid, rep.pay_len, self.want_len, -1,
                                      rep.zxid, self.chk, self.last_zxid)

    def _expire_prev(self, sess_dev):
        """The previous session expires: both of its batches go (its id, the
        current one's less one, through TC_SESS); `removed` counts them."""
        sess_dev.sub_(1)
        self.removed.zero_()
        self.tree.expire(_lib.SESS_DEV, self.removed)
        self.sessions.close(sess_dev)        # (the expired id, on the device)

    def _tally(self, validate, acc, expire_ok):
        if not validate:
            return None
        good = torch.where(self.hs_ok[0] & self.len_ok[0] & expire_ok,
                           self.chk[0], 0)
        if acc is None:
            return good
        acc[:1] += good
        return acc

    def _step_two_streams(self, resume, sess_dev, validate, acc):
        """One member's step on two streams: the handshake (K9 encode, the
        server's session table, K1 + K9 decode, its check) on the side
        stream beside the request encode; the serve once both are done; then
        the expiry of the previous session on the side stream beside the
        reply-stream scan, decode and check.  The tree is touched by one
        stream at a time (the handshake reads the zxid counter before the
        serve, the expiry writes the tree after it, the reply decode never
        reads it)."""
        d = self.drv
        cur = torch.cuda.current_stream(self.dev)
        side = self.side
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            o, bound, outcome, resp = self._handshake(resume)
            self._check_handshake(resume, sess_dev, o, bound, outcome, resp)
        rb = self._batch()
        tx, _, total, _ = B.encode_requests(rb, d.xt, out=d.tx)
        cur.wait_stream(side)
        rx, rtotal, _, _ = d.server.serve(tx, _len(total),
                                          session=_lib.SESS_DEV,
                                          ordered=d.passes > 0,
                                          passes=max(d.passes, 1))
        expiring = not resume and self.k >= 1
        if expiring:
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                self._expire_prev(sess_dev)
        if d.rscanner is None:
            d.rscanner = B.FrameScanner(self.n, self.dev, window=d.rwindow)
        ft = d.rscanner.scan(rx, _len(rtotal))
        rep = B.decode_replies(rx, ft, d.xt, out=d.reply)
        self.last = (rb, rep)
        self._check_replies(rb, rep)
        expire_ok = True
        if expiring:
            cur.wait_stream(side)
            expire_ok = self.removed[0] == 2 * self.n
        return self._tally(validate, acc, expire_ok)

    # -- the replicated tree --------------------------------------------------

    def _stream_len(self, total, attr):
        """The byte length of a batch's encoded stream: the same every step
        (fixed-size records), read from the device once; later steps check
        it on the device (len_ok)."""
        v = getattr(self, attr)
        if v is None:
            v = int(total.item())
            setattr(self, attr, v)
            return v
        self.len_ok &= total.view(-1)[0] == v
        return v

    def _replicated_run(self, rb, resume):
        """Every member's batch applied on every member, in rank order; the
        reply stream of the client this member answers goes back to it."""
        d = self.drv
        W, r, n = self.world, self.rank, self.n
        tx, _, total, _ = B.encode_requests(rb, d.xt, out=d.tx)
        S = self._stream_len(total, 'req_bytes')
        if not hasattr(self, 'tx_all'):
            self.tx_all = torch.empty(W * S, dtype=U8, device=self.dev)
        self._gather(self.tx_all, tx[:S])
        # the client this member answers: its own, or after a move the
        # previous member's
        ans = (r - 1) % W if resume else r
        sess_dev = self.tree.counters[_lib.TC_SESS:_lib.TC_SESS + 1]
        for m in range(W):
            sess_dev.copy_(self.sess_tab[m:m + 1])
            rx, rtotal, _, _ = d.server.serve(
                self.tx_all[m * S:(m + 1) * S], S, session=_lib.SESS_DEV,
                ordered=d.passes > 0, passes=max(d.passes, 1))
            if m == ans:
                R = self._stream_len(rtotal, 'rep_bytes')
                if not hasattr(self, 'rep_out'):
                    self.rep_out = torch.empty(R + 64, dtype=U8,
                                               device=self.dev)
                    self.rep_all = torch.empty(W * R, dtype=U8,
                                               device=self.dev)
                    self.my_rx = torch.empty(R + 64, dtype=U8,
                                             device=self.dev)
                self.rep_out[:R].copy_(rx[:R])
        R = self.rep_bytes
        if resume:
            # my answers come from the member my session moved to
            self._gather(self.rep_all, self.rep_out[:R])
            src = (r + 1) % W
            self.my_rx[:R].copy_(self.rep_all[src * R:(src + 1) * R])
        else:
            self.my_rx[:R].copy_(self.rep_out[:R])
        if d.rscanner is None:
            d.rscanner = B.FrameScanner(self.n, self.dev, window=d.rwindow)
        ft = d.rscanner.scan(self.my_rx, R)
        return B.decode_replies(self.my_rx, ft, d.xt, out=d.reply)

    def cross_read(self):
        """Write visibility across members: this rank's client reads its
        current session's FIRST batch (created through the member the
        session was born on) with EXISTS at the NEXT member — the requests
        go there and the replies come back through all-gathers.  Returns
        the device count of nodes found with this session as their
        ephemeral owner (every member calls it together)."""
        if self.world < 2 or self.first is None:
            raise RuntimeError('cross_read needs an ensemble across GPUs '
                               'and a born session')
        d = self.drv
        W, r, n, dev = self.world, self.rank, self.n, self.dev
        arena, poff, plen = self.first
        z32 = torch.zeros(n, dtype=I32, device=dev)
        rb = B.RequestBatch(n, torch.full((n,), consts.OP_CODES['EXISTS'],
                                          dtype=I32, device=dev),
                            d.xids(n), z32, poff, plen,
                            torch.zeros(n, dtype=I64, device=dev), z32, z32,
                            arena, arena, self.acl_off, self.acl_len,
                            self.acl_arena)
        tx, _, total, _ = B.encode_requests(rb, d.xt, out=d.tx)
        S = int(total.item())
        sizes = self._gather(torch.empty(W, dtype=I64, device=dev),
                             torch.tensor([S], dtype=I64, device=dev)).cpu()
        Smax = int(sizes.max())
        buf = torch.zeros(Smax, dtype=U8, device=dev)
        buf[:S].copy_(tx[:S])
        allq = torch.empty(W * Smax, dtype=U8, device=dev)
        self._gather(allq, buf)
        # serve the previous rank's reads here (member r + 1 of its client)
        src = (r - 1) % W
        rx, rtotal, _, _ = d.server.serve(
            allq[src * Smax:src * Smax + int(sizes[src])], int(sizes[src]),
            session=self.sid(src, self.k))
        R = int(rtotal.item())
        ra = self._gather(torch.empty(W, dtype=I64, device=dev),
                          torch.tensor([R], dtype=I64, device=dev)).cpu()
        Rmax = int(ra.max())
        out = torch.zeros(Rmax, dtype=U8, device=dev)
        out[:R].copy_(rx[:R])
        alla = torch.empty(W * Rmax, dtype=U8, device=dev)
        self._gather(alla, out)
        dst = (r + 1) % W
        mine = alla[dst * Rmax:dst * Rmax + int(ra[dst])].clone()
        sc = B.FrameScanner(n, dev, window=256)
        ft = sc.scan(mine, int(ra[dst]))
        rep = B.decode_replies(mine, ft, d.xt)
        owner = self.sid(r, self.k)
        found = ((rep.status[:n] == 0) & (rep.err[:n] == 0) &
                 (rep.stat64[4][:n] == owner)).sum()
        return found

    def diagnose(self):
        rb, rep = self.last
        n = self.n
        e, c = torch.unique(rep.err[:n], return_counts=True)
        return {'removed': int(self.removed.item()),
                'handshakes_ok': bool(self.hs_ok.item()),
                'outcome': self.sessions.outcome[:2].cpu().tolist(),
                'err_hist': dict(zip(e.cpu().tolist(), c.cpu().tolist())),
                'status_bad': int((rep.status[:n] != 0).sum().item()),
                'pay_len_bad': int((rep.pay_len[:n] != self.want_len)
                                   .sum().item()),
                'stats': dict(self.stats),
                'counters': self.tree.counters.cpu().tolist()}


class _StormCycle(object):
    """The storm's two captured step shapes replayed in turn, the host
    bookkeeping of each step done first (see StormPipeline.capture)."""

    def __init__(self, pipe, graphs):
        self.pipe = pipe
        self.graphs = graphs

    def replay(self):
        resume = self.pipe._advance()
        self.graphs[1 if resume else 0].replay()


class WatchPipeline(object):
    """Watch fan-out across the node driven by real writes (BASELINE config
    4's data path, R1 at scale).  Every rank's GPU server keeps a watch
    table (:class:`GpuTree` ``watch_cap``); one step on rank ``r``:

      arm     the watcher session (slot 0) sends ``batch`` GET_DATA with
              watch=1 for distinct nodes (K10 -> K1 -> lookup + arm -> K13
              -> K1 + K2-K4, every reply checked on the device)
      write   the writer session (slot 1) SET_DATAs the same nodes; each
              write fires its node's watch (lib/zk-session.js:558-574): the
              server expands the fired masks and K13-encodes one
              NodeDataChanged notification frame (xid -1) per node, in
              write order; the writes' replies are checked too
      R1      the notification streams of all ranks travel in equal-size
              slots ({bytes, frames} header + frames) through one
              ``all_gather_into_tensor`` (RCCL over xGMI with ``nccl``;
              :meth:`~zkmi.parallel.fanout.FrameFanout.gather_slots`, the
              one R1 path's sync-free transport); every rank concatenates
              them (``seg_unpack``), K1 + K8
              decodes ALL ranks' notifications and checks each on the
              device: NodeDataChanged, SyncConnected, and the path of the
              node that rank's writer set at that position

    One step delivers ``world * batch`` notifications to every rank:
    ``world**2 * batch`` deliveries node-wide (:attr:`per_step`).
    ``coll_device='cpu'`` runs the all-gather on host tensors (gloo
    rehearsal).  A step makes no device-to-host read; on one GPU, or with
    the all-gather on it, steps are captured as HIP graphs
    (:meth:`capture`)."""

    def __init__(self, tree, batch, seed=0, group=None, coll_device=None):
        import torch.distributed as dist
        if tree.watch is None:
            raise ValueError('WatchPipeline needs GpuTree(watch_cap=...)')
        self.dist = dist
        self.group = group
        on = dist.is_available() and dist.is_initialized()
        self.world = W = dist.get_world_size(group) if on else 1
        self.rank = dist.get_rank(group) if on else 0
        self.tree = tree
        # distinct nodes per step: at most the tree's leaves
        self.n = n = min(batch, tree.n_leaves)
        dev = tree.device
        self.dev = dev
        self.coll_device = torch.device(coll_device) if coll_device else dev
        self.per_step = W * W * n
        maxpath = int(tree.node_path_len.max().item())
        self.data_bytes = min(tree.data_bytes, 128)
        self.j = torch.arange(n, dtype=I64, device=dev)
        self.jw = torch.arange(W * n, dtype=I64, device=dev) % n
        self.rank_of = torch.arange(W * n, dtype=I64, device=dev) // n
        # the sessions' next xid, on the device: a captured step replays
        # with new xids
        self.xid_iota = torch.arange(n, dtype=I64, device=dev)
        self.xid_dev = torch.zeros(1, dtype=I64, device=dev)
        self.ops_get = torch.full((n,), consts.OP_CODES['GET_DATA'],
                                  dtype=I32, device=dev)
        self.ops_set = torch.full((n,), consts.OP_CODES['SET_DATA'],
                                  dtype=I32, device=dev)
        self.one32 = torch.ones(n, dtype=I32, device=dev)
        self.neg32 = torch.full((n,), -1, dtype=I32, device=dev)
        self.zero32 = torch.zeros(n, dtype=I32, device=dev)
        self.zero64 = torch.zeros(n, dtype=I64, device=dev)
        g = torch.Generator(device=dev)
        g.manual_seed(seed + 23)
        self.data_arena = torch.randint(0, 256, (n * self.data_bytes + 16,),
                                        dtype=U8, device=dev, generator=g)
        self.data_off = self.j * self.data_bytes
        self.data_len = torch.full((n,), self.data_bytes, dtype=I32,
                                   device=dev)
        self.acl_off = torch.zeros(1, dtype=I64, device=dev)
        self.acl_len = torch.zeros(1, dtype=I32, device=dev)
        self.acl_arena = torch.zeros(16, dtype=U8, device=dev)
        self.tx = torch.empty(n * (33 + maxpath + self.data_bytes) + 64,
                              dtype=U8, device=dev)
        self.xt = B.XidTable(bits=max(12, (n - 1).bit_length() + 1),
                             device=dev)
        rep_max = 4 + 16 + 4 + max(tree.data_bytes, 128) + 68
        self.server = GpuServer(tree, n, n * rep_max + 64,
                                window=B.frame_window(33 + maxpath +
                                                      self.data_bytes),
                                seq_order=False)
        self.rscan = B.FrameScanner(n, dev, window=B.frame_window(rep_max))
        self.reply = B.alloc_replies(n, dev)
        # R1 slots: one notification stream per rank
        rec = 4 + 16 + 4 + 4 + 4 + maxpath
        self.rec_max = rec
        self.slot = (16 + n * rec + 15) & ~15
        from ..parallel.fanout import FrameFanout
        self.fan = FrameFanout(group, device=dev,
                               coll_device=self.coll_device)
        self.pstats = None
        self.nscan = B.FrameScanner(W * n, dev, window=B.frame_window(rec))
        self.nreply = B.alloc_replies(W * n, dev)
        self.nxt = B.XidTable(bits=10, device=dev)
        self.sid_w = (2 << 56) | (self.rank + 1)
        self.sid_wr = (3 << 56) | (self.rank + 1)
        self.seed = seed
        self.step_no = 0
        self.last = None
        self.stats = {'armed': 0, 'written': 0, 'notified': 0}

    def _affine(self, rank, step):
        """(a, b) of the distinct nodes rank ``rank`` watches and writes at
        ``step``: node leaf0 + (a * j + b) % n_leaves, a coprime with
        n_leaves (a permutation, so the batch's nodes are distinct)."""
        import math
        nl = self.tree.n_leaves
        h = (rank + 1) * 0x9E3779B97F4A7C15 + (step + 1) * 0xBF58476D1CE4E5B9 \
            + self.seed * 0x94D049BB133111EB
        h &= (1 << 62) - 1
        a = (h % max(nl - 1, 1)) + 1
        while math.gcd(a, nl) != 1:
            a += 1
        b = (h >> 20) % nl
        return a, b

    def _batch(self, ops, arg, idx, xid, data):
        t = self.tree
        poff = t.node_path_off[idx]
        plen = t.node_path_len[idx]
        if data:
            doff, dlen = self.data_off, self.data_len
        else:
            doff, dlen = self.zero64, self.zero32
        return B.RequestBatch(self.n, ops, xid, arg, poff, plen, doff, dlen,
                              self.zero32, t.path_arena, self.data_arena,
                              self.acl_off, self.acl_len, self.acl_arena)

    def _xids(self):
        x = ((self.xid_iota + self.xid_dev) & 0x7fffffff).to(I32)
        self.xid_dev.add_(self.n)
        return x

    @property
    def capturable(self):
        """The R1 all-gather is captured with the step when it runs on this
        GPU (RCCL); a gloo rehearsal's host all-gather is not."""
        return self.world == 1 or self.coll_device == self.dev

    def capture(self, acc, cycle=8):
        """``cycle`` HIP graphs, replayed in turn: a step's watched and
        written nodes are an affine permutation the host picks per step
        (:meth:`_affine`), so each graph holds one step of a cycle of
        ``cycle`` node sets; xids come from a device counter."""
        return _capture_steps(self, acc, cycle, counter='step_no')

    def _roundtrip(self, rb, session, wslot, check=None):
        tx, _, total, _ = B.encode_requests(rb, self.xt, out=self.tx)
        out, rtotal, _, _ = self.server.serve(tx, total, session=session,
                                              wslot=wslot)
        ft = self.rscan.scan(out, rtotal)
        return B.decode_replies(out, ft, self.xt, out=self.reply,
                                check=check)

    def step(self, validate=True, acc=None):
        t = self.tree
        n = self.n
        W = self.world
        L = _lib.lib()
        if acc is None:
            acc = torch.zeros(1, dtype=I64, device=self.dev)
        nl = t.n_leaves
        a, b = self._affine(self.rank, self.step_no)
        idx = t.leaf0 + (self.j * a + b) % nl
        # arm: GET_DATA watch=1 from the watcher session (slot 0)
        xid = self._xids()
        arm = acc.new_zeros(1)
        self._roundtrip(self._batch(self.ops_get, self.one32, idx, xid,
                                    False), self.sid_w, 0,
                        check=(idx, xid, t.data_len, arm))
        # write: SET_DATA of the same nodes from the writer (slot 1)
        rep = self._roundtrip(self._batch(self.ops_set, self.neg32, idx,
                                          self._xids(), True),
                              self.sid_wr, 1)
        wrote = ((rep.status[:n] == 0) & (rep.err[:n] == 0)).sum()
        # R1: every rank's notification stream to every rank (FrameFanout's
        # fixed-slot transport: no host read in the step)
        nbuf, ntotal, _, ncount = self.server.notif
        self.rx, self.nrx, self.src_counts, self.pstats = \
            self.fan.gather_slots(nbuf, self.server.notif_rec_off, ncount,
                                  self.server.ecap, ntotal, self.slot)
        ft = self.nscan.scan(self.rx, self.nrx)
        nrep = B.decode_replies(self.rx, ft, self.nxt, out=self.nreply)
        self.step_no += 1
        self.last = (nrep, ft, idx)
        if not validate:
            return None
        # the nodes every rank's writer set, in write order
        want = torch.empty(W * n, dtype=I64, device=self.dev)
        for r in range(W):
            ar, br = self._affine(r, self.step_no - 1)
            want[r * n:(r + 1) * n] = t.leaf0 + (self.j * ar + br) % nl
        good = torch.zeros(1, dtype=I64, device=self.dev)
        L.bench_check_notif(W * n, n, self.zero64[:1], t.leaf0, nl,
                            t.node_path_off, t.node_path_len, t.path_arena,
                            self.rx, nrep.tensors(), good, want)
        # a step counts only if every arm and write answered OK
        ok = (arm[0] == n) & (wrote == n) & (ft.count[0] == W * n)
        acc[:1] += torch.where(ok, good, torch.zeros_like(good))
        self.stats['armed'] += n
        self.stats['written'] += n
        self.stats['notified'] += W * n
        return acc

    def diagnose(self):
        nrep, ft, idx = self.last
        return {'frames': ft.host_result(),
                'status_bad': int((nrep.status != 0).sum().item()),
                'opcodes': torch.unique(nrep.opcode).cpu().tolist(),
                'events': self.server.ev_total.cpu().tolist(),
                'overflow': self.pstats.cpu().tolist()}
