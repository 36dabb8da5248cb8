"""R2 request batching on the GPU: a node's sessions share one tree sharded
by path hash, and every read travels to the rank that owns its path.

The reference pipelines all of a client's requests over its one
connection, keyed by xid (``lib/connection-fsm.js:384-408``).  On a node of
``world`` GPU sessions one step of :class:`ShardedGetPipeline`
on rank ``r`` is, per pipelined connection:

  client  draw ``batch`` GET_DATA requests over the whole tree; route them
          (csrc/kernels/route.hip): owner = FNV-1a(path) % world, stable
          split by owner; K10 encode -> one byte segment per owner;
          ``seg_pack`` cuts the stream into one fixed-capacity slot per
          owner ({bytes, records} header + payload)
  R2      ``all_to_all_single`` of the slots (RCCL over xGMI with
          ``nccl``): fixed splits, no size exchange; the local segment
          stays in a slot of its own and crosses no collective (a 16-byte
          stub stands in for it)
  server  ``seg_unpack`` appends the received payloads to this rank's own
          segment, which never moved (the router groups requests by owner
          from this rank on, so it heads the stream; route.hip
          SEG_INPLACE); K1 + K12 over that stream,
          lookup in my shard, K13 encode; ``seg_pack`` cuts the reply
          stream back into one slot per source rank (the per-source record
          counts came with the request headers)
  R2      ``all_to_all_single`` of the reply slots
  client  ``seg_unpack`` after the local replies, in the server's own
          reply buffer; K1 + K2-K4 over the replies (they come back owner
          by owner, in the order the router sent them) and the on-device
          check of every reply.  With one rank (``force_route``) the step
          copies nothing

A step makes **no device-to-host read**: every length the kernels need
travels in the slot headers, so with RCCL the whole step (collectives
included) is stream-ordered device work, and it is captured as one HIP
graph, RCCL collectives included (the step replays with one host call).
Slots are sized for the expected share of a uniform hash plus a wide
margin (``n/W + 6 sqrt(n/W) + 64`` records); a segment that would not
fit is sent empty and counted, so the reply check fails loudly instead of
reading past a slot.  With one rank there is nothing to route: the step
is the local GET pipeline (no router, no slots), unless ``force_route``:
then the W > 1 step runs as is over a one-rank RCCL group (route ->
seg_pack -> all_to_all_single -> seg_unpack on HBM tensors), which
executes and captures the multi-rank code path on one GPU.

Each rank's :class:`~zkmi.bench.synthetic.GpuTree` indexes only its shard
(``shard=(rank, world)``): a read that reached the wrong rank would answer
NO_NODE and fail the check.  ``coll_device='cpu'`` runs the all-to-alls on
host tensors (a gloo rehearsal on ranks that share one GPU).
"""

import math

import torch
import torch.distributed as dist

from .. import consts
from ..ops import _lib
from ..ops import batch as B
from ..bench.synthetic import _GET_SRV_GROUP, _SERVE_RO, _i64

I64, I32, U8 = torch.int64, torch.int32, torch.uint8

SEG_HDR = 16


def _r16(x):
    return (int(x) + 15) & ~15


# xGMI: 7 point-to-point links per MI355X, ~153 GB/s each, both directions
# together (cdna guides): one direction of one link
XGMI_LINK_GBS = 76.5


def xgmi_lower_bound_ms(slot_bytes, world):
    """A lower bound on one step's all-to-all time: every rank sends one
    slot to each peer over that peer's own link, all links at once, so a
    step's collectives need at least ``sum(slot bytes) / one link``."""
    if world <= 1:
        return 0.0
    return sum(slot_bytes) / (XGMI_LINK_GBS * 1e9) * 1e3


def slot_records(n, world):
    """Records one per-peer slot holds: the uniform share plus 6 standard
    deviations and a constant margin (a hash split of ``n`` requests over
    ``world`` owners overflowing it is a < 1e-9 event)."""
    if world == 1:
        return n
    m = n / world
    return int(math.ceil(m + 6 * math.sqrt(m) + 64))


class ShardedGetPipeline(object):
    """Sharded GET over ``streams`` pipelined connections per rank (their
    phases interleaved on separate HIP streams, as in
    :class:`~zkmi.bench.synthetic.GetPipeline`)."""

    # client | R2 out | server decode | tree + encode | R2 back | client
    PHASES = 6

    def __init__(self, tree, batch, seed=0, group=None, coll_device=None,
                 streams=1, force_route=False):
        on = dist.is_available() and dist.is_initialized()
        self.group = group
        self.world = W = dist.get_world_size(group) if on else 1
        self.rank = dist.get_rank(group) if on else 0
        if force_route and not on:
            raise ValueError('force_route needs a process group')
        # the multi-rank step (router, slots, all-to-alls): always with
        # more than one rank, and on one rank when forced
        self.route = W > 1 or force_route
        if tree.shard is not None and tuple(tree.shard) != (self.rank, W):
            raise ValueError('tree shard %r on rank %d of %d'
                             % (tree.shard, self.rank, W))
        self.tree = tree
        self.batch = batch
        self.dev = dev = tree.device
        self.coll = torch.device(coll_device) if coll_device else dev
        self.seed = seed
        # device counters: requests [overflow, bytes to peers, records to
        # peers], replies [overflow, bytes to peers, -], received [bytes]
        self.req_stats = torch.zeros(3, dtype=I64, device=dev)
        self.rep_stats = torch.zeros(3, dtype=I64, device=dev)
        self.recv_stats = torch.zeros(1, dtype=I64, device=dev)
        self.steps = 0
        self.subs = []
        self.comm = None
        if streams > 1:
            per = [batch // streams + (1 if k < batch % streams else 0)
                   for k in range(streams)]
            self.subs = [_Conn(self, m, seed * streams + k)
                         for k, m in enumerate(per)]
            self.streams = [torch.cuda.Stream(dev) for _ in per]
            # one stream issues every collective (the communicator runs
            # them in order anyway): the connections' kernels overlap the
            # all-to-alls, and a captured graph has one collective chain
            if self.route and self.coll == dev:
                self.comm = torch.cuda.Stream(dev)
        else:
            self.subs = [_Conn(self, batch, seed)]
            self.streams = None
        self.last = None

    # -- collectives ----------------------------------------------------------

    def splits(self, slot):
        """The all-to-all's split sizes: a slot per peer, the 16-byte stub
        for this rank (its segment stays local, see route.hip slot_at)."""
        return [SEG_HDR if w == self.rank else slot
                for w in range(self.world)]

    def a2a(self, out, inp, slot):
        """``all_to_all_single`` of the slots on the collective device
        (device tensors with RCCL; host staging for a gloo rehearsal)."""
        sp = self.splits(slot)
        if self.coll == self.dev:
            if self.comm is None:
                dist.all_to_all_single(out, inp, sp, sp, group=self.group)
                return out
            cur = torch.cuda.current_stream(self.dev)
            self.comm.wait_stream(cur)
            with torch.cuda.stream(self.comm):
                dist.all_to_all_single(out, inp, sp, sp, group=self.group)
            cur.wait_stream(self.comm)
            return out
        o = torch.empty(out.shape, dtype=out.dtype, device=self.coll)
        dist.all_to_all_single(o, inp.to(self.coll), sp, sp,
                               group=self.group)
        out.copy_(o)
        return out

    @property
    def capturable(self):
        """The whole step is device work on our streams when the
        collectives run on the device (RCCL): it is captured with them.  A
        gloo rehearsal stages through the host and runs eager."""
        return not self.route or self.coll == self.dev

    def capture(self, acc):
        if not self.capturable:
            raise RuntimeError('host-staged collectives run eager')
        for c in self.subs:
            c.device_seed()
        torch.cuda.synchronize(self.dev)
        g = torch.cuda.CUDAGraph()
        # Under capture the collectives go on the capture's origin stream:
        # RCCL work issued from a forked stream of the capture faulted in
        # hipStreamEndCapture (tools/microbench/fr_probe.py: --mode comm vs
        # origin); the connections' own kernels still run on their streams.
        origin = torch.cuda.Stream(self.dev)
        comm, self.comm = self.comm, origin if self.comm is not None else None
        try:
            with torch.cuda.graph(g, stream=origin,
                                  capture_error_mode='thread_local'):
                self.step(acc=acc)
        finally:
            self.comm = comm
        self.graph = g
        return g

    # -- one step -------------------------------------------------------------

    def step(self, validate=True, acc=None):
        if validate and acc is None:
            acc = torch.zeros(1, dtype=I64, device=self.dev)
        self.steps += 1
        if self.streams is None:
            for _ in self.subs[0].phases(validate, acc):
                pass
            self.last = self.subs[0].last
            return acc if validate else None
        cur = torch.cuda.current_stream(self.dev)
        live = []
        for c, s in zip(self.subs, self.streams):
            s.wait_stream(cur)
            live.append((s, c.phases(validate, acc)))
        # round-robin: every rank issues the connections' collectives in the
        # same order (a requirement of RCCL / gloo), and one connection's
        # kernels overlap the other's all-to-all
        while live:
            nxt = []
            for s, g in live:
                with torch.cuda.stream(s):
                    if next(g, StopIteration) is not StopIteration:
                        nxt.append((s, g))
            live = nxt
        for s in self.streams:
            cur.wait_stream(s)
        self.last = self.subs[-1].last
        return acc if validate else None

    # -- reporting ------------------------------------------------------------

    @property
    def stats(self):
        """Host view of the R2 counters (one device read; call after the
        timed steps): payload bytes sent to / received from the other
        ranks, requests served remotely, overflowing segments, and the
        bytes every all-to-all moves between ranks (slots, padding
        included)."""
        rq = self.req_stats.cpu().tolist()
        rp = self.rep_stats.cpu().tolist()
        rv = self.recv_stats.cpu().tolist()
        W = self.world
        wire = sum((W - 1) * (c.req_slot + c.rep_slot) for c in self.subs) \
            * self.steps if W > 1 else 0
        # bytes the step's kernels copy per connection at most: the peers'
        # segments into the slots (seg_pack) and out of them (seg_unpack),
        # requests and replies (a uniform hash sends (W-1)/W of them); this
        # rank's own segments stay in place and the all-to-all moves the
        # peers' slots only
        copied = sum(2 * (c.n * c.req_max + c.n * c.rep_max) * (W - 1) // W
                     for c in self.subs)
        slots = [b for c in self.subs for b in (c.req_slot, c.rep_slot)]
        return {'bytes_sent': rq[1] + rp[1], 'bytes_recv': rv[0],
                'remote_reqs': rq[2], 'overflow_segments': rq[0] + rp[0],
                'wire_bytes_sent': wire, 'steps': self.steps,
                'req_slot_bytes': [c.req_slot for c in self.subs],
                'rep_slot_bytes': [c.rep_slot for c in self.subs],
                'xgmi_lower_bound_ms': xgmi_lower_bound_ms(slots, W),
                'copy_bytes_per_step_max': copied,
                'local_bytes_through_collective': 2 * SEG_HDR * len(self.subs)}


class _Conn(object):
    """One pipelined connection of a :class:`ShardedGetPipeline`: its own
    request / reply buffers, xid table, GPU server and slots."""

    def __init__(self, pipe, n, seed):
        from ..bench.synthetic import GpuServer
        self.p = pipe
        t = pipe.tree
        W = pipe.world
        dev = pipe.dev
        self.n = n
        self.seed = seed
        self.step_no = 0
        self.xid_base = 0
        self.gstate = None
        self.xt = B.XidTable(bits=max(20, (n - 1).bit_length() + 1),
                             device=dev)
        e64 = lambda: torch.empty(n, dtype=I64, device=dev)   # noqa: E731
        e32 = lambda: torch.empty(n, dtype=I32, device=dev)   # noqa: E731
        self.idx, self.xid, self.poff, self.plen = e64(), e32(), e64(), e32()
        if pipe.route:
            self.idx_s, self.xid_s, self.poff_s, self.plen_s = (
                e64(), e32(), e64(), e32())
            self.owner = e32()
            self.counts = torch.empty(W, dtype=I64, device=dev)
            self.rws = torch.empty(_lib.lib().route_workspace(n, W),
                                   dtype=I64, device=dev)
        else:
            self.idx_s, self.xid_s, self.poff_s, self.plen_s = (
                self.idx, self.xid, self.poff, self.plen)
        self.opcode = torch.full((n,), consts.OP_CODES['GET_DATA'],
                                 dtype=I32, device=dev)
        self.zero32 = torch.zeros(n, dtype=I32, device=dev)
        self.zero64 = torch.zeros(n, dtype=I64, device=dev)
        self.acl_off = torch.zeros(1, dtype=I64, device=dev)
        self.acl_len = torch.zeros(1, dtype=I32, device=dev)
        self.acl_arena = torch.zeros(16, dtype=U8, device=dev)
        maxpath = int(t.node_path_len.max().item())
        maxdata = int(t.data_len.max().item())
        self.req_max = 17 + maxpath
        self.rep_max = 4 + 16 + 4 + maxdata + 68
        k = slot_records(n, W)
        self.slot_recs = k
        cap = W * k                      # requests this rank can receive
        self.req_slot = _r16(SEG_HDR + k * self.req_max)
        self.rep_slot = _r16(SEG_HDR + k * self.rep_max)
        # routed: the request stream buffer is also the server's input (the
        # peers' segments land after this rank's own, which stays in place),
        # and the server's reply buffer the client's (same for the replies)
        self.tx = torch.empty(max(n * self.req_max,
                                  W * (self.req_slot - SEG_HDR)) + 64,
                              dtype=U8, device=dev)
        self.server = GpuServer(t, cap, max(cap * self.rep_max,
                                            W * (self.rep_slot - SEG_HDR))
                                + 64, window=B.frame_window(self.req_max),
                                seq_order=False, group=_GET_SRV_GROUP)
        # every routed request is a GET_DATA: the serve's read-only instance
        self.server.read_only = _SERVE_RO
        # the replies to this connection's own n requests come back
        lo, hi = t.data_dist or (t.data_bytes, t.data_bytes)
        self.rscanner = B.FrameScanner(n, dev,
                                       window=B.frame_window(self.rep_max),
                                       frame_hint=4 + 16 + 4 + 68 +
                                       (lo + hi) // 2)
        self.reply = B.alloc_replies(n, dev)
        if pipe.route:
            u8 = lambda m: torch.empty(m, dtype=U8, device=dev)  # noqa: E731
            # the collective buffers: the peers' slots + this rank's stub;
            # this rank's own slots apart
            cq = (W - 1) * self.req_slot + SEG_HDR
            cp = (W - 1) * self.rep_slot + SEG_HDR
            self.sq, self.rq = u8(cq), u8(cq)
            self.sp, self.rp = u8(cp), u8(cp)
            # this rank's own segments stay in the streams (SEG_INPLACE):
            # only their 16-byte {bytes, records} headers are written apart
            self.sq_self, self.sp_self = u8(SEG_HDR), u8(SEG_HDR)
            self.nrx = torch.zeros(1, dtype=I64, device=dev)
            self.ncrx = torch.zeros(1, dtype=I64, device=dev)
            self.src_counts = torch.zeros(W, dtype=I64, device=dev)
            self.back_counts = torch.zeros(W, dtype=I64, device=dev)
        self.last = None

    def base_seed(self):
        """Per-rank, per-connection request seed (bench.hip draws step s
        from base * golden + s)."""
        return self.seed + 1000003 * (self.p.rank + 1)

    def device_seed(self):
        """Draw the requests from a device {seed, step} pair advanced on
        the device, so a captured graph replays new batches."""
        if self.gstate is None:
            self.gstate = torch.tensor([self.base_seed(), self.step_no],
                                       dtype=I64, device=self.p.dev)

    def phases(self, validate, acc):
        """One step of this connection as a generator, yielding between the
        PHASES phases (the parent interleaves connections there)."""
        p = self.p
        t = p.tree
        n = self.n
        W = p.world
        L = _lib.lib()
        seed = (self.base_seed() * 0x9E3779B97F4A7C15 + self.step_no) \
            & (2**64 - 1)
        self.step_no += 1
        L.bench_gen_get(n, _i64(seed), t.leaf0, t.n_leaves, self.xid_base,
                        t.node_pw, self.idx, self.xid, self.poff, self.plen,
                        self.gstate)
        self.xid_base = (self.xid_base + n) & 0x7fffffff
        if p.route:
            # grouped by owner from this rank on (rotation): the local
            # segment heads the stream and is never copied
            L.route_requests(n, W, self.poff, self.plen, t.path_arena,
                             self.idx, self.xid, self.owner, self.idx_s,
                             self.xid_s, self.poff_s, self.plen_s,
                             self.counts, self.rws, p.rank)
        rb = B.RequestBatch(n, self.opcode, self.xid_s, self.zero32,
                            self.poff_s, self.plen_s, self.zero64,
                            self.zero32, self.zero32, t.path_arena, t.slab,
                            self.acl_off, self.acl_len, self.acl_arena)
        tx, rec_off, total, _ = B.encode_requests(rb, self.xt, out=self.tx)
        if p.route:
            L.seg_pack(tx, rec_off, None, n, total, self.counts, W, p.rank,
                       self.req_slot, self.sq, p.req_stats, self.sq_self,
                       True)
        yield
        if p.route:
            p.a2a(self.rq, self.sq, self.req_slot)
        yield
        if p.route:
            # the peers' segments after this rank's own, in the request
            # stream's buffer (its peer part went out with seg_pack)
            L.seg_unpack(self.rq, W, p.rank, self.req_slot, tx,
                         self.nrx, self.src_counts, None, self.sq_self, True)
            rxq, nrx = tx, self.nrx
        else:
            rxq, nrx = tx, total
        srv = self.server.serve_steps(rxq, nrx)
        next(srv)
        yield
        for _ in srv:
            pass
        rout, rtotal, _, ft = self.server.result
        if p.route:
            # replies in request order = source rank order; the source
            # counts came with the request slots' headers
            L.seg_pack(rout, self.server.last_rec_off, ft.count,
                       self.server.cap_frames, rtotal, self.src_counts, W,
                       p.rank, self.rep_slot, self.sp, p.rep_stats,
                       self.sp_self, True)
        yield
        if p.route:
            p.a2a(self.rp, self.sp, self.rep_slot)
        yield
        if p.route:
            L.seg_unpack(self.rp, W, p.rank, self.rep_slot, rout,
                         self.ncrx, self.back_counts, p.recv_stats,
                         self.sp_self, True)
            crx, ncrx = rout, self.ncrx
        else:
            crx, ncrx = rout, rtotal
        cft = self.rscanner.scan(crx, ncrx)
        chk = (self.idx_s, self.xid_s, t.data_len, acc, t.slab_all,
               t.slot_off) if validate else None
        rep = B.decode_replies(crx, cft, self.xt, out=self.reply, check=chk,
                               tick=self.gstate if validate else None)
        if self.gstate is not None and not validate:
            self.gstate[1:].add_(1)
        self.last = (rep, crx, cft)
