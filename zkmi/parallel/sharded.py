"""R2 request batching on the GPU: a node's sessions share one tree sharded
by path hash, and every read travels to the rank that owns its path.

The reference pipelines all of a client's requests over its one
connection, keyed by xid (``lib/connection-fsm.js:384-408``).  On a node of
``world`` GPU sessions one step of :class:`ShardedGetPipeline`
on rank ``r`` is:

  client  draw ``batch`` GET_DATA requests over the whole tree;
          route them (csrc/kernels/route.hip): owner = FNV-1a(path) % world,
          stable split by owner; K10 encode -> one byte segment per owner
  R2      exchange (bytes, requests) per rank pair — ``all_to_all_single``
          of a [world, 2] int64 tensor, the one size exchange — then
          ``all_to_all_single`` of the encoded request bytes (RCCL over xGMI
          with ``nccl``)
  server  K1 + K12 over the received stream (every rank's requests for my
          shard, in rank order), lookup in my shard, K13 encode
  R2      reply sizes per source rank from the reply frame offsets, one
          ``all_to_all_single`` of them, one of the reply bytes back
  client  K1 + K2-K4 over the replies (they come back owner by owner, in
          the order the router sent them) and the on-device check

Host reads per step: the size table after the request-size exchange and
the reply-size table (two small D2H copies; ``all_to_all_single`` takes its
splits on the host).  Each rank's :class:`~zkmi.bench.synthetic.GpuTree`
indexes only its shard (``shard=(rank, world)``): a read that reached the
wrong rank would answer NO_NODE and fail the check.
"""

import torch
import torch.distributed as dist

from .. import consts
from ..ops import _lib
from ..ops import batch as B
from ..bench.synthetic import _i64

I64, I32, U8 = torch.int64, torch.int32, torch.uint8


class ShardedGetPipeline(object):

    def __init__(self, tree, batch, seed=0, group=None, coll_device=None):
        from ..bench.synthetic import GpuServer
        on = dist.is_available() and dist.is_initialized()
        self.group = group
        self.world = W = dist.get_world_size(group) if on else 1
        self.rank = dist.get_rank(group) if on else 0
        if tree.shard is not None and tuple(tree.shard) != (self.rank, W):
            raise ValueError('tree shard %r on rank %d of %d'
                             % (tree.shard, self.rank, W))
        self.tree = tree
        self.batch = n = batch
        self.dev = dev = tree.device
        self.coll = torch.device(coll_device) if coll_device else dev
        self.seed = seed
        self.step_no = 0
        self.xid_base = 0
        self.xt = B.XidTable(bits=max(20, (n - 1).bit_length() + 1),
                             device=dev)
        e64 = lambda: torch.empty(n, dtype=I64, device=dev)   # noqa: E731
        e32 = lambda: torch.empty(n, dtype=I32, device=dev)   # noqa: E731
        self.idx, self.xid, self.poff, self.plen = e64(), e32(), e64(), e32()
        self.idx_s, self.xid_s, self.poff_s, self.plen_s = (e64(), e32(),
                                                            e64(), e32())
        self.owner = e32()
        self.counts = torch.empty(W, dtype=I64, device=dev)
        L = _lib.lib()
        self.rws = torch.empty(L.route_workspace(n, W), dtype=I64,
                               device=dev)
        self.opcode = torch.full((n,), consts.OP_CODES['GET_DATA'],
                                 dtype=I32, device=dev)
        self.zero32 = torch.zeros(n, dtype=I32, device=dev)
        self.zero64 = torch.zeros(n, dtype=I64, device=dev)
        self.acl_off = torch.zeros(1, dtype=I64, device=dev)
        self.acl_len = torch.zeros(1, dtype=I32, device=dev)
        self.acl_arena = torch.zeros(16, dtype=U8, device=dev)
        self.maxpath = int(tree.node_path_len.max().item())
        self.req_max = 17 + self.maxpath
        self.rep_max = 4 + 16 + 4 + max(tree.data_bytes, 128) + 68
        self.tx = torch.empty(n * self.req_max + 64, dtype=U8, device=dev)
        self._server_cap = 0
        self._mk_server(n + n // 4 + 1024)
        self.rscanner = B.FrameScanner(n, dev,
                                       window=B.frame_window(self.rep_max))
        self.reply = B.alloc_replies(n, dev)
        self.crx = torch.empty(n * self.rep_max + 64, dtype=U8, device=dev)
        self.GpuServer = GpuServer
        self.stats = {'bytes_sent': 0, 'bytes_recv': 0, 'remote_reqs': 0}
        self.last = None

    def _mk_server(self, cap):
        from ..bench.synthetic import GpuServer
        self._server_cap = cap
        self.server = GpuServer(self.tree, cap, cap * self.rep_max + 64,
                                window=B.frame_window(self.req_max))
        self.rxq = torch.empty(cap * self.req_max + 64, dtype=U8,
                               device=self.dev)

    # -- collectives ----------------------------------------------------------

    def _a2a(self, out, inp, out_splits, in_splits):
        """``all_to_all_single`` on the collective device (device tensors
        with RCCL; host staging for a gloo rehearsal)."""
        if self.coll == self.dev:
            dist.all_to_all_single(out, inp, out_splits, in_splits,
                                   group=self.group)
            return out
        o = torch.empty(out.shape, dtype=out.dtype, device=self.coll)
        dist.all_to_all_single(o, inp.to(self.coll), out_splits, in_splits,
                               group=self.group)
        out.copy_(o)
        return out

    @staticmethod
    def _seg_bytes(rec_off, total, counts):
        """Bytes of each owner's contiguous run of records: offsets of the
        runs' first records (the stream total closes the last run)."""
        ext = torch.cat([rec_off, total.view(1)])
        ends = torch.cumsum(counts, 0)
        return ext[ends] - ext[ends - counts]

    # -- one step -------------------------------------------------------------

    def step(self, validate=True, acc=None):
        t = self.tree
        n = self.batch
        W = self.world
        L = _lib.lib()
        if validate and acc is None:
            acc = torch.zeros(1, dtype=I64, device=self.dev)
        seed = ((self.rank + 1) * 0x9E3779B97F4A7C15 + self.seed * 7919 +
                self.step_no) & (2**64 - 1)
        self.step_no += 1
        L.bench_gen_get(n, _i64(seed), t.leaf0, t.n_leaves, self.xid_base,
                        t.node_pw, self.idx, self.xid, self.poff, self.plen)
        self.xid_base = (self.xid_base + n) & 0x7fffffff
        L.route_requests(n, W, self.poff, self.plen, t.path_arena, self.idx,
                         self.xid, self.owner, self.idx_s, self.xid_s,
                         self.poff_s, self.plen_s, self.counts, self.rws)
        rb = B.RequestBatch(n, self.opcode, self.xid_s, self.zero32,
                            self.poff_s, self.plen_s, self.zero64,
                            self.zero32, self.zero32, t.path_arena, t.slab,
                            self.acl_off, self.acl_len, self.acl_arena)
        tx, rec_off, total, _ = B.encode_requests(rb, self.xt, out=self.tx)
        if W == 1:
            m = n
            rxq, nrx = tx, total
        else:
            # the size exchange: (bytes, requests) for every rank pair
            send = torch.stack([self._seg_bytes(rec_off, total, self.counts),
                                self.counts], 1).contiguous()
            recv = torch.empty_like(send)
            self._a2a(recv, send, None, None)
            sz = torch.cat([send, recv]).cpu().tolist()      # host read 1
            sbytes = [r[0] for r in sz[:W]]
            rbytes = [r[0] for r in sz[W:]]
            rcounts = [r[1] for r in sz[W:]]
            m = sum(rcounts)
            nrx = sum(rbytes)
            if m > self._server_cap:
                self._mk_server(m + m // 4)
            rxq = self._a2a(self.rxq[:nrx], tx[:sum(sbytes)], rbytes, sbytes)
            self.stats['bytes_sent'] += sum(sbytes) - sbytes[self.rank]
            self.stats['bytes_recv'] += nrx - rbytes[self.rank]
            self.stats['remote_reqs'] += m - rcounts[self.rank]
        rout, rtotal, _, _ = self.server.serve(rxq, nrx)
        if W == 1:
            crx, ncrx = rout, rtotal
        else:
            rc = torch.tensor(rcounts, dtype=I64, device=self.dev)
            rep_bytes = self._seg_bytes(self.server.last_rec_off[:m], rtotal,
                                        rc)
            back = torch.empty_like(rep_bytes)
            self._a2a(back, rep_bytes, None, None)
            sz = torch.cat([rep_bytes, back]).cpu().tolist()  # host read 2
            out_b, in_b = sz[:W], sz[W:]
            ncrx = sum(in_b)
            crx = self._a2a(self.crx[:ncrx], rout[:sum(out_b)], in_b, out_b)
        ft = self.rscanner.scan(crx, ncrx)
        rep = B.decode_replies(crx, ft, self.xt, out=self.reply)
        self.last = (rep, crx, ft)
        if not validate:
            return None
        L.bench_check_get(n, rep.tensors(), self.idx_s, self.xid_s,
                          t.data_len, acc)
        return acc
