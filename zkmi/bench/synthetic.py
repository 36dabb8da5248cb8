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
request asked for.  Nothing is skipped inside a step; the only host work is
reading back the two stream lengths (needed to size the frame-scan grids).

:class:`MixPipeline` does the same for the create/set/delete mix with
version CAS and ACL encode (BASELINE config 3).
"""

import ctypes
import time

import numpy as np
import torch

from .. import consts
from ..ops import _lib
from ..ops import batch as B

I64, I32, U8 = torch.int64, torch.int32, torch.uint8


def _next_pow2(x):
    p = 1
    while p < x:
        p <<= 1
    return p


def slot_bytes(data_cap):
    """Bytes of one wire-format node slot (zk_batch.h ZkNodeStore)."""
    return _lib.SLOT_DATA + ((data_cap + 15) & ~15) + 4


class GpuTree(object):
    """``n_nodes`` znodes ``/bench/dDDDDD/nNNNNNNNN`` (``fanout`` children per
    directory) with ``data_bytes`` of random data each.  Node ``v`` has
    ``czxid == v + 1``."""

    def __init__(self, n_nodes=1_000_000, data_bytes=100, fanout=1000,
                 device=None, spare=0.25, seed=0):
        dev = torch.device(device) if device is not None else \
            torch.device('cuda', torch.cuda.current_device())
        self.device = dev
        L = _lib.lib()
        ndirs = (n_nodes + fanout - 1) // fanout
        # node order: 0 = /bench, 1..ndirs = dirs, then leaves
        paths = ['/bench'] + ['/bench/d%06d' % d for d in range(ndirs)]
        leaf0 = len(paths)
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
        self.data_bytes = data_bytes
        cap = int(nst * (1 + spare)) + 1024
        self.cap = cap
        enc = [p.encode() for p in paths]
        plen = np.fromiter((len(e) for e in enc), np.int32, nst)
        poff = np.zeros(nst, np.int64)
        np.cumsum(plen[:-1], out=poff[1:])
        arena = b''.join(enc)
        self.path_cap = int(len(arena) * (1 + spare)) + (1 << 16)
        self.path_arena = torch.zeros(self.path_cap, dtype=U8, device=dev)
        self.path_arena[:len(arena)] = torch.frombuffer(
            bytearray(arena), dtype=U8).to(dev)
        self.node_path_off = torch.zeros(cap, dtype=I64, device=dev)
        self.node_path_len = torch.zeros(cap, dtype=I32, device=dev)
        self.node_path_off[:nst] = torch.from_numpy(poff).to(dev)
        self.node_path_len[:nst] = torch.from_numpy(plen).to(dev)
        self.node_parent = torch.full((cap,), -1, dtype=I64, device=dev)
        self.node_parent[:nst] = torch.from_numpy(parents).to(dev)
        # wire-format slots; data capacity >= 128 so sets can grow
        dcap = max(data_bytes, 128)
        sb = slot_bytes(dcap)
        self.slot = sb
        self.slab_cap = cap * sb
        g = torch.Generator(device=dev)
        g.manual_seed(seed)
        self.slab = torch.randint(0, 256, (self.slab_cap,), dtype=U8,
                                  device=dev, generator=g)
        self.slot_off = torch.arange(cap, dtype=I64, device=dev) * sb
        self.data_len = torch.zeros(cap, dtype=I32, device=dev)
        self.data_len[leaf0:nst] = data_bytes
        self.slot_cap = torch.full((cap,), dcap, dtype=I32, device=dev)
        nkids = np.zeros(nst, np.int32)
        nkids[0] = ndirs
        nkids[1:leaf0] = np.bincount(np.arange(n_nodes) // fanout,
                                     minlength=ndirs)[:ndirs]
        nk = torch.from_numpy(nkids).to(dev)
        hcap = _next_pow2(2 * cap)
        self.keys = torch.zeros(hcap, dtype=I64, device=dev)
        self.vals = torch.full((hcap,), -3, dtype=I64, device=dev)
        self.counters = torch.tensor([nst, nst, len(arena), nst * sb],
                                     dtype=I64, device=dev)
        self._struct = self._make_struct(hcap - 1)
        sp = _lib.stream_ptr()
        _lib.check(L.zk_tree_fill(ctypes.byref(self._struct), 0, nst,
                                  _lib.ptr(nk), int(time.time() * 1000), sp),
                   'zk_tree_fill')
        _lib.check(L.zk_tree_build(ctypes.byref(self._struct), 0, nst, sp),
                   'zk_tree_build')
        torch.cuda.synchronize(dev)

    def _make_struct(self, mask):
        st = _lib.ZkNodeStore(self.slab.data_ptr(), self.slot_off.data_ptr(),
                              self.data_len.data_ptr(),
                              self.slot_cap.data_ptr(), self.cap)
        self.store = st
        return _lib.ZkTree(self.keys.data_ptr(), self.vals.data_ptr(), mask,
                           self.node_path_off.data_ptr(),
                           self.node_path_len.data_ptr(),
                           self.node_parent.data_ptr(),
                           self.path_arena.data_ptr(), self.path_cap,
                           self.slab_cap, self.counters.data_ptr(), st)

    @property
    def struct(self):
        return self._struct

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

    def __init__(self, tree, cap_frames, out_cap):
        self.tree = tree
        dev = tree.device
        self.rt = B.alloc_request_table(cap_frames, dev)
        self.resp = B.ResponseBatch(
            torch.empty(cap_frames, dtype=I32, device=dev),
            torch.empty(cap_frames, dtype=I32, device=dev),
            torch.empty(cap_frames, dtype=I32, device=dev),
            torch.empty(cap_frames, dtype=I64, device=dev),
            torch.empty(cap_frames, dtype=I64, device=dev),
            None, None, None,
            torch.zeros(cap_frames, dtype=I32, device=dev), None)
        self.out = torch.empty(out_cap, dtype=U8, device=dev)
        self.cap_frames = cap_frames
        self.ws = None

    def serve(self, rx, n):
        L = _lib.lib()
        ft = B.frame_scan(rx, n, cap=self.cap_frames, workspace=self.ws)
        rt = B.decode_requests(rx, ft, out=self.rt)
        r = self.resp
        r.path_off, r.path_len, r.path_arena = rt.path_off, rt.path_len, rx
        r.count = ft.count
        q = rt.struct()
        _lib.check(L.zk_tree_serve(
            ctypes.byref(self.tree.struct), _lib.ptr(rx), ctypes.byref(q),
            _lib.ptr(ft.count), self.cap_frames, _lib.ptr(r.opcode),
            _lib.ptr(r.xid), _lib.ptr(r.err), _lib.ptr(r.node),
            _lib.ptr(r.zxid), int(time.time() * 1000), _lib.stream_ptr()),
            'zk_tree_serve')
        out, rec_off, total, err = B.encode_responses(
            r, self.tree.store, self.out.numel(), out=self.out)
        return out, total, err, ft


class GetPipeline(object):
    """Batched get() over the synthetic tree (BASELINE config 2)."""

    def __init__(self, tree, batch, seed=0):
        self.tree = tree
        self.batch = batch
        dev = tree.device
        self.dev = dev
        self.xt = B.XidTable(bits=max(20, (batch - 1).bit_length() + 1),
                             device=dev)
        self.gen = torch.Generator(device=dev)
        self.gen.manual_seed(seed + 1)
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
        self.server = GpuServer(tree, n, n * (4 + 16 + 4 + dmax + 68) + 64)
        self.reply = B.alloc_replies(n, dev)
        self.xid_base = 0
        self.last = None

    def step(self, validate=True):
        t = self.tree
        n = self.batch
        idx = torch.randint(t.leaf0, t.leaf0 + t.n_leaves, (n,),
                            generator=self.gen, device=self.dev)
        xid = (torch.arange(n, dtype=I32, device=self.dev) +
               self.xid_base) & 0x7fffffff
        self.xid_base = (self.xid_base + n) & 0x7fffffff
        rb = B.RequestBatch(n, self.opcode, xid, self.arg,
                            t.node_path_off[idx], t.node_path_len[idx],
                            self.zero64, self.zero32, self.zero32,
                            t.path_arena, t.slab, self.acl_off,
                            self.acl_len, self.acl_arena)
        tx, rec_off, total, err = B.encode_requests(rb, self.xt, out=self.tx)
        ntx = int(total.item())
        rx, rtotal, rerr, _ = self.server.serve(tx, ntx)
        nrx = int(rtotal.item())
        ft = B.frame_scan(rx, nrx, cap=n)
        rep = B.decode_replies(rx, ft, self.xt, out=self.reply)
        self.last = (idx, rep, rx, ft)
        if validate:
            ok = ((rep.status[:n] == 0) & (rep.err[:n] == 0) &
                  (rep.opcode[:n] == consts.OP_CODES['GET_DATA']) &
                  (rep.xid[:n] == xid) &
                  (rep.stat64[0, :n] == idx + 1) &
                  (rep.pay_len[:n] == t.data_len[idx]))
            return ok.sum()
        return None
