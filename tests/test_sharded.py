"""R2 on the GPU (zkmi/parallel/sharded.py, csrc/kernels/route.hip): reads
routed to the rank owning the path's hash shard, bytes moved with
all_to_all.  The multi-rank case runs two ranks on one GPU with gloo
collectives (RCCL needs one GPU per rank) and checks the routed replies
byte for byte against serving the same requests from an unsharded tree."""

import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_router_matches_host_hash(gpu):
    """route.hip's owners equal the host FNV-1a mirror; the split is stable
    and grouped by owner."""
    from zkmi.bench.synthetic import GpuTree, path_owner
    from zkmi.parallel.sharded import ShardedGetPipeline
    tree = GpuTree(20000, 37, fanout=100, device=gpu, seed=0)
    pipe = ShardedGetPipeline(tree, 5000)
    pipe.step()
    c = pipe.subs[0]
    from zkmi.ops import _lib
    L = _lib.lib()
    i64 = lambda: torch.empty(5000, dtype=torch.int64, device=gpu)  # noqa
    i32 = lambda: torch.empty(5000, dtype=torch.int32, device=gpu)  # noqa
    owner, idx_s, xid_s, poff_s, plen_s = i32(), i64(), i32(), i64(), i32()
    for W in (3, 8):
        rws = torch.empty(L.route_workspace(5000, W), dtype=torch.int64,
                          device=gpu)
        cnt = torch.empty(W, dtype=torch.int64, device=gpu)
        L.route_requests(5000, W, c.poff, c.plen, tree.path_arena, c.idx,
                         c.xid, owner, idx_s, xid_s, poff_s, plen_s, cnt,
                         rws)
        arena = tree.path_arena.cpu().numpy().tobytes()
        po, pl = c.poff.cpu().tolist(), c.plen.cpu().tolist()
        want = path_owner([arena[o:o + n] for o, n in zip(po, pl)], W)
        assert owner.cpu().numpy().tolist() == want.tolist()
        order = np.argsort(want, kind='stable')
        assert idx_s.cpu().numpy().tolist() == \
            c.idx.cpu().numpy()[order].tolist()
        assert cnt.cpu().tolist() == np.bincount(want, minlength=W).tolist()
        # grouped from owner `me` on (rotation): the local group first
        me = W - 2
        L.route_requests(5000, W, c.poff, c.plen, tree.path_arena, c.idx,
                         c.xid, owner, idx_s, xid_s, poff_s, plen_s, cnt,
                         rws, me)
        order = np.argsort((want - me) % W, kind='stable')
        assert idx_s.cpu().numpy().tolist() == \
            c.idx.cpu().numpy()[order].tolist()
        assert cnt.cpu().tolist() == np.bincount(want, minlength=W).tolist()


def test_seg_pack_unpack_roundtrip(gpu):
    """seg_pack cuts a framed stream into per-destination slots with
    {bytes, records} headers (any byte alignment, empty segments, an
    overflowing segment sent empty and counted); seg_unpack concatenates
    slots back with the device length and per-source counts."""
    from zkmi.ops import _lib
    L = _lib.lib()
    rng = np.random.default_rng(3)
    W = 5
    counts = [7, 0, 13, 1, 30]
    sizes = rng.integers(1, 60, sum(counts))
    stream = rng.integers(0, 256, int(sizes.sum()), dtype=np.uint8)
    rec_off = np.zeros(len(sizes), np.int64)
    rec_off[1:] = np.cumsum(sizes)[:-1]
    dev = gpu
    src = torch.from_numpy(np.concatenate([stream, np.zeros(64, np.uint8)]))\
        .to(dev)
    ro = torch.from_numpy(rec_off).to(dev)
    total = torch.tensor([len(stream)], dtype=torch.int64, device=dev)
    cnt = torch.tensor(counts, dtype=torch.int64, device=dev)
    segs = []
    f = 0
    for c in counts:
        a = rec_off[f] if f < len(sizes) else len(stream)
        b = rec_off[f + c] if f + c < len(sizes) else len(stream)
        segs.append(bytes(stream[a:b]))
        f += c
    # slot payload capacity 16 * 40 bytes: segment 4 (30 records) overflows
    slot = 16 + 16 * 40
    assert len(segs[4]) > slot - 16 and max(map(len, segs[:4])) <= slot - 16
    out = torch.full((W * slot,), 0xEE, dtype=torch.uint8, device=dev)
    st = torch.zeros(3, dtype=torch.int64, device=dev)
    L.seg_pack(src, ro, None, len(sizes), total, cnt, W, 2, slot, out, st)
    ob = out.cpu().numpy().tobytes()
    for w in range(W):
        hb, hr = np.frombuffer(ob[w * slot:w * slot + 16], np.int64)
        if w == 4:
            assert (hb, hr) == (0, 0)
        else:
            assert (hb, hr) == (len(segs[w]), counts[w])
            assert ob[w * slot + 16:w * slot + 16 + hb] == segs[w]
    sent = sum(len(segs[w]) for w in range(4) if w != 2)
    assert st.cpu().tolist() == [1, sent, sum(counts[:4]) - counts[2]]
    # unpack: a shifted copy so the destination offsets are unaligned
    back = torch.zeros(W * (slot - 16) + 64, dtype=torch.uint8, device=dev)
    tot = torch.zeros(1, dtype=torch.int64, device=dev)
    rc = torch.zeros(W, dtype=torch.int64, device=dev)
    rs = torch.zeros(1, dtype=torch.int64, device=dev)
    L.seg_unpack(out, W, 1, slot, back, tot, rc, rs)
    want = b''.join(segs[:4])
    assert tot.item() == len(want)
    assert back[:len(want)].cpu().numpy().tobytes() == want
    assert rc.cpu().tolist() == counts[:4] + [0]
    assert rs.item() == len(want) - len(segs[1])
    # the local segment in a slot of its own (the all-to-all carries the
    # peers' slots and a 16-byte stub for this rank): same segments, same
    # concatenation
    me = 2
    coll = torch.full(((W - 1) * slot + 16,), 0xEE, dtype=torch.uint8,
                      device=dev)
    own = torch.full((slot,), 0xEE, dtype=torch.uint8, device=dev)
    st2 = torch.zeros(3, dtype=torch.int64, device=dev)
    L.seg_pack(src, ro, None, len(sizes), total, cnt, W, me, slot, coll, st2,
               own)
    cb, ob2 = coll.cpu().numpy().tobytes(), own.cpu().numpy().tobytes()

    def at(w):
        if w == me:
            return ob2[:slot]
        p0 = w * slot if w < me else (w - 1) * slot + 16
        return cb[p0:p0 + slot]
    for w in range(W):
        hb, hr = np.frombuffer(at(w)[:16], np.int64)
        if w == 4:
            assert (hb, hr) == (0, 0)
        else:
            assert (hb, hr) == (len(segs[w]), counts[w])
            assert at(w)[16:16 + hb] == segs[w]
    assert st2.cpu().tolist() == st.cpu().tolist()
    back2 = torch.zeros(W * (slot - 16) + 64, dtype=torch.uint8, device=dev)
    L.seg_unpack(coll, W, me, slot, back2, tot, rc, None, own)
    assert tot.item() == len(want)
    assert back2[:len(want)].cpu().numpy().tobytes() == want


def test_seg_pack_unpack_inplace(gpu):
    """SEG_INPLACE: segments in rotation order from this rank (its own
    first, at offset 0), only the own segment's header written apart, and
    the peers' payloads unpacked after it in the same buffer — the local
    bytes never move."""
    from zkmi.ops import _lib
    L = _lib.lib()
    rng = np.random.default_rng(5)
    W, me = 4, 2
    counts = [5, 9, 11, 3]                 # records owned by rank w
    rot = [(me + k) % W for k in range(W)]  # stream order: 2, 3, 0, 1
    sizes = rng.integers(1, 70, sum(counts))
    stream = rng.integers(0, 256, int(sizes.sum()), dtype=np.uint8)
    rec_off = np.zeros(len(sizes), np.int64)
    rec_off[1:] = np.cumsum(sizes)[:-1]
    segs, f = {}, 0
    for w in rot:
        a = rec_off[f] if f < len(sizes) else len(stream)
        b = rec_off[f + counts[w]] if f + counts[w] < len(sizes) \
            else len(stream)
        segs[w] = bytes(stream[a:b])
        f += counts[w]
    slot = 16 + 16 * 60
    cap = W * (slot - 16) + 64
    dev = gpu
    buf = torch.zeros(cap, dtype=torch.uint8, device=dev)
    buf[:len(stream)] = torch.from_numpy(stream).to(dev)
    ro = torch.from_numpy(rec_off).to(dev)
    total = torch.tensor([len(stream)], dtype=torch.int64, device=dev)
    cnt = torch.tensor(counts, dtype=torch.int64, device=dev)
    coll = torch.full(((W - 1) * slot + 16,), 0xEE, dtype=torch.uint8,
                      device=dev)
    hdr = torch.zeros(16, dtype=torch.uint8, device=dev)
    st = torch.zeros(3, dtype=torch.int64, device=dev)
    L.seg_pack(buf, ro, None, len(sizes), total, cnt, W, me, slot, coll, st,
               hdr, True)
    cb = coll.cpu().numpy().tobytes()
    assert tuple(np.frombuffer(hdr.cpu().numpy().tobytes(), np.int64)) == \
        (len(segs[me]), counts[me])
    for w in range(W):
        if w == me:
            continue
        p0 = w * slot if w < me else (w - 1) * slot + 16
        hb, hr = np.frombuffer(cb[p0:p0 + 16], np.int64)
        assert (hb, hr) == (len(segs[w]), counts[w])
        assert cb[p0 + 16:p0 + 16 + hb] == segs[w]
    peers = [w for w in range(W) if w != me]
    assert st.cpu().tolist() == [0, sum(len(segs[w]) for w in peers),
                                 sum(counts[w] for w in peers)]
    # the peers' part of the buffer is free once packed: scribble over it,
    # then unpack in place behind the untouched local segment
    buf[len(segs[me]):] = 0x5A
    tot = torch.zeros(1, dtype=torch.int64, device=dev)
    rc = torch.zeros(W, dtype=torch.int64, device=dev)
    L.seg_unpack(coll, W, me, slot, buf, tot, rc, None, hdr, True)
    want = b''.join(segs[w] for w in rot)
    assert tot.item() == len(want)
    assert buf[:len(want)].cpu().numpy().tobytes() == want
    assert rc.cpu().tolist() == counts


def test_sharded_get_one_rank(gpu):
    from zkmi.bench.synthetic import GpuTree
    from zkmi.parallel.sharded import ShardedGetPipeline
    tree = GpuTree(20000, 37, fanout=100, device=gpu, seed=0, shard=(0, 1))
    for streams in (1, 2):
        pipe = ShardedGetPipeline(tree, 4096, streams=streams)
        for _ in range(3):
            assert int(pipe.step().item()) == 4096
        acc = torch.zeros(1, dtype=torch.int64, device=gpu)
        g = pipe.capture(acc)
        acc.zero_()
        for _ in range(3):
            g.replay()
        assert int(acc.item()) == 3 * 4096


def _mask_zxid(stream):
    """Reply frames with the header zxid zeroed: each GPU server's zxid
    advances with the batches it served, the bodies must match exactly."""
    from zkmi import jute
    frames, _, bad = jute.scan_frames(stream)
    assert bad < 0
    return [b'%s\0\0\0\0\0\0\0\0%s' % (stream[o:o + 4], stream[o + 12:o + n])
            for o, n in frames]


def _rank(rank, world, port, q, streams):
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from zkmi.bench.synthetic import GpuTree, GpuServer
        from zkmi.ops import batch as B
        from zkmi.parallel.sharded import ShardedGetPipeline
        dev = torch.device('cuda', 0)
        n = 3000
        tree = GpuTree(20000, 37, fanout=100, device=dev, seed=0,
                       shard=(rank, world), ctime_ms=1 << 40)
        pipe = ShardedGetPipeline(tree, n, seed=5, coll_device='cpu',
                                  streams=streams)
        oks = [int(pipe.step().item()) for _ in range(3)]
        c = pipe.subs[-1]
        rep, crx, ft = pipe.last
        got = bytes(crx[:int(c.ncrx.item())].cpu().numpy().tobytes())
        # the same (routed-order) requests served by an unsharded replica
        full = GpuTree(20000, 37, fanout=100, device=dev, seed=0,
                       ctime_ms=1 << 40)
        srv = GpuServer(full, c.n, c.n * 300)
        rb = B.RequestBatch(c.n, c.opcode, c.xid_s, c.zero32, c.poff_s,
                            c.plen_s, c.zero64, c.zero32, c.zero32,
                            tree.path_arena, tree.slab, c.acl_off,
                            c.acl_len, c.acl_arena)
        tx, _, total, _ = B.encode_requests(rb, B.XidTable(bits=14,
                                                           device=dev))
        out, rtotal, _, _ = srv.serve(tx, total)
        want = bytes(out[:int(rtotal.item())].cpu().numpy().tobytes())
        q.put((rank, oks, _mask_zxid(got) == _mask_zxid(want), len(got),
               pipe.stats))
    finally:
        dist.destroy_process_group()


def _run_world(world, streams):
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q, streams))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    assert all(p.exitcode == 0 for p in procs)
    res = {}
    for _ in range(world):
        r = q.get(timeout=5)
        res[r[0]] = r[1:]
    n = 3000
    for rank, (oks, same, nbytes, st) in res.items():
        assert oks == [n] * 3, (rank, oks)
        assert same and nbytes > (n // streams) * 100, rank
        assert st['overflow_segments'] == 0
        # most reads are remote: bytes really moved between the ranks
        assert st['remote_reqs'] > 3 * n * (world - 1) / world * 0.8
        assert st['bytes_sent'] > 0 and st['bytes_recv'] > 0
        assert st['wire_bytes_sent'] >= st['bytes_sent']


@pytest.mark.parametrize('world,streams', [(2, 1), (3, 2)])
def test_sharded_get_multi_rank_gloo(gpu, world, streams):
    _run_world(world, streams)


def test_sharded_get_eight_ranks_gloo(gpu):
    """The 8-rank rehearsal: eight ranks share the one GPU (gloo
    collectives), two pipelined connections each."""
    _run_world(8, 2)


@pytest.mark.parametrize('streams', [1, 2])
def test_sharded_forced_route_rccl_captured(gpu, streams):
    """The multi-rank sharded step on one GPU over a one-rank RCCL group
    (route -> seg_pack -> all_to_all_single on HBM tensors -> seg_unpack,
    K1 / K12 / K13 / K1 / K2-K4 around it), captured with its collectives
    as one HIP graph and replayed: every reply checks out on the device."""
    import torch.distributed as dist
    from zkmi.bench.synthetic import GpuTree
    from zkmi.parallel.sharded import ShardedGetPipeline
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group('nccl', device_id=gpu, rank=0, world_size=1,
                            init_method='tcp://127.0.0.1:%d' % port)
    g = pipe = None
    try:
        assert dist.get_backend() == 'nccl'
        tree = GpuTree(20000, 100, fanout=100, device=gpu, seed=0,
                       shard=(0, 1))
        n = 8192
        pipe = ShardedGetPipeline(tree, n, seed=3, streams=streams,
                                  force_route=True)
        assert pipe.route and pipe.capturable
        acc = torch.zeros(64, dtype=torch.int64, device=gpu)
        for _ in range(2):
            pipe.step(acc=acc)
        torch.cuda.synchronize()
        assert int(acc.sum().item()) == 2 * n
        g = pipe.capture(acc)
        torch.cuda.synchronize()
        acc.zero_()
        torch.cuda.synchronize()
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        assert int(acc.sum().item()) == 3 * n
        st = pipe.stats
        assert st['overflow_segments'] == 0
        assert st['xgmi_lower_bound_ms'] == 0.0
    finally:
        # the graph holds the communicator's captured work: release it
        # before the group goes (destroying the group under a live graph
        # waits forever in the communicator's shutdown)
        g = pipe = None
        import gc
        gc.collect()
        torch.cuda.synchronize()
        dist.destroy_process_group()
