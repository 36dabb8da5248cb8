"""Numerics of the HIP batch codec (K1-K13) against the pure-Python Jute
oracle (zkmi/jute.py), which itself is pinned to the reference's golden
vectors in test_proto.py.  All tests here need an MI355X."""

import os

import numpy as np
import pytest
import torch

from zkmi import consts, jute
from zkmi.utils import synth

pytestmark = pytest.mark.gpu


def _dev_bytes(b, dev):
    a = np.frombuffer(bytes(b) if b else b'\0', np.uint8).copy()
    return torch.from_numpy(a).to(dev)


def _norm(pkt):
    out = dict(pkt)
    for k in ('stat',):
        if k in out and out[k] is not None:
            out[k] = out[k].as_tuple()
    return out


def test_encode_requests_matches_oracle(gpu):
    from zkmi.ops import batch as B
    r = synth.rng(1)
    pkts = [synth.rand_request(r, xid) for xid in range(2000)]
    rb = B.pack_requests(pkts, gpu)
    xt = B.XidTable(bits=12, device=gpu)
    out, rec_off, total, err = B.encode_requests(rb, xt)
    torch.cuda.synchronize()
    assert err.item() == 0
    want = b''.join(jute.frame(jute.encode_request(p)) for p in pkts)
    got = bytes(out[:total.item()].cpu().numpy().tobytes())
    assert got == want
    # xid table records the opcode of every request
    tab = xt.tab.cpu().tolist()
    for p in pkts[-100:]:
        e = tab[p['xid'] & xt.mask]
        assert (e >> 32) == p['xid']
        assert (e & 0xffffffff) - (1 << 32 if e & 0x80000000 else 0) == \
            consts.OP_CODES[p['opcode']]


def test_encode_set_watches_matches_oracle(gpu):
    from zkmi.ops import batch as B
    ev = {'dataChanged': ['/d', '/d2/x'], 'createdOrDestroyed': ['/e'],
          'childrenChanged': ['/c', '/', '/zz']}
    got = B.encode_set_watches(0x517, ev['dataChanged'],
                               ev['createdOrDestroyed'],
                               ev['childrenChanged'], gpu)
    want = jute.frame(jute.encode_request(
        {'xid': -8, 'opcode': 'SET_WATCHES', 'relZxid': 0x517,
         'events': ev}))
    assert bytes(got.cpu().numpy().tobytes()) == want
    got0 = B.encode_set_watches(5, [], [], [], gpu)
    want0 = jute.frame(jute.encode_request(
        {'xid': -8, 'opcode': 'SET_WATCHES', 'relZxid': 5,
         'events': {}}))
    assert bytes(got0.cpu().numpy().tobytes()) == want0


def test_encode_requests_error_word(gpu):
    """K10's err is written whole by the encode (no zero fill before it):
    0 clean, 1 an unknown opcode, 2 over capacity — and a clean encode
    after a failed one reads 0 again from a reused buffer."""
    from zkmi.ops import batch as B
    pk = [{'xid': i, 'opcode': 'GET_DATA', 'path': '/a/%d' % i,
           'watch': False} for i in range(3000)]
    rb = B.pack_requests(pk, gpu)
    _, _, total, err = B.encode_requests(rb)
    assert int(err.item()) == 0
    small = torch.empty(64, dtype=torch.uint8, device=gpu)
    _, _, total, err = B.encode_requests(rb, out=small)
    assert int(err.item()) & 2
    rb.opcode[1000] = 12345                      # no such opcode
    _, _, total, err = B.encode_requests(rb)
    assert int(err.item()) == 1
    rb.opcode[1000] = 4
    _, _, total, err = B.encode_requests(rb)
    assert int(err.item()) == 0


def _frames_stream(r, n, maxbody):
    parts = []
    for _ in range(n):
        k = r.choice([0, 1, 16, r.randint(0, maxbody)])
        parts.append(jute.frame(bytes(r.getrandbits(8) for _ in range(k))))
    return b''.join(parts)


# K1 entry windows: frames longer than the window take the slow path and
# must stay exact (the 600 / 5000 / 40000-byte cases at window 256), also
# in long-frame mode (bit 16: zkmi.ops.batch.FS_WIN_LONG)
WINDOWS = [256, 1024, 2048, 256 | 1 << 16, 1024 | 1 << 16]


@pytest.mark.parametrize('window', WINDOWS)
@pytest.mark.parametrize('maxbody,n', [(64, 3000), (600, 800), (5000, 120),
                                       (40000, 12)])
def test_frame_scan_matches_oracle(gpu, maxbody, n, window):
    from zkmi.ops import batch as B
    r = synth.rng(maxbody)
    s = _frames_stream(r, n, maxbody)
    # add a partial trailing frame (carry)
    tail = jute.frame(b'x' * 50)[:-7]
    s = s + tail
    frames, consumed, bad = jute.scan_frames(s)
    buf = _dev_bytes(s, gpu)
    ft = B.frame_scan(buf, len(s), window=window)
    res = ft.host_result()
    assert res['frames'] == len(frames)
    assert res['consumed'] == consumed == len(s) - len(tail)
    assert not res['bad']
    off = ft.off[:len(frames)].cpu().tolist()
    ln = ft.length[:len(frames)].cpu().tolist()
    assert list(zip(off, ln)) == frames


@pytest.mark.parametrize('window', WINDOWS)
def test_frame_scan_bad_length_exact(gpu, window):
    from zkmi.ops import batch as B
    r = synth.rng(7)
    good = _frames_stream(r, 500, 300)
    bad = b'\xff\xff\xff\xfe\x01\x02'
    s = good + bad + _frames_stream(r, 50, 30)
    frames, consumed, bad_at = jute.scan_frames(s)
    assert bad_at == len(good)
    ft = B.frame_scan(_dev_bytes(s, gpu), len(s), window=window)
    res = ft.host_result()
    assert res['bad'] and res['consumed'] == len(good)
    assert res['frames'] == len(frames)
    # too-large length
    s2 = good + b'\x7f\x00\x00\x00' + b'\0' * 100
    ft2 = B.frame_scan(_dev_bytes(s2, gpu), len(s2), window=window)
    res2 = ft2.host_result()
    assert res2['bad'] and res2['consumed'] == len(good)


@pytest.mark.parametrize('window', [256, 2048])
def test_terminated_stream_scans_over_a_bound(gpu, window):
    """K10 terminate=True + K1 over a host upper bound (stale bytes after
    the terminator) frames exactly the encoded stream: the sync-free
    pipeline contract."""
    from zkmi.ops import batch as B
    r = synth.rng(11)
    pkts = [{'xid': i, 'opcode': 'GET_DATA', 'watch': bool(i & 1),
             'path': '/p/%d' % r.randint(0, 10 ** r.randint(1, 9))}
            for i in range(5000)]
    rb = B.pack_requests(pkts, gpu)
    cap = 64 * len(pkts) + (1 << 16)
    out = torch.randint(0, 256, (cap,), dtype=torch.uint8, device=gpu)
    tx, _, total, err = B.encode_requests(rb, out=out, terminate=True)
    ft = B.frame_scan(tx, cap, window=window)
    res = ft.host_result()
    want = b''.join(jute.frame(jute.encode_request(p)) for p in pkts)
    assert int(total.item()) == len(want) and int(err.item()) == 0
    assert bytes(tx[:len(want)].cpu().numpy().tobytes()) == want
    assert res['frames'] == len(pkts)
    assert res['consumed'] == len(want) and res['bad']
    frames, _, _ = jute.scan_frames(want)
    got = list(zip(ft.off[:len(pkts)].cpu().tolist(),
                   ft.length[:len(pkts)].cpu().tolist()))
    assert got == frames


@pytest.mark.parametrize('window', [256, 1024])
@pytest.mark.parametrize('maxbody,n', [(64, 4000), (300, 2000), (5000, 150),
                                       (40000, 12)])
def test_frame_scan_device_length_garbage_tail(gpu, window, maxbody, n):
    """K1 over a DEVICE length (an encoder's total): the buffer's capacity
    is 4x the stream and the tail past the length is random garbage, which
    must neither be walked into frames nor change the result."""
    from zkmi.ops import batch as B
    r = synth.rng(maxbody + window)
    s = _frames_stream(r, n, maxbody)
    tail = jute.frame(b'y' * 40)[:-5]          # partial frame: carry
    s = s + tail
    frames, consumed, bad = jute.scan_frames(s)
    cap = 4 * len(s) + 16384
    buf = torch.randint(0, 256, (cap,), dtype=torch.uint8, device=gpu)
    buf[:len(s)] = _dev_bytes(s, gpu)
    n_dev = torch.tensor([len(s)], dtype=torch.int64, device=gpu)
    sc = B.FrameScanner(len(frames) + 8, gpu, window=window)
    for _ in range(2):                 # a reused scanner: words re-zeroed
        ft = sc.scan(buf, n_dev)
        res = ft.host_result()
        assert res['frames'] == len(frames)
        assert res['consumed'] == consumed == len(s) - len(tail)
        assert not res['bad'] and not res['overflow']
        got = list(zip(ft.off[:len(frames)].cpu().tolist(),
                       ft.length[:len(frames)].cpu().tolist()))
        assert got == frames
    # the same scanner over a shorter device length (a cut stream)
    cut = frames[len(frames) // 2][0] - 4 + 2
    n_dev.fill_(cut)
    res = sc.scan(buf, n_dev).host_result()
    want, wc, _ = jute.scan_frames(s[:cut])
    assert res['frames'] == len(want) and res['consumed'] == wc


@pytest.mark.parametrize('window', [256, 1024])
def test_frame_scanner_clean_reuse_many_streams(gpu, window):
    """A FrameScanner reused over one capacity skips the workspace memset
    (the previous scan cleared its flags): many different streams in a row
    — short and long frames (repairs), BAD_LENGTH, carries, cut lengths —
    must each match the oracle exactly."""
    from zkmi.ops import batch as B
    r = synth.rng(4242 + window)
    cap = 1 << 20
    sc = B.FrameScanner(cap // 4, gpu, window=window)
    buf = torch.randint(0, 256, (cap,), dtype=torch.uint8, device=gpu)
    n_dev = torch.zeros(1, dtype=torch.int64, device=gpu)
    for it in range(12):
        maxbody = r.choice([16, 200, 900, 6000, 30000])
        s = _frames_stream(r, r.randint(1, 4000 if maxbody < 1000 else 40),
                           maxbody)
        if it % 3 == 1:
            s += b'\xff\xff\xff\xf0' + b'junk'        # BAD_LENGTH
        elif it % 3 == 2:
            s += jute.frame(b'z' * 70)[:-9]             # carry
        s = s[:cap]
        buf[:len(s)] = _dev_bytes(s, gpu)
        n = len(s) if it % 4 else max(len(s) - r.randint(1, 64), 0)
        n_dev.fill_(n)
        ft = sc.scan(buf, n_dev)
        res = ft.host_result()
        frames, consumed, bad_at = jute.scan_frames(s[:n])
        assert res['frames'] == len(frames), it
        assert res['consumed'] == consumed, it
        assert bool(res['bad']) == (bad_at >= 0), it
        got = list(zip(ft.off[:len(frames)].cpu().tolist(),
                       ft.length[:len(frames)].cpu().tolist()))
        assert got == frames, it


def test_frame_scan_device_length_bad_frame(gpu):
    from zkmi.ops import batch as B
    r = synth.rng(77)
    good = _frames_stream(r, 3000, 200)
    s = good + b'\x80\x00\x00\x01' + _frames_stream(r, 300, 200)
    cap = 2 * len(s)
    buf = torch.randint(0, 256, (cap,), dtype=torch.uint8, device=gpu)
    buf[:len(s)] = _dev_bytes(s, gpu)
    n_dev = torch.tensor([len(s)], dtype=torch.int64, device=gpu)
    ft = B.frame_scan(buf, n_dev, window=256)
    res = ft.host_result()
    frames, consumed, bad_at = jute.scan_frames(s)
    assert res['bad'] and res['consumed'] == len(good) == bad_at
    assert res['frames'] == len(frames)
    # zero length: nothing framed
    n_dev.zero_()
    res = B.frame_scan(buf, n_dev).host_result()
    assert res == {'frames': 0, 'consumed': 0, 'bad': False,
                   'overflow': False}


def test_frame_scan_encoder_total_no_sync(gpu):
    """encode_requests' device total feeds K1 directly: the sync-free
    pipeline contract without a terminator or a host bound."""
    from zkmi.ops import batch as B
    r = synth.rng(12)
    pkts = [{'xid': i, 'opcode': 'GET_DATA', 'watch': bool(i & 1),
             'path': '/p/%d' % r.randint(0, 10 ** r.randint(1, 9))}
            for i in range(20000)]
    rb = B.pack_requests(pkts, gpu)
    cap = 64 * len(pkts) + (1 << 16)
    out = torch.randint(0, 256, (cap,), dtype=torch.uint8, device=gpu)
    tx, _, total, err = B.encode_requests(rb, out=out)
    ft = B.frame_scan(tx, total, window=256)
    res = ft.host_result()
    want = b''.join(jute.frame(jute.encode_request(p)) for p in pkts)
    assert res['frames'] == len(pkts) and res['consumed'] == len(want)
    assert not res['bad']
    frames, _, _ = jute.scan_frames(want)
    got = list(zip(ft.off[:len(pkts)].cpu().tolist(),
                   ft.length[:len(pkts)].cpu().tolist()))
    assert got == frames


@pytest.mark.parametrize('window', [256, 2048])
def test_frame_scan_large_multi_level(gpu, window):
    """> 256 tiles forces the hierarchical composition path."""
    from zkmi.ops import batch as B
    r = synth.rng(3)
    bodies = [bytes([i & 0xff]) * r.randint(16, 400) for i in range(40000)]
    s = b''.join(jute.frame(b) for b in bodies)
    assert len(s) > 256 * 16384
    ft = B.frame_scan(_dev_bytes(s, gpu), len(s), window=window)
    res = ft.host_result()
    assert res['frames'] == len(bodies)
    assert res['consumed'] == len(s)
    ln = ft.length[:len(bodies)].cpu().numpy()
    assert (ln == np.array([len(b) for b in bodies])).all()


def test_decode_replies_matches_oracle(gpu):
    from zkmi.ops import batch as B
    r = synth.rng(11)
    reps = []
    xid_map = {}
    for xid in range(3000):
        if r.random() < 0.1:
            reps.append(synth.rand_notification(r))
            continue
        rep = synth.rand_reply(r, xid)
        xid_map[xid] = rep['opcode']
        reps.append(rep)
    reps.append({'xid': -2, 'zxid': 77, 'err': 'OK', 'opcode': 'PING'})
    s = b''.join(jute.frame(jute.encode_response(p)) for p in reps)
    want = [jute.decode_response(jute.encode_response(p), xid_map)
            for p in reps]
    buf = _dev_bytes(s, gpu)
    xt = B.XidTable(bits=12, device=gpu)
    # populate the xid table the way the encoder would
    tab = xt.tab.cpu()
    for xid, op in xid_map.items():
        tab[xid & xt.mask] = (xid << 32) | (consts.OP_CODES[op] & 0xffffffff)
    xt.tab.copy_(tab)
    ft = B.frame_scan(buf, len(s))
    rep = B.decode_replies(buf, ft, xt)
    got = B.replies_to_packets(buf, rep)
    assert len(got) == len(want)
    for g, w in zip(got, want):
        assert _norm(g) == _norm(w)


def test_expand_children_and_acl(gpu):
    from zkmi.ops import batch as B
    r = synth.rng(5)
    reps = []
    xid_map = {}
    for xid in range(500):
        op = 'GET_CHILDREN2' if xid % 2 else 'GET_ACL'
        rep = {'xid': xid, 'zxid': 1, 'err': 'OK', 'opcode': op,
               'stat': synth.rand_stat(r)}
        if op == 'GET_CHILDREN2':
            rep['children'] = ['c%d' % k for k in range(xid % 7)]
        else:
            rep['acl'] = synth.rand_acl(r)
            for a in rep['acl']:
                a['perms'] = [p.upper() for p in a['perms']]
        xid_map[xid] = op
        reps.append(rep)
    s = b''.join(jute.frame(jute.encode_response(p)) for p in reps)
    buf = _dev_bytes(s, gpu)
    xt = B.XidTable(bits=10, device=gpu)
    tab = xt.tab.cpu()
    for xid, op in xid_map.items():
        tab[xid] = (xid << 32) | consts.OP_CODES[op]
    xt.tab.copy_(tab)
    ft = B.frame_scan(buf, len(s))
    rb = B.decode_replies(buf, ft, xt)
    n = len(reps)
    ch = torch.where(rb.opcode[:n] == 12, rb.aux0[:n],
                     torch.zeros_like(rb.aux0[:n]))
    base, soff, slen = B.expand_strings(buf, rb.pay_off[:n], ch)
    hb = s
    so, sl, bs = soff.cpu().tolist(), slen.cpu().tolist(), \
        base.cpu().tolist()
    for i, rep in enumerate(reps):
        if rep['opcode'] == 'GET_CHILDREN2':
            kids = [hb[so[bs[i] + k]:so[bs[i] + k] + sl[bs[i] + k]].decode()
                    for k in range(len(rep['children']))]
            assert kids == rep['children']
    ac = torch.where(rb.opcode[:n] == 6, rb.aux0[:n],
                     torch.zeros_like(rb.aux0[:n]))
    base, perms, s_o, s_l, i_o, i_l = B.expand_acl(buf, rb.pay_off[:n], ac)
    pm, so, sl, io, il, bs = (x.cpu().tolist() for x in
                              (perms, s_o, s_l, i_o, i_l, base))
    for i, rep in enumerate(reps):
        if rep['opcode'] == 'GET_ACL':
            for k, a in enumerate(rep['acl']):
                j = bs[i] + k
                assert pm[j] == jute.perms_to_mask(a['perms'])
                assert hb[so[j]:so[j] + sl[j]].decode() == a['id']['scheme']
                assert hb[io[j]:io[j] + il[j]].decode() == a['id']['id']


def test_decode_requests_matches_oracle(gpu):
    from zkmi.ops import batch as B
    r = synth.rng(13)
    pkts = [synth.rand_request(r, xid) for xid in range(2000)]
    s = b''.join(jute.frame(jute.encode_request(p)) for p in pkts)
    buf = _dev_bytes(s, gpu)
    ft = B.frame_scan(buf, len(s))
    rt = B.decode_requests(buf, ft)
    n = len(pkts)
    cols = {k: getattr(rt, k)[:n].cpu().tolist() for k in (
        'xid', 'opcode', 'status', 'path_off', 'path_len', 'data_off',
        'data_len', 'arg', 'vec_count')}
    for i, p in enumerate(pkts):
        w = jute.decode_request(jute.encode_request(p))
        assert cols['status'][i] == 0
        assert cols['xid'][i] == w['xid']
        assert cols['opcode'][i] == consts.OP_CODES[w['opcode']]
        if 'path' in w:
            po, pl = cols['path_off'][i], cols['path_len'][i]
            assert s[po:po + pl].decode() == w['path']
        if 'data' in w:
            do, dl = cols['data_off'][i], cols['data_len'][i]
            assert s[do:do + dl] == w['data']
        if 'watch' in w:
            assert cols['arg'][i] == int(w['watch'])
        if 'version' in w:
            assert cols['arg'][i] == w['version']
        if w['opcode'] == 'CREATE':
            assert cols['arg'][i] == jute.flags_to_mask(w['flags'])
            assert cols['vec_count'][i] == len(w['acl'])


def _small_tree(gpu, n=5000, data=100, spare=0.25):
    from zkmi.bench.synthetic import GpuTree
    return GpuTree(n, data, fanout=100, device=gpu, spare=spare)


def test_encode_responses_matches_oracle(gpu):
    """K13 (LDS-staged writer) against jute.encode_response."""
    from zkmi.ops import batch as B
    tree = _small_tree(gpu)
    r = synth.rng(21)
    n = 3000
    ops, errs, nodes, zx, paths = [], [], [], [], []
    for i in range(n):
        op = r.choice(['GET_DATA', 'EXISTS', 'SET_DATA', 'CREATE', 'DELETE',
                       'NOTIFICATION'])
        ops.append(op)
        errs.append(0 if r.random() < 0.8 else -101)
        nodes.append(r.randrange(tree.leaf0, tree.n_static))
        zx.append(r.randint(0, 2**40))
        paths.append(synth.rand_path(r))
    parena = b''.join(p.encode() for p in paths)
    poff = np.cumsum([0] + [len(p.encode()) for p in paths[:-1]])
    T = lambda a, dt: torch.tensor(a, dtype=dt, device=gpu)  # noqa: E731
    resp = B.ResponseBatch(
        T([consts.OP_CODES[o] for o in ops], torch.int32),
        T(list(range(n)), torch.int32), T(errs, torch.int32),
        T(nodes, torch.int64), T(zx, torch.int64),
        T(poff.tolist(), torch.int64),
        T([len(p.encode()) for p in paths], torch.int32),
        _dev_bytes(parena, gpu),
        T([r.choice([1, 2, 3, 4]) for _ in range(n)], torch.int32),
        T([n], torch.int64))
    out, rec_off, total, err = B.encode_responses(resp, tree.store, 1 << 22)
    torch.cuda.synchronize()
    assert err.item() == 0
    got = bytes(out[:total.item()].cpu().numpy().tobytes())
    slots = {}
    want = []
    for i in range(n):
        nd = nodes[i]
        if nd not in slots:
            slots[nd] = tree.node_slot_host(nd)
        data, st = slots[nd]
        assert st.czxid == nd + 1 and st.dataLength == len(data) == 100
        rep = {'xid': i, 'zxid': zx[i], 'err': errs[i], 'opcode': ops[i],
               'stat': st, 'path': paths[i], 'data': data,
               'type': int(resp.aux[i].item()), 'state': 'SYNC_CONNECTED'}
        want.append(jute.frame(jute.encode_response(rep)))
    assert got == b''.join(want)


@pytest.mark.parametrize('dist,mix', [(None, False), ((0, 300), False),
                                      ((0, 300), True), ((0, 2000), False),
                                      ((0, 2000), True), ((300, 1024), False)])
def test_encode_responses_serve_mix_matches_oracle(gpu, dist, mix):
    """K13 on the serve path's usual replies (GET_DATA / Stat / header-only,
    errors among them) against jute.encode_response: fixed and variable
    data lengths, a terminated stream (four 0xFF bytes right after it,
    nothing written past the last 16-byte chunk), and with ``mix`` a CREATE
    in every third block.  Payloads past ~300 bytes exercise the holes (the
    16-byte aligned interiors the waves copy slot -> out, the image streamed
    out segment by segment between them).  Round 3 measured a gather variant
    of the writer
    (each aligned 16-byte chunk built from its record's slot) 2.4x slower
    than the LDS-staged one (README, Measured and rejected)."""
    from zkmi.bench.synthetic import GpuTree
    from zkmi.ops import batch as B
    tree = GpuTree(5000, 100, fanout=100, device=gpu, spare=0.25,
                   data_dist=dist)
    r = synth.rng(22)
    n = 256 * 9 + 77
    ops, errs, nodes, zx, paths = [], [], [], [], []
    for i in range(n):
        op = r.choice(['GET_DATA', 'GET_DATA', 'GET_DATA', 'EXISTS',
                       'SET_DATA', 'DELETE'])
        if mix and (i // 256) % 3 == 1 and i % 256 == 100:
            op = 'CREATE'
        ops.append(op)
        errs.append(0 if r.random() < 0.85 else -101)
        nodes.append(r.randrange(tree.leaf0, tree.n_static))
        zx.append(r.randint(0, 2**40))
        paths.append(synth.rand_path(r))
    parena = b''.join(p.encode() for p in paths)
    poff = np.cumsum([0] + [len(p.encode()) for p in paths[:-1]])
    T = lambda a, dt: torch.tensor(a, dtype=dt, device=gpu)  # noqa: E731
    resp = B.ResponseBatch(
        T([consts.OP_CODES[o] for o in ops], torch.int32),
        T(list(range(n)), torch.int32), T(errs, torch.int32),
        T(nodes, torch.int64), T(zx, torch.int64),
        T(poff.tolist(), torch.int64),
        T([len(p.encode()) for p in paths], torch.int32),
        _dev_bytes(parena, gpu), T([1] * n, torch.int32), T([n], torch.int64))
    slots = {}
    want = []
    for i in range(n):
        nd = nodes[i]
        if nd not in slots:
            slots[nd] = tree.node_slot_host(nd)
        data, st = slots[nd]
        rep = {'xid': i, 'zxid': zx[i], 'err': errs[i], 'opcode': ops[i],
               'stat': st, 'path': paths[i], 'data': data}
        want.append(jute.frame(jute.encode_response(rep)))
    want = b''.join(want)
    cap = 1 << 22
    out = torch.full((cap,), 0xAB, dtype=torch.uint8, device=gpu)
    out, rec_off, total, err = B.encode_responses(resp, tree.store, cap,
                                                  out=out, terminate=True)
    torch.cuda.synchronize()
    assert err.item() == 0
    t = int(total.item())
    assert t == len(want)
    hb = bytes(out[:t + 64].cpu().numpy().tobytes())
    assert hb[:t] == want
    assert hb[t:t + 4] == b'\xff' * 4
    end = (t + 4 + 15) & ~15
    assert hb[end:] == b'\xab' * (t + 64 - end)
    # record offsets: where each frame starts
    starts, o = [], 0
    while o < t:
        starts.append(o)
        o += 4 + int.from_bytes(want[o:o + 4], 'big')
    assert rec_off[:n].cpu().tolist() == starts


def test_encode_responses_get_blocks_matches_oracle(gpu):
    """K13 on blocks of equal-size successful GET_DATA replies (the GET
    workload's reply stream: the blocks the uniform writer takes), a ragged
    last block and one block with an error reply in it (the LDS image's),
    against jute.encode_response."""
    from zkmi.ops import batch as B
    tree = _small_tree(gpu)
    r = synth.rng(23)
    n = 256 * 5 + 33
    nodes = [r.randrange(tree.leaf0, tree.n_static) for _ in range(n)]
    zx = [r.randint(0, 2**40) for _ in range(n)]
    errs = [0] * n
    errs[256 * 2 + 17] = -101
    T = lambda a, dt: torch.tensor(a, dtype=dt, device=gpu)  # noqa: E731
    resp = B.ResponseBatch(
        T([consts.OP_CODES['GET_DATA']] * n, torch.int32),
        T(list(range(n)), torch.int32), T(errs, torch.int32),
        T(nodes, torch.int64), T(zx, torch.int64),
        T([0] * n, torch.int64), T([0] * n, torch.int32),
        _dev_bytes(b'\0' * 16, gpu), T([1] * n, torch.int32),
        T([n], torch.int64))
    out, rec_off, total, err = B.encode_responses(resp, tree.store, 1 << 22)
    torch.cuda.synchronize()
    assert err.item() == 0
    got = bytes(out[:total.item()].cpu().numpy().tobytes())
    want = []
    for i in range(n):
        data, st = tree.node_slot_host(nodes[i])
        want.append(jute.frame(jute.encode_response(
            {'xid': i, 'zxid': zx[i], 'err': errs[i], 'opcode': 'GET_DATA',
             'stat': st, 'data': data})))
    assert got == b''.join(want)


def test_encode_responses_get_blocks_lds_image(gpu):
    """The same blocks through the LDS image writer instead of the uniform
    one (ZKMI_ENC_UNIFORM=0 is read once per process: a child process)."""
    import subprocess
    import sys
    env = dict(os.environ, ZKMI_ENC_UNIFORM='0')
    res = subprocess.run(
        [sys.executable, '-m', 'pytest', '-q', '-x', '-p', 'no:cacheprovider',
         os.path.abspath(__file__) +
         '::test_encode_responses_get_blocks_matches_oracle'],
        env=env, capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stdout[-3000:] + res.stderr[-2000:]


def test_gpu_get_pipeline_end_to_end(gpu):
    from zkmi.bench.synthetic import GetPipeline
    tree = _small_tree(gpu, 20000, 37)
    pipe = GetPipeline(tree, 8192)
    for _ in range(3):
        ok = pipe.step()
        assert int(ok.item()) == 8192
    idx, rep, rx, ft = pipe.last
    # data bytes returned equal the node's data
    n = 64
    po = rep.pay_off[:n].cpu().tolist()
    hb = rx.cpu().numpy()
    for k, nd in enumerate(idx[:n].cpu().tolist()):
        data, st = tree.node_slot_host(nd)
        assert bytes(hb[po[k]:po[k] + 37].tobytes()) == data


def test_gpu_presized_request_encode_matches(gpu):
    """The GET pipeline's request encode takes its sizes and block sums from
    the generator (bench_gen_get) instead of its own sizes pass: the stream,
    the record offsets and the total must be the general encode's, byte for
    byte, for a batch that is not a multiple of the 256-request block."""
    from zkmi.bench.synthetic import GetPipeline
    from zkmi.ops import batch as B
    from zkmi.ops import _lib
    tree = _small_tree(gpu, 20000, 37)
    n = 5000
    pipe = GetPipeline(tree, n)
    pipe.step()
    t = tree
    L = _lib.lib()
    sizes = torch.empty(n, dtype=torch.int64, device=gpu)
    bsum = torch.empty((n + 255) // 256, dtype=torch.int64, device=gpu)
    L.bench_gen_get(n, 77, t.leaf0, t.n_leaves, 5, t.node_pw, pipe.idx,
                    pipe.xid, pipe.poff, pipe.plen, None, sizes, bsum)
    rb = B.RequestBatch(n, pipe.opcode, pipe.xid, pipe.arg, pipe.poff,
                        pipe.plen, pipe.zero64, pipe.zero32, pipe.zero32,
                        t.path_arena, t.slab, pipe.acl_off, pipe.acl_len,
                        pipe.acl_arena)
    out_a, off_a, tot_a, err_a = B.encode_requests(rb)
    out_b, off_b, tot_b, err_b = B.encode_requests(rb, presized=(sizes, bsum))
    ta, tb = int(tot_a.item()), int(tot_b.item())
    assert ta == tb and int(err_a.item()) == int(err_b.item()) == 0
    assert torch.equal(off_a, off_b)
    assert torch.equal(out_a[:ta], out_b[:tb])
    assert int(bsum.sum().item()) == ta


def test_gpu_get_check_samples_payload_bytes(gpu):
    """The fused GET check compares the payload bytes of one reply in 16
    with its node's slot: a reply stream whose every payload has one byte
    flipped keeps its lengths, and fails exactly the sampled replies."""
    from zkmi.bench.synthetic import GetPipeline
    from zkmi.ops import batch as B
    tree = _small_tree(gpu, 20000, 37)
    n = 8192
    pipe = GetPipeline(tree, n)
    pipe.step()
    idx, rep, rx, ft = pipe.last

    def check(buf, tick=None):
        acc = torch.zeros(1, dtype=torch.int64, device=gpu)
        B.decode_replies(buf, ft, pipe.xt, check=(idx, pipe.xid,
                                                  tree.data_len, acc,
                                                  tree.slab_all,
                                                  tree.slot_off), tick=tick)
        return int(acc.item())
    assert check(rx) == n
    bad = rx.clone()
    po = rep.pay_off[:n]
    bad[po + 5] ^= 0x5A
    assert check(bad) == n - (n + 15) // 16
    # the sample rotates with the step counter: salt 3 -> i % 16 == 13
    tick = torch.tensor([0, 3], dtype=torch.int64, device=gpu)
    assert check(bad, tick) == n - len(range(13, n, 16))
    # the flipped byte of an unsampled reply goes unnoticed, by design
    one = rx.clone()
    one[po[1] + 5] ^= 0x5A
    assert check(one) == n


def test_gpu_get_pipeline_two_connections(gpu):
    """The bench's default shape: the batch split over two pipelined
    connections (own HIP streams, buffers, xid tables), no host read-back
    inside a step; every reply checked on the device, the accumulator read
    on the caller's stream."""
    from zkmi.bench.synthetic import GetPipeline
    tree = _small_tree(gpu, 20000, 37)
    pipe = GetPipeline(tree, 8193, streams=2)
    acc = torch.zeros(1, dtype=torch.int64, device=gpu)
    for _ in range(3):
        pipe.step(acc=acc)
    assert int(acc.item()) == 3 * 8193
    assert [p.batch for p in pipe.subs] == [4097, 4096]


def test_gpu_get_pipeline_graph_replay(gpu):
    """bench --graph: one step captured as a HIP graph; every replay draws
    a NEW batch (device-resident seed) and checks all its replies."""
    from zkmi.bench.synthetic import GetPipeline
    tree = _small_tree(gpu, 20000, 37)
    pipe = GetPipeline(tree, 8193, streams=2)
    acc = torch.zeros(1, dtype=torch.int64, device=gpu)
    pipe.step(acc=acc)
    acc.zero_()
    g = pipe.capture(acc)
    seen = []
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        seen.append(pipe.subs[0].idx[:64].clone())
    assert int(acc.item()) == 3 * 8193
    assert not torch.equal(seen[0], seen[1])
    assert not torch.equal(seen[1], seen[2])


def test_gpu_get_pipeline_staggered_streams(gpu):
    """bench's default: the second connection runs half a step (2 phases)
    behind the first; each step() issues one step of work per connection
    and the lagging connection's checks land one call later."""
    from zkmi.bench.synthetic import GetPipeline
    tree = _small_tree(gpu, 20000, 37)
    pipe = GetPipeline(tree, 8193, streams=2, stagger=True)
    acc = torch.zeros(1, dtype=torch.int64, device=gpu)
    pipe.step(acc=acc)
    assert int(acc.item()) == 4097              # connection 1 not checked yet
    for _ in range(3):
        pipe.step(acc=acc)
    assert int(acc.item()) == 4 * 4097 + 3 * 4096
    acc.zero_()
    pipe.step(acc=acc)
    assert int(acc.item()) == 8193              # steady state: a full step


def test_gpu_tree_mutations(gpu):
    """SET_DATA version CAS, CREATE (parent must exist, NODE_EXISTS),
    DELETE through the GPU server, checked reply by reply."""
    from zkmi.ops import batch as B
    from zkmi.bench.synthetic import GpuServer
    tree = _small_tree(gpu, 1000, 16)
    leaf = '/bench/d000000/n000000003'
    pk = [
        {'xid': 0, 'opcode': 'SET_DATA', 'path': leaf, 'data': b'new!',
         'version': 0},
        {'xid': 1, 'opcode': 'SET_DATA', 'path': '/bench/d000000/n000000004',
         'data': b'x', 'version': 7},                        # BAD_VERSION
        {'xid': 2, 'opcode': 'CREATE', 'path': '/bench/d000000/new',
         'data': b'hello', 'acl': jute.DEFAULT_ACL, 'flags': []},
        {'xid': 3, 'opcode': 'CREATE', 'path': '/nope/x', 'data': b'',
         'acl': jute.DEFAULT_ACL, 'flags': []},          # NO_NODE
        {'xid': 4, 'opcode': 'CREATE', 'path': leaf, 'data': b'',
         'acl': jute.DEFAULT_ACL, 'flags': []},          # NODE_EXISTS
        {'xid': 5, 'opcode': 'DELETE', 'path': '/bench/d000000/n000000005',
         'version': -1},
        {'xid': 6, 'opcode': 'GET_DATA', 'path': '/bench/d000000/missing',
         'watch': False},                                    # NO_NODE
        {'xid': 7, 'opcode': 'EXISTS', 'path': '/bench', 'watch': False},
        {'xid': 8, 'opcode': 'CREATE', 'path': '/bench/d000000/noacl',
         'data': b'', 'acl': [], 'flags': []},               # INVALID_ACL
    ]
    s = b''.join(jute.frame(jute.encode_request(p)) for p in pk)
    buf = _dev_bytes(s, gpu)
    srv = GpuServer(tree, 64, 1 << 16)
    out, total, err, _ = srv.serve(buf, len(s))
    torch.cuda.synchronize()
    rx = bytes(out[:total.item()].cpu().numpy().tobytes())
    frames, consumed, bad = jute.scan_frames(rx)
    xmap = {p['xid']: p['opcode'] for p in pk}
    reps = [jute.decode_response(rx[o:o + ln], xmap) for o, ln in frames]
    errs = [r['err'] for r in reps]
    assert errs == ['OK', 'BAD_VERSION', 'OK', 'NO_NODE', 'NODE_EXISTS',
                    'OK', 'NO_NODE', 'OK', 'INVALID_ACL']
    assert reps[0]['stat'].version == 1 and reps[0]['stat'].dataLength == 4
    assert reps[2]['path'] == '/bench/d000000/new'
    assert reps[7]['stat'].numChildren == 10
    data, st = tree.node_slot_host(tree.leaf0 + 3)
    assert data == b'new!' and st.version == 1
    # the new node is visible and the deleted one is gone
    pk2 = [{'xid': 10, 'opcode': 'GET_DATA', 'path': '/bench/d000000/new',
            'watch': False},
           {'xid': 11, 'opcode': 'EXISTS', 'path':
            '/bench/d000000/n000000005', 'watch': False},
           {'xid': 12, 'opcode': 'EXISTS', 'path': '/bench/d000000',
            'watch': False}]
    s2 = b''.join(jute.frame(jute.encode_request(p)) for p in pk2)
    out, total, err, _ = srv.serve(_dev_bytes(s2, gpu), len(s2))
    rx = bytes(out[:total.item()].cpu().numpy().tobytes())
    frames, _, _ = jute.scan_frames(rx)
    xmap = {p['xid']: p['opcode'] for p in pk2}
    reps = [jute.decode_response(rx[o:o + ln], xmap) for o, ln in frames]
    assert reps[0]['err'] == 'OK' and reps[0]['data'] == b'hello'
    assert reps[1]['err'] == 'NO_NODE'
    # d000000 had 100 children (fanout 100); +1 create -1 delete
    assert reps[2]['stat'].numChildren == 100
    assert reps[2]['stat'].cversion == 102


def test_handshake_records_k9(gpu):
    from zkmi.ops import batch as B
    r = synth.rng(31)
    reqs = [{'protocolVersion': 0, 'lastZxidSeen': r.randint(0, 2**40),
             'timeOut': r.randint(1000, 40000),
             'sessionId': r.randint(0, 2**62),
             'passwd': bytes(r.getrandbits(8) for _ in range(
                 r.choice([8, 16])))} for _ in range(300)]
    got = B.encode_connect_requests(reqs, gpu)
    want = b''.join(jute.frame(jute.encode_connect_request(q)) for q in reqs)
    assert bytes(got.cpu().numpy().tobytes()) == want
    resps = [{'protocolVersion': 0, 'timeOut': q['timeOut'],
              'sessionId': q['sessionId'], 'passwd': q['passwd']}
             for q in reqs]
    s = b''.join(jute.frame(jute.encode_connect_response(
        p, read_only=(i % 2 == 0))) for i, p in enumerate(resps))
    buf = _dev_bytes(s, gpu)
    ft = B.frame_scan(buf, len(s))
    o = B.decode_connect_responses(buf, ft, len(resps))
    sid = o['sessionId'].cpu().tolist()
    po, pl = o['passwd_off'].cpu().tolist(), o['passwd_len'].cpu().tolist()
    assert o['status'].cpu().tolist() == [0] * len(resps)
    for i, p in enumerate(resps):
        assert sid[i] == p['sessionId']
        assert s[po[i]:po[i] + pl[i]] == p['passwd']


def test_gpu_free_ring_recycles_nodes(gpu):
    """DELETE pushes the node on the free ring, the NEXT batch's CREATE pops
    it (same batch never does) and reuses its slot and path storage."""
    from zkmi.bench.synthetic import GpuServer
    from zkmi.ops import _lib
    tree = _small_tree(gpu, 1000, 16)
    srv = GpuServer(tree, 64, 1 << 16)
    leaf = '/bench/d000000/n000000007'
    v = tree.find_host(leaf)
    hw = int(tree.counters[_lib.TC_NODES].item())

    def serve(pk):
        s = b''.join(jute.frame(jute.encode_request(p)) for p in pk)
        out, total, _, _ = srv.serve(_dev_bytes(s, gpu), len(s))
        rx = bytes(out[:total.item()].cpu().numpy().tobytes())
        frames, _, _ = jute.scan_frames(rx)
        xmap = {p['xid']: p['opcode'] for p in pk}
        return [jute.decode_response(rx[o:o + ln], xmap) for o, ln in frames]
    reps = serve([{'xid': 1, 'opcode': 'DELETE', 'path': leaf,
                   'version': 0},
                  {'xid': 2, 'opcode': 'DELETE', 'path': leaf,
                   'version': -1}])
    # exactly one of two concurrent deletes of the same node wins
    assert sorted(r['err'] for r in reps) == ['NO_NODE', 'OK']
    assert tree.find_host(leaf) == -1
    reps = serve([{'xid': 3, 'opcode': 'CREATE', 'path':
                   '/bench/d000000/recycled01', 'data': b'r' * 20,
                   'acl': jute.DEFAULT_ACL, 'flags': []}])
    assert reps[0]['err'] == 'OK'
    assert tree.find_host('/bench/d000000/recycled01') == v
    assert int(tree.counters[_lib.TC_NODES].item()) == hw   # no growth
    data, st = tree.node_slot_host(v)
    assert data == b'r' * 20 and st.version == 0


def test_gpu_ephemeral_sequential_and_expire(gpu):
    """SEQUENTIAL appends the parent's cversion as %010d — in stream (xid)
    order: one session's pipelined creates are numbered in the order it
    sent them, as a ZooKeeper leader names them —, EPHEMERAL records the
    session, children of ephemerals are refused, and expiring the session
    removes exactly its ephemerals."""
    from zkmi.bench.synthetic import GpuServer
    tree = _small_tree(gpu, 1000, 16)
    srv = GpuServer(tree, 64, 1 << 16)
    E = ['EPHEMERAL']
    ES = ['EPHEMERAL', 'SEQUENTIAL']

    def serve(pk, session):
        s = b''.join(jute.frame(jute.encode_request(p)) for p in pk)
        out, total, _, _ = srv.serve(_dev_bytes(s, gpu), len(s),
                                     session=session)
        rx = bytes(out[:total.item()].cpu().numpy().tobytes())
        frames, _, _ = jute.scan_frames(rx)
        xmap = {p['xid']: p['opcode'] for p in pk}
        return [jute.decode_response(rx[o:o + ln], xmap) for o, ln in frames]

    def create(x, path, flags):
        return {'xid': x, 'opcode': 'CREATE', 'path': path, 'data': b'e',
                'acl': jute.DEFAULT_ACL, 'flags': flags}
    reps = serve([create(i, '/bench/d000001/q-', ES) for i in range(5)] +
                 [create(9, '/bench/d000001/eph', E)], session=0x1234)
    assert all(r['err'] == 'OK' for r in reps)
    seqs = [r['path'] for r in reps[:5]]          # reply (= xid) order
    # d000001 has 100 children, cversion 100 after the fill
    assert seqs == ['/bench/d000001/q-%010d' % k for k in range(100, 105)]
    reps = serve([create(10, '/bench/d000001/eph/child', [])], session=0x1234)
    assert reps[0]['err'] == 'NO_CHILDREN_FOR_EPHEMERALS'
    reps = serve([create(11, '/bench/d000001/other', E)], session=0x999)
    v = tree.find_host('/bench/d000001/eph')
    assert tree.node_slot_host(v)[1].ephemeralOwner == 0x1234
    removed = tree.expire(0x1234)
    assert int(removed.item()) == 6
    assert tree.find_host('/bench/d000001/eph') == -1
    assert tree.find_host('/bench/d000001/other') >= 0
    reps = serve([{'xid': 12, 'opcode': 'EXISTS', 'path': '/bench/d000001',
                   'watch': False}], session=0)
    assert reps[0]['stat'].numChildren == 101


def _seq_batch(parents, n, xid0=0, flags=('EPHEMERAL', 'SEQUENTIAL')):
    """n SEQUENTIAL creates cycling over `parents` (request k under
    parents[k % len]), in xid order."""
    return [{'xid': xid0 + k, 'opcode': 'CREATE',
             'path': parents[k % len(parents)] + '/s-', 'data': b'%d' % k,
             'acl': jute.DEFAULT_ACL, 'flags': list(flags)} for k in range(n)]


def _serve_decode(srv, pk, gpu, session=0):
    s = b''.join(jute.frame(jute.encode_request(p)) for p in pk)
    out, total, _, _ = srv.serve(_dev_bytes(s, gpu), len(s), session=session)
    rx = bytes(out[:total.item()].cpu().numpy().tobytes())
    frames, _, _ = jute.scan_frames(rx)
    xmap = {p['xid']: p['opcode'] for p in pk}
    return [jute.decode_response(rx[o:o + ln], xmap) for o, ln in frames]


@pytest.mark.parametrize('n,nparents', [(7, 1), (3000, 3), (2500, 700)])
def test_gpu_sequential_names_in_stream_order(gpu, n, nparents):
    """SEQUENTIAL numbers follow the stream: under each parent the batch's
    creates are numbered cversion-before-the-batch + their rank in request
    order — across the 1024-request chunks of the ordering pass (3000 under
    3 parents: 1000 a parent spanning 3 chunks), for many small groups, and
    for one pipelined session.  The parent's cversion moves by the count;
    a second batch continues after it.  (reference test/basic.test.js:
    550-611; a ZooKeeper leader names them in zxid order.)"""
    from zkmi.bench.synthetic import GpuServer
    tree = _small_tree(gpu, 1000 * 10, 16, spare=1.0)
    srv = GpuServer(tree, 4096, 1 << 22)
    parents = ['/bench/d%06d' % (d % 10) for d in range(nparents)]
    if nparents > 10:     # more parents than directories: create them
        parents = ['/bench/d000003/p%04d' % d for d in range(nparents)]
        reps = _serve_decode(srv, [
            {'xid': 100000 + d, 'opcode': 'CREATE', 'path': p, 'data': b'',
             'acl': jute.DEFAULT_ACL, 'flags': []}
            for d, p in enumerate(parents)], gpu)
        assert all(r['err'] == 'OK' for r in reps)
    base, kids0 = {}, {}
    for p in parents:
        st = _serve_decode(srv, [{'xid': 1, 'opcode': 'EXISTS', 'path': p,
                                  'watch': False}], gpu)[0]['stat']
        base[p] = st.cversion
        kids0[p] = st.numChildren
    for rnd in range(2):
        pk = _seq_batch(parents, n, xid0=rnd * n)
        reps = _serve_decode(srv, pk, gpu, session=0x77)
        assert [r['err'] for r in reps] == ['OK'] * n
        rank = {}
        for k, r in enumerate(reps):
            p = parents[k % nparents]
            want = '%s/s-%010d' % (p, base[p] + rank.get(p, 0))
            assert r['path'] == want, (k, r['path'], want)
            rank[p] = rank.get(p, 0) + 1
        for p in set(parents):
            base[p] += rank[p]
    # the parents' Stat: cversion = before + creates, numChildren with it
    p = parents[0]
    st = _serve_decode(srv, [{'xid': 9, 'opcode': 'EXISTS', 'path': p,
                              'watch': False}], gpu)[0]['stat']
    assert st.cversion == base[p]
    assert st.numChildren == kids0[p] + 2 * rank[p]


def test_gpu_sequential_replicas_agree(gpu):
    """Two replicas of one tree serving the same batches come out with the
    same znodes, names, zxids, owners and data (GpuTree.digest), whatever
    order their waves ran in; a failed SEQUENTIAL create leaves a gap (its
    number is not reused), and the next batch numbers after it."""
    from zkmi.bench.synthetic import GpuServer
    trees = [_small_tree(gpu, 4000, 16, spare=2.0) for _ in range(2)]
    srvs = [GpuServer(t, 4096, 1 << 22) for t in trees]
    parents = ['/bench/d%06d' % d for d in range(40)]
    pk = _seq_batch(parents, 4000)
    # request 40 (parents[0]'s second) has no ACL: INVALID_ACL after its
    # number was assigned — a gap under parents[0]
    pk[40]['acl'] = []
    got = []
    for srv, t in zip(srvs, trees):
        r1 = _serve_decode(srv, pk, gpu, session=5)
        r2 = _serve_decode(srv, _seq_batch(parents[:3], 300, xid0=5000),
                           gpu, session=6)
        got.append(([r.get('path') for r in r1 + r2], t.digest()))
    assert got[0][0] == got[1][0]
    assert got[0][1][:2] == got[1][1][:2]
    assert got[0][1][1] == trees[0].n_static + 3999 + 300
    names = got[0][0]
    assert names[40] is None
    assert names[0] == '/bench/d000000/s-%010d' % 100
    assert names[80] == '/bench/d000000/s-%010d' % 102      # the gap
    # the next batch numbers after the whole first one (100 creates a
    # parent: cversion 100 -> 200)
    assert names[4000] == '/bench/d000000/s-%010d' % 200
    # the failed create's child count was taken back: 100 + 99 + 100
    st = _serve_decode(srvs[0], [{'xid': 9999, 'opcode': 'EXISTS',
                                  'path': parents[0], 'watch': False}],
                       gpu)[0]['stat']
    assert st.numChildren == 299 and st.cversion == 300


def test_gpu_expiry_reclaims_tombstones(gpu):
    """Never-reused SEQUENTIAL names do not fill the hash index: session
    expiry empties the entries it tombstones when nothing after them
    continues a probe chain (tree.hip ht_reclaim), and the next batch's
    names take over the tombstones their probes pass (tree_insert<true>),
    so the tombstone count settles instead of growing until a rebuild."""
    from zkmi.bench.synthetic import GpuServer
    tree = _small_tree(gpu, 4000, 16, spare=1.5)
    srv = GpuServer(tree, 4096, 1 << 22)
    parents = ['/bench/d%06d' % d for d in range(40)]
    d0, live0, used0, tomb0 = tree.digest()
    assert tomb0 == 0 and used0 == live0
    tombs = []
    for k in range(40):
        reps = _serve_decode(srv, _seq_batch(parents, 4000, xid0=k * 4000),
                             gpu, session=100 + k)
        assert all(r['err'] == 'OK' for r in reps)
        assert int(tree.expire(100 + k).item()) == 4000
        d, live, used, tomb = tree.digest()
        assert live == live0
        assert used - tomb == live
        tombs.append(tomb)
    print('tombstones per round', tombs, 'of', tree.hcap, 'entries')
    # settled: the last ten rounds no higher than the ten before, and the
    # index (live + tombstones) under half full
    assert max(tombs[30:]) <= max(tombs[20:30]) * 1.15 + 50, tombs
    assert live0 + tombs[-1] < tree.hcap // 2


def test_gpu_mix_pipeline(gpu):
    from zkmi.bench.synthetic import MixPipeline
    from zkmi.ops import _lib
    tree = _small_tree(gpu, 20000, 37, spare=1.0)
    pipe = MixPipeline(tree, 3 * 4096, ndirs=64)
    hw = None
    for s in range(6):
        ok = pipe.step()
        assert int(ok.item()) == 3 * 4096
        if s == 2:
            hw = int(tree.counters[_lib.TC_NODES].item())
    # steady state: recycled nodes, no growth of the node table
    assert int(tree.counters[_lib.TC_NODES].item()) == hw


def test_gpu_bench_check_writes_and_xids(gpu):
    """The write pipelines' fused check counts exactly the clean replies
    (status, err, xid, payload length — per request or one constant) and
    folds the largest zxid into zmax; the fused xids wrap at 2^31."""
    from zkmi.ops import _lib
    L = _lib.lib()
    n = 70000
    g = torch.Generator(device=gpu).manual_seed(5)
    i32 = dict(dtype=torch.int32, device=gpu)
    status = torch.zeros(n, **i32)
    err = torch.zeros(n, **i32)
    xid = torch.arange(n, **i32)
    rxid = xid.clone()
    want = torch.randint(1, 50, (n,), generator=g, device=gpu).to(torch.int32)
    pay = want.clone()
    zx = torch.randint(0, 1 << 40, (n,), generator=g, device=gpu)
    status[3] = 1
    err[700] = -101
    rxid[4096] += 1
    pay[69999] += 1
    ok = torch.zeros(1, dtype=torch.int64, device=gpu)
    zmax = torch.tensor([5], dtype=torch.int64, device=gpu)
    L.bench_check_writes(n, status, err, rxid, xid, pay, want, -1, zx, ok,
                         zmax)
    assert int(ok.item()) == n - 4
    assert int(zmax.item()) == int(zx.max().item())
    ok.zero_()
    L.bench_check_writes(n, status, err, rxid, xid, want * 0 + 7, None, 7,
                         zx, ok, zmax)
    assert int(ok.item()) == n - 3
    base = torch.tensor([(1 << 31) - 5], dtype=torch.int64, device=gpu)
    out = torch.empty(10, **i32)
    L.bench_xids(10, base, out)
    assert out.cpu().tolist() == [(1 << 31) - 5 + k if k < 5 else k - 5
                                  for k in range(10)]


def test_gpu_storm_pipeline(gpu):
    from zkmi.bench.synthetic import StormPipeline
    tree = _small_tree(gpu, 20000, 37, spare=1.5)
    pipe = StormPipeline(tree, 8192, ndirs=64)
    for _ in range(12):
        ok = pipe.step()
        assert int(ok.item()) == 8192
    # 13 steps: 7 sessions born, 6 resumed (5 next to a refused expired
    # one), 6 expired with exactly their two batches
    assert pipe.stats == {'born': 7, 'resumed': 6, 'expired': 6,
                          'expired_resume_refused': 5,
                          'cross_rank_resumes': 0}
    assert bool(pipe.hs_ok.item())


def test_gpu_storm_pipeline_captured(gpu):
    """The storm step replayed from HIP graphs: session ids come from the
    device (TC_SESS), so every replay serves, expires and checks the NEXT
    session; the hash index is never rebuilt (the expiry reclaims it).
    Then eager steps carry on from the replayed state."""
    from zkmi.bench.synthetic import StormPipeline
    tree = _small_tree(gpu, 20000, 37, spare=1.5)
    pipe = StormPipeline(tree, 8192, ndirs=64)
    acc = torch.zeros(64, dtype=torch.int64, device=gpu)
    g = pipe.capture(acc)
    torch.cuda.synchronize()
    acc.zero_()
    for _ in range(14):
        g.replay()
    torch.cuda.synchronize()
    assert int(acc.sum().item()) == 14 * 8192
    _, live, used, tomb = tree.digest()
    assert used - tomb == live and tomb < tree.hcap // 20
    for _ in range(2):
        assert int(pipe.step().item()) == 8192
    assert bool(pipe.hs_ok.item())
    st = pipe.stats
    assert st['born'] == (pipe.step_no + 1) // 2
    assert st['resumed'] == pipe.step_no // 2
    assert st['expired'] == st['born'] - 1
    assert int(pipe.kdev.item()) == pipe.k


def test_gpu_session_handshake_k9_server(gpu):
    """The GPU server's handshake against the oracle's records: new
    session, resume with the right password, wrong password and unknown id
    get the expired answer, a too-new lastZxidSeen is refused."""
    from zkmi.bench.synthetic import GpuSessionTable
    from zkmi.ops import _lib
    tree = _small_tree(gpu, 1000, 16)
    st = GpuSessionTable(tree)

    def hs(reqs, n_new):
        raw = b''.join(jute.frame(jute.encode_connect_request(q))
                       for q in reqs)
        buf = _dev_bytes(raw, gpu)
        resp, bound, oc = st.connect(buf, len(raw), n_new)
        rb = bytes(resp[:41 * len(reqs)].cpu().numpy().tobytes())
        frames, _, bad = jute.scan_frames(rb)
        assert bad < 0 and len(frames) == len(reqs)
        return ([jute.decode_connect_response(rb[o:o + n])
                 for o, n in frames], oc[:len(reqs)].cpu().tolist())
    base = {'protocolVersion': 0, 'lastZxidSeen': 0, 'timeOut': 100000,
            'sessionId': 0, 'passwd': b'\0' * 8}
    (r,), oc = hs([base], 1)
    assert oc == [_lib.SC_NEW] and r['sessionId'] == st.sid_of(0)
    assert r['timeOut'] == 40000 and len(r['passwd']) == 16
    sid, pw = r['sessionId'], r['passwd']
    reqs = [dict(base, sessionId=sid, passwd=pw, timeOut=1000),
            dict(base, sessionId=sid, passwd=b'x' * 16),
            dict(base, sessionId=st.sid_of(7), passwd=pw),
            dict(base, sessionId=sid, passwd=pw, lastZxidSeen=1 << 50)]
    rs, oc = hs(reqs, 0)
    assert oc == [_lib.SC_RESUMED, _lib.SC_EXPIRED, _lib.SC_EXPIRED,
                  _lib.SC_REFUSED]
    assert rs[0] == {'protocolVersion': 0, 'timeOut': 4000,
                     'sessionId': sid, 'passwd': pw}
    assert [x['sessionId'] for x in rs[1:]] == [0, 0, 0]
    st.close(torch.tensor([sid], dtype=torch.int64, device=gpu))
    (r,), oc = hs([dict(base, sessionId=sid, passwd=pw)], 0)
    assert oc == [_lib.SC_EXPIRED] and r['sessionId'] == 0


def test_gpu_watch_pipeline_single_rank(gpu):
    """Write-triggered notification fan-out on one rank: GET_DATA watch=1
    arms the server's watch table, SET_DATA of the same nodes fires one
    NodeDataChanged each (K13), K1 + K8 decode and the device check; a few
    records against the Jute oracle, and nothing fires twice."""
    from zkmi.bench.synthetic import GpuTree, WatchPipeline
    tree = GpuTree(20000, 37, fanout=100, device=gpu, seed=0,
                   watch_cap=8192)
    pipe = WatchPipeline(tree, 5000)
    for _ in range(2):
        ok = pipe.step()
        assert int(ok.item()) == 5000
    rep, ft, idx = pipe.last
    assert ft.host_result()['frames'] == 5000
    assert pipe.server.ev_total.cpu().tolist() == [5000, 5000]
    hb = bytes(pipe.rx[:4096].cpu().numpy().tobytes())
    frames, _, _ = jute.scan_frames(hb)
    arena = tree.path_arena.cpu().numpy().tobytes()
    po = tree.node_path_off[idx[:20]].cpu().tolist()
    pl = tree.node_path_len[idx[:20]].cpu().tolist()
    for k, (o, ln) in enumerate(frames[:20]):
        pkt = jute.decode_response(hb[o:o + ln], {})
        assert pkt['opcode'] == 'NOTIFICATION' and pkt['xid'] == -1
        assert pkt['type'] == 'DATA_CHANGED'
        assert pkt['state'] == 'SYNC_CONNECTED'
        assert pkt['path'].encode() == arena[po[k]:po[k] + pl[k]]
    # a write nobody watches any more fires nothing
    from zkmi.ops import batch as B
    rb = pipe._batch(pipe.ops_set, pipe.neg32, idx, pipe._xids(), True)
    tx, _, total, _ = B.encode_requests(rb, pipe.xt, out=pipe.tx)
    pipe.server.serve(tx, total, session=pipe.sid_wr, wslot=1)
    assert pipe.server.ev_total.cpu().tolist() == [0, 0]


def _watch_rank(rank, world, port, q):
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from zkmi.bench.synthetic import GpuTree, WatchPipeline
        dev = torch.device('cuda', 0)
        tree = GpuTree(20000, 37, fanout=100, device=dev, seed=rank,
                       watch_cap=8192)
        pipe = WatchPipeline(tree, 3000, coll_device='cpu')
        ok = pipe.step()
        q.put((rank, int(ok.item())))
    finally:
        dist.destroy_process_group()


def test_gpu_watch_pipeline_two_ranks_gloo(gpu):
    """Two ranks sharing the GPU, collective on gloo (the RCCL path needs
    one GPU per rank): every rank decodes and checks BOTH ranks'
    notifications (each rank drew its own nodes)."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_watch_rank, args=(r, 2, port, q))
             for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    assert all(p.exitcode == 0 for p in procs)
    got = dict(q.get(timeout=5) for _ in range(2))
    assert got == {0: 6000, 1: 6000}


def test_gpu_get_pipeline_variable_sizes(gpu):
    """GET over variable data (0..1024 bytes) and path lengths: every reply
    checked on the device, and K1's frames of the reply stream equal the
    host framer's.  (Structured reply bytes keep garbage chains alive deep
    into K1's tiles; a join past the first 2 KiB of a tile once took the
    wrong survivor index.)"""
    from zkmi.bench.synthetic import GpuTree, GetPipeline
    tree = GpuTree(100_000, 0, fanout=1000, device=gpu, data_dist=(0, 1024),
                   name_pad=(0, 16))
    pipe = GetPipeline(tree, 1 << 16)
    for _ in range(3):
        assert int(pipe.step().item()) == 1 << 16
    idx, rep, rx, ft = pipe.last
    n = 1 << 16
    ro = pipe.server.last_rec_off[:n].cpu().numpy()
    end = int(ro[-1]) + 4 + int(rep.pay_len[n - 1].item()) + 16 + 4 + 68
    frames, cons, bad = jute.scan_frames(
        bytes(rx[:end].cpu().numpy().tobytes()))
    assert bad < 0 and cons == end and len(frames) == n
    assert ft.off[:n].cpu().numpy().tolist() == [o for o, _ in frames]
