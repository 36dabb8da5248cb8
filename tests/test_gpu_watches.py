"""ZooKeeper watches in the GPU server (csrc/kernels/tree.hip wt_*):
reads with watch=1 arm one-shot watches per watcher slot, writes fire
NodeDataChanged / NodeCreated / NodeDeleted / NodeChildrenChanged as xid -1
notification frames (K13), and SET_WATCHES catches a resumed session up.

Every batch is also applied, one request at a time, to the fake server's
database (zkmi/server/fakezk.py, the semantics of SURVEY Appendix D); the
notifications each watcher receives must be the same, in the same order.
Reference: lib/zk-session.js:558-574 (trigger table, client side),
:986-1005 (arming requests), lib/zk-buffer.js:364-370 (notification)."""

import pytest

from zkmi import jute
from zkmi.ops import batch as B

pytestmark = pytest.mark.gpu

FANOUT = 100
NLEAF = 2000


class _Handle(object):
    def cancel(self):
        pass


class _Loop(object):
    """Enough loop for a ZKDatabase that never expires a session."""

    def call_later(self, ms, fn, *a):
        return _Handle()

    def time_ms(self):
        return 0


class _Conn(object):
    def __init__(self):
        self.got = []

    def send_notification(self, evtype, path):
        self.got.append((evtype, path))


def leaf(i):
    return '/bench/d%06d/n%09d' % (i // FANOUT, i)


class Mirror(object):
    """The GPU tree and the fake server's database side by side."""

    def __init__(self, dev):
        from zkmi.bench.synthetic import GpuTree, GpuServer
        from zkmi.server.fakezk import ZKDatabase
        self.dev = dev
        self.tree = GpuTree(NLEAF, 24, fanout=FANOUT, device=dev, seed=3,
                            watch_cap=4096, scratch=1 << 20)
        self.srv = GpuServer(self.tree, 256, 256 * 400, window=256)
        self.db = ZKDatabase(_Loop())
        w = ZKDatabase._world()
        self.db.create('/bench', b'', [w], [], None)
        for d in range((NLEAF + FANOUT - 1) // FANOUT):
            self.db.create('/bench/d%06d' % d, b'', [w], [], None)
        for i in range(NLEAF):
            self.db.create(leaf(i), b'x', [w], [], None)
        self.conns = {}
        self.sids = {}
        for slot in range(3):
            s = self.db.new_session(30000)
            s.conn = self.conns[slot] = _Conn()
            self.sids[slot] = s.sid
        self.xid = 1
        self.gpu_notes = {k: [] for k in range(3)}

    def batch(self, slot, pkts, ordered=True):
        """Serve ``pkts`` from watcher ``slot``'s session on the GPU and
        apply them in order to the fake database; returns the GPU replies'
        error names."""
        for p in pkts:
            p['xid'] = self.xid
            self.xid += 1
        xmap = {p['xid']: p['opcode'] for p in pkts}
        rb = B.pack_requests(pkts, self.dev)
        tx, _, total, _ = B.encode_requests(rb, B.XidTable(bits=12,
                                                           device=self.dev))
        out, rtotal, _, _ = self.srv.serve(tx, total, session=self.sids[slot],
                                           wslot=slot, ordered=ordered,
                                           passes=8)
        errs = self._replies(out, rtotal, xmap)
        self._collect(self.srv.notif)
        for p in pkts:
            rep = self.db.handle(dict(p, acl=p.get('acl', [])),
                                 self.sids[slot])
            assert rep['err'] == errs[p['xid']], (p, rep['err'],
                                                  errs[p['xid']])
        return errs

    def resume(self, slot, rel_gpu, data=(), exist=(), child=()):
        """SET_WATCHES for ``slot``: the GPU server gets relZxid = rel_gpu,
        the fake database its own zxid at the same point (rel_db)."""
        fr = B.encode_set_watches(rel_gpu, data, exist, child,
                                  device=self.dev)
        out, rtotal, _, _ = self.srv.serve(fr, fr.numel(),
                                           session=self.sids[slot],
                                           wslot=slot, resume=True)
        errs = self._replies(out, rtotal, {})
        assert list(errs.values()) == ['OK']
        self._collect(self.srv.notif)
        buf, total, res = self.srv.resume_notif
        n = int(total.item())
        raw = bytes(buf[:n].cpu().numpy().tobytes())
        frames, _, bad = jute.scan_frames(raw)
        assert bad < 0 and len(frames) == int(res[0].item())
        for o, ln in frames:
            pkt = jute.decode_response(raw[o:o + ln], {})
            self.gpu_notes[slot].append((pkt['type'], pkt['path']))
        return int(res[1].item())

    def _replies(self, out, rtotal, xmap):
        raw = bytes(out[:int(rtotal.item())].cpu().numpy().tobytes())
        frames, _, bad = jute.scan_frames(raw)
        assert bad < 0
        errs = {}
        for o, ln in frames:
            pkt = jute.decode_response(raw[o:o + ln], xmap)
            errs[pkt['xid']] = pkt['err']
        return errs

    def _collect(self, notif):
        buf, total, slots, count = notif
        n = int(count.item())
        raw = bytes(buf[:int(total.item())].cpu().numpy().tobytes())
        frames, _, bad = jute.scan_frames(raw)
        assert bad < 0 and len(frames) == n
        sl = slots[:n].cpu().tolist()
        for (o, ln), s in zip(frames, sl):
            pkt = jute.decode_response(raw[o:o + ln], {})
            assert pkt['xid'] == -1 and pkt['state'] == 'SYNC_CONNECTED'
            self.gpu_notes[s].append((pkt['type'], pkt['path']))

    def check(self):
        for slot in range(3):
            assert self.gpu_notes[slot] == self.conns[slot].got, slot


def _get(p, w=True):
    return {'opcode': 'GET_DATA', 'path': p, 'watch': w}


def _exists(p, w=True):
    return {'opcode': 'EXISTS', 'path': p, 'watch': w}


def _set(p, v=-1):
    return {'opcode': 'SET_DATA', 'path': p, 'data': b'new', 'version': v}


def _create(p, flags=()):
    return {'opcode': 'CREATE', 'path': p, 'data': b'c',
            'acl': [jute_world()], 'flags': list(flags)}


def _delete(p, v=-1):
    return {'opcode': 'DELETE', 'path': p, 'version': v}


def jute_world():
    return {'perms': ['READ', 'WRITE', 'CREATE', 'DELETE', 'ADMIN'],
            'id': {'scheme': 'world', 'id': 'anyone'}}


def test_watch_trigger_rules_match_fake_server(gpu):
    m = Mirror(gpu)
    d0 = '/bench/d000000'
    # watcher 0: data watches, exist watches on missing paths, a GET of a
    # missing path (NO_NODE: no watch), an unwatched read
    m.batch(0, [_get(leaf(k)) for k in range(10)] +
            [_exists(d0 + '/new%d' % k) for k in range(5)] +
            [_exists(leaf(k)) for k in range(10, 15)] +
            [_get(d0 + '/miss'), _get(leaf(40), False)])
    # watcher 2 overlaps watcher 0 on leaves 5..9
    m.batch(2, [_get(leaf(k)) for k in range(5, 10)] +
            [_get(leaf(k)) for k in range(20, 25)])
    m.check()
    assert all(not v for v in m.gpu_notes.values())
    # writer (slot 1): every trigger kind; one-shot (leaf 0 set twice);
    # writes nobody watches; a failed write fires nothing
    m.batch(1, [_set(leaf(k)) for k in range(10)] +
            [_create(d0 + '/new%d' % k) for k in range(3)] +
            [_delete(leaf(k)) for k in range(10, 13)] +
            [_delete(leaf(20)), _set(leaf(0)), _create(d0 + '/miss'),
             _set(leaf(40)), _set(leaf(21), 7), _delete(leaf(22), 5)])
    m.check()
    assert len(m.gpu_notes[0]) == 10 + 3 + 3
    assert len(m.gpu_notes[2]) == 5 + 1
    # re-arm after a fire, then a same-batch read-then-write on one path
    # (ordered serve: the watch armed first fires)
    m.batch(0, [_get(leaf(0)), _exists(d0 + '/new3')])
    m.batch(1, [_get(leaf(30)), _set(leaf(0)), _create(d0 + '/new3'),
                _delete(d0 + '/new3'), _set(leaf(30))])
    m.batch(2, [_get(leaf(31)), _set(leaf(31))])
    m.check()


def test_set_watches_catch_up_matches_fake_server(gpu):
    m = Mirror(gpu)
    d0 = '/bench/d000000'
    from zkmi.ops import _lib
    m.batch(1, [_create(d0 + '/late')])
    rel = int(m.tree.counters[_lib.TC_ZXID].item())
    rel_db = m.db.zxid
    # changes after the watcher's last seen zxid
    m.batch(1, [_set(leaf(1)), _delete(leaf(2)), _create(d0 + '/born')])
    # the watcher resumes: data [changed, deleted, unchanged], exist
    # [created meanwhile, still missing, existing before], child [deleted]
    data = [leaf(1), leaf(2), leaf(3)]
    exist = [d0 + '/born', d0 + '/never', d0 + '/late']
    child = [leaf(2)]
    rearmed = m.resume(0, rel, data, exist, child)
    m.db.set_watches(rel_db, {'dataChanged': data,
                              'createdOrDestroyed': exist,
                              'childrenChanged': child}, m.sids[0])
    m.check()
    assert [t for t, _ in m.gpu_notes[0]] == ['DATA_CHANGED', 'DELETED',
                                              'CREATED', 'CREATED',
                                              'DELETED']
    assert rearmed == 2                       # leaf 3, /never
    # the re-armed watches fire on the next writes
    m.batch(1, [_set(leaf(3)), _create(d0 + '/never')])
    m.check()
    assert m.gpu_notes[0][-2:] == [('DATA_CHANGED', leaf(3)),
                                   ('CREATED', d0 + '/never')]
