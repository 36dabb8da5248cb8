"""Watches and ensemble members of the native server (csrc/host/
zk_fastserver.cpp): the trigger table, SET_WATCHES catch-up and member
outages, checked against the fake server's database (zkmi/server/fakezk.py,
SURVEY Appendix D) applied one request at a time, over raw wire sessions.

Reference: lib/zk-session.js:558-574 (trigger table, client side), :421-471
(watch resume with SET_WATCHES), test/multi-node.test.js:233-350 (member
failover)."""

import socket

import pytest

from zkmi import consts
from zkmi import jute
from zkmi.server import fast

pytestmark = pytest.mark.skipif(not fast.available(),
                                reason='zk_fastserver not built')

FANOUT = 100
NLEAF = 300


def leaf(i):
    return '/bench/d%06d/n%09d' % (i // FANOUT, i)


class Raw(object):
    """One wire session: blocking calls; notifications collected in order."""

    def __init__(self, port, sid=0, passwd=b'\0' * 16):
        self.s = socket.create_connection(('127.0.0.1', port), timeout=10)
        self.buf = b''
        self.notes = []
        self.xid = 1
        self.s.sendall(jute.frame(jute.encode_connect_request(
            {'timeOut': 30000, 'sessionId': sid, 'passwd': passwd})))
        rep = jute.decode_connect_response(self._frame())
        self.sid, self.passwd = rep['sessionId'], rep['passwd']

    def _frame(self):
        while True:
            if len(self.buf) >= 4:
                n = int.from_bytes(self.buf[:4], 'big')
                if len(self.buf) >= 4 + n:
                    body = self.buf[4:4 + n]
                    self.buf = self.buf[4 + n:]
                    return body
            chunk = self.s.recv(1 << 16)
            if not chunk:
                raise ConnectionError('closed')
            self.buf += chunk

    def call(self, pkt):
        if pkt['opcode'] == 'SET_WATCHES':
            xid = consts.XID_SET_WATCHES
        elif pkt['opcode'] == 'PING':
            xid = consts.XID_PING
        else:
            xid = self.xid
            self.xid += 1
        pkt = dict(pkt, xid=xid)
        self.s.sendall(jute.frame(jute.encode_request(pkt)))
        while True:
            rep = jute.decode_response(self._frame(), {xid: pkt['opcode']})
            if rep['xid'] == consts.XID_NOTIFICATION:
                assert rep['state'] == 'SYNC_CONNECTED'
                self.notes.append((rep['type'], rep['path']))
                continue
            assert rep['xid'] == xid
            return rep

    def sync(self):
        """A ping round trip: every notification of writes before it is in."""
        self.call({'opcode': 'PING'})

    def close(self):
        self.s.close()


class _Handle(object):
    def cancel(self):
        pass


class _Loop(object):
    def call_later(self, ms, fn, *a):
        return _Handle()

    def time_ms(self):
        return 0


class _Conn(object):
    def __init__(self):
        self.got = []

    def send_notification(self, evtype, path):
        self.got.append((evtype, path))


class Mirror(object):
    """The native server and the fake database side by side."""

    def __init__(self, members=1):
        from zkmi.server.fakezk import ZKDatabase
        self.srv = fast.FastZKServer(preload=NLEAF, data_bytes=8,
                                     fanout=FANOUT, members=members)
        self.db = ZKDatabase(_Loop())
        w = ZKDatabase._world()
        self.db.create('/bench', b'', [w], [], None)
        for d in range((NLEAF + FANOUT - 1) // FANOUT):
            self.db.create('/bench/d%06d' % d, b'', [w], [], None)
        for i in range(NLEAF):
            self.db.create(leaf(i), b'x', [w], [], None)
        self.raw, self.conns, self.sids = {}, {}, {}
        for slot in range(3):
            self.raw[slot] = Raw(self.srv.ports[0])
            s = self.db.new_session(30000)
            s.conn = self.conns[slot] = _Conn()
            self.sids[slot] = s.sid

    def batch(self, slot, pkts):
        errs = []
        for p in pkts:
            rep = self.raw[slot].call(p)
            want = self.db.handle(dict(p, xid=0, acl=p.get('acl', [])),
                                  self.sids[slot])
            assert rep['err'] == want['err'], (p, rep['err'], want['err'])
            errs.append(rep['err'])
        return errs

    def check(self):
        for slot in range(3):
            self.raw[slot].sync()
            assert self.raw[slot].notes == self.conns[slot].got, slot

    def close(self):
        for r in self.raw.values():
            r.close()
        self.srv.shutdown()


def _get(p, w=True):
    return {'opcode': 'GET_DATA', 'path': p, 'watch': w}


def _exists(p, w=True):
    return {'opcode': 'EXISTS', 'path': p, 'watch': w}


def _kids(p, w=True):
    return {'opcode': 'GET_CHILDREN2', 'path': p, 'watch': w}


def _set(p, v=-1, data=b'new'):
    return {'opcode': 'SET_DATA', 'path': p, 'data': data, 'version': v}


def _create(p):
    return {'opcode': 'CREATE', 'path': p, 'data': b'c',
            'acl': [{'perms': ['READ', 'WRITE', 'CREATE', 'DELETE', 'ADMIN'],
                     'id': {'scheme': 'world', 'id': 'anyone'}}],
            'flags': []}


def _delete(p, v=-1):
    return {'opcode': 'DELETE', 'path': p, 'version': v}


def test_trigger_rules_match_fake_server():
    m = Mirror()
    try:
        d0 = '/bench/d000000'
        m.batch(0, [_get(leaf(k)) for k in range(10)] +
                [_exists(d0 + '/new%d' % k) for k in range(5)] +
                [_exists(leaf(k)) for k in range(10, 15)] +
                [_get(d0 + '/miss'), _get(leaf(40), False), _kids(d0)])
        m.batch(2, [_get(leaf(k)) for k in range(5, 10)] +
                [_get(leaf(k)) for k in range(20, 25)] + [_kids(leaf(21))])
        m.check()
        assert not any(r.notes for r in m.raw.values())
        m.batch(1, [_set(leaf(k)) for k in range(10)] +
                [_create(d0 + '/new%d' % k) for k in range(3)] +
                [_delete(leaf(k)) for k in range(10, 13)] +
                [_delete(leaf(20)), _set(leaf(0)), _create(d0 + '/miss'),
                 _set(leaf(40)), _set(leaf(21), 7), _delete(leaf(22), 5),
                 _delete(leaf(21))])
        m.check()
        # re-arm after a fire; a session's own write fires its own watch
        # (the notification ahead of the write's reply)
        m.batch(0, [_get(leaf(0)), _exists(d0 + '/new3')])
        m.batch(0, [_set(leaf(0))])
        assert m.raw[0].notes[-1] == ('DATA_CHANGED', leaf(0))
        m.batch(1, [_get(leaf(30)), _create(d0 + '/new3'),
                    _delete(d0 + '/new3'), _set(leaf(30))])
        m.check()
        assert len(m.raw[0].notes) > 10 and len(m.raw[2].notes) > 5
    finally:
        m.close()


def test_set_watches_catch_up_matches_fake_server():
    m = Mirror()
    try:
        d0 = '/bench/d000000'
        m.batch(1, [_create(d0 + '/late')])
        rel = m.raw[1].call({'opcode': 'EXISTS', 'path': d0,
                             'watch': False})['zxid']
        rel_db = m.db.zxid
        m.batch(1, [_set(leaf(1)), _delete(leaf(2)), _create(d0 + '/born')])
        data = [leaf(1), leaf(2), leaf(3)]
        exist = [d0 + '/born', d0 + '/never', d0 + '/late']
        child = [leaf(2), d0]
        ev = {'dataChanged': data, 'createdOrDestroyed': exist,
              'childrenChanged': child}
        rep = m.raw[0].call({'opcode': 'SET_WATCHES', 'relZxid': rel,
                             'events': ev})
        assert rep['err'] == 'OK'
        m.db.set_watches(rel_db, ev, m.sids[0])
        m.check()
        assert [t for t, _ in m.raw[0].notes] == [
            'DATA_CHANGED', 'DELETED', 'CREATED', 'CREATED', 'DELETED',
            'CHILDREN_CHANGED']
        # the re-armed ones fire on the next writes
        m.batch(1, [_set(leaf(3)), _create(d0 + '/never')])
        m.check()
        assert m.raw[0].notes[-2:] == [('DATA_CHANGED', leaf(3)),
                                       ('CREATED', d0 + '/never')]
    finally:
        m.close()


def test_large_set_watches_catch_up_and_rearm():
    """A SET_WATCHES past the server's parallel lookup size (8192 paths:
    the lookups run on the helper threads with a prefetch lookahead, the
    session's watch index is a flat set) replays the changes since relZxid
    in list order and re-arms the rest: later writes fire exactly those."""
    n = 12000
    srv = fast.FastZKServer(preload=n, data_bytes=8, fanout=FANOUT,
                            serve_threads=4)
    try:
        a = Raw(srv.port)
        w = Raw(srv.port)
        rel = a.call(_get(leaf(0), False))['zxid']
        changed = list(range(5, n, 997))
        for i in changed:
            w.call(_set(leaf(i)))
        paths = [leaf(i) for i in range(n)] + ['/bench/none%d' % k
                                               for k in range(3)]
        rep = a.call({'opcode': 'SET_WATCHES', 'relZxid': rel,
                      'events': {'dataChanged': paths}})
        assert rep['err'] == 'OK'
        assert a.notes == [('DATA_CHANGED', leaf(i)) for i in changed] + \
            [('DELETED', '/bench/none%d' % k) for k in range(3)]
        later = [7, 4001, 11999]
        for i in later:
            w.call(_set(leaf(i)))
        a.sync()
        assert a.notes[len(changed) + 3:] == [('DATA_CHANGED', leaf(i))
                                              for i in later]
        a.close()
        for i in (8, 9):                   # the closed session's watches
            w.call(_set(leaf(i)))
        w.sync()
        assert w.notes == []
        w.close()
    finally:
        srv.shutdown()


def test_member_outage_and_resume():
    """A session on member 0 watches two nodes; member 0 goes down while
    one of them is written; the session resumes on member 1, SET_WATCHES
    replays the change and re-arms the other watch; member 0 comes back."""
    srv = fast.FastZKServer(preload=NLEAF, data_bytes=8, fanout=FANOUT,
                            members=3)
    try:
        assert len(srv.ports) == 3
        a = Raw(srv.ports[0])
        w = Raw(srv.ports[2])
        for k in (1, 2):
            assert a.call(_get(leaf(k)))['err'] == 'OK'
        rel = a.call(_get(leaf(3), False))['zxid']
        z = srv.outage(0, [(leaf(1), b'during')])
        assert z > rel
        with pytest.raises((ConnectionError, OSError)):
            a.sync()
        with pytest.raises(OSError):
            socket.create_connection(('127.0.0.1', srv.ports[0]), timeout=2)
        b = Raw(srv.ports[1], a.sid, a.passwd)
        assert b.sid == a.sid
        b.call({'opcode': 'SET_WATCHES', 'relZxid': rel,
                'events': {'dataChanged': [leaf(1), leaf(2)]}})
        assert b.notes == [('DATA_CHANGED', leaf(1))]
        assert b.call(_get(leaf(1)))['data'] == b'during'
        w.call(_set(leaf(2)))
        b.sync()
        assert b.notes[-1] == ('DATA_CHANGED', leaf(2))
        assert srv.start(0) == srv.ports[0]
        c = Raw(srv.ports[0])
        c.sync()
        for r in (b, c, w):
            r.close()
    finally:
        srv.shutdown()


def _read_burst(port, reqs, nreplies):
    """One raw session: the whole request stream in one send, then every
    reply frame (bytes, in order)."""
    r = Raw(port)
    r.s.sendall(reqs)
    out = []
    for _ in range(nreplies):
        out.append(r._frame())
    r.s.close()
    return out


def test_parallel_read_burst_matches_serial():
    """A connection's large read burst (>= 8192 plain reads) is served in
    chunks by the server's helper threads; its replies must be the serial
    server's, byte for byte and in order: GET_DATA / EXISTS (some with
    watch=1) / GET_CHILDREN2 / SYNC, present and missing nodes."""
    ops = []
    for i in range(12000):
        k = i % 5
        p = leaf(i % NLEAF) if i % 7 else '/bench/missing%d' % i
        if k == 0:
            ops.append({'opcode': 'GET_DATA', 'path': p, 'watch': i % 3 == 0})
        elif k == 1:
            ops.append({'opcode': 'EXISTS', 'path': p, 'watch': i % 4 == 0})
        elif k == 2:
            ops.append({'opcode': 'GET_CHILDREN2',
                        'path': '/bench/d%06d' % (i % 3), 'watch': False})
        elif k == 3:
            ops.append({'opcode': 'SYNC', 'path': p})
        else:
            ops.append({'opcode': 'GET_DATA', 'path': p, 'watch': False})
    reqs = b''.join(jute.frame(jute.encode_request(dict(o, xid=i + 1)))
                    for i, o in enumerate(ops))
    got = {}
    for st in (0, 4):
        srv = fast.FastZKServer(preload=NLEAF, data_bytes=24, fanout=FANOUT,
                                serve_threads=st)
        try:
            got[st] = _read_burst(srv.port, reqs, len(ops))
            w = srv.timing()
        finally:
            srv.shutdown()
        assert (w['par_bursts'] > 0) == (st > 0), w
    # (the two servers' preloads ran at different times: ctime / mtime)
    xmap = {i + 1: o['opcode'] for i, o in enumerate(ops)}

    def norm(body):
        rep = jute.decode_response(body, xmap)
        st = rep.get('stat')
        if st is not None:
            rep['stat'] = (st.czxid, st.mzxid, st.version, st.cversion,
                           st.dataLength, st.numChildren, st.pzxid,
                           st.ephemeralOwner)
        return rep
    assert len(got[0]) == len(got[4])
    assert [norm(b) for b in got[0]] == [norm(b) for b in got[4]]


def test_parallel_write_burst_matches_serial():
    """A connection's burst of >= 512 SET_DATAs on distinct paths (config
    4's bulk write) is applied on the helper threads: lookups and checks in
    parallel, zxids in request order, nodes updated and replies built in
    chunks, watches fired in request order with one wake per watching
    connection.  Its replies and the watcher's notifications must be the
    serial server's, in order: version CAS hits and misses, missing nodes,
    watched and unwatched paths."""
    n = 3000
    ops = []
    for i in range(n):
        p = leaf(i) if i % 97 else '/bench/missing%d' % i
        ops.append({'opcode': 'SET_DATA', 'path': p, 'data': b'v%d' % i,
                    'version': -1 if i % 5 else (0 if i % 2 else 3)})
    reqs = b''.join(jute.frame(jute.encode_request(dict(o, xid=i + 1)))
                    for i, o in enumerate(ops))
    got, notes = {}, {}
    for st in (0, 4):
        srv = fast.FastZKServer(preload=n, data_bytes=8, fanout=FANOUT,
                                serve_threads=st)
        try:
            w = Raw(srv.port)
            for i in range(0, n, 3):
                w.call(_get(leaf(i)))                 # data watch
            got[st] = _read_burst(srv.port, reqs, n)
            w.sync()
            notes[st] = list(w.notes)
            w.close()
            t = srv.timing()
        finally:
            srv.shutdown()
        assert (t['par_bursts'] > 0) == (st > 0), t
    xmap = {i + 1: o['opcode'] for i, o in enumerate(ops)}

    def norm(body):
        rep = jute.decode_response(body, xmap)
        st = rep.get('stat')
        if st is not None:
            rep['stat'] = (st.czxid, st.mzxid, st.version, st.dataLength)
        return rep
    a = [norm(b) for b in got[0]]
    assert a == [norm(b) for b in got[4]]
    errs = {r['err'] for r in a}
    assert errs == {'OK', 'BAD_VERSION', 'NO_NODE'}, errs
    assert notes[0] == notes[4]
    assert len(notes[0]) > 500


def test_parallel_write_burst_own_watches():
    """The writer watches some of the paths it writes (config 4 at one
    rank): the parallel burst must still match the serial server frame for
    frame — each own notification right before its write's reply — and
    the other watcher's notifications too."""
    n = 2000
    ops = [{'opcode': 'SET_DATA', 'path': leaf(i), 'data': b'w%d' % i,
            'version': -1} for i in range(n)]
    reqs = b''.join(jute.frame(jute.encode_request(dict(o, xid=1000 + i)))
                    for i, o in enumerate(ops))
    got, notes = {}, {}
    for st in (0, 4):
        srv = fast.FastZKServer(preload=n, data_bytes=8, fanout=FANOUT,
                                serve_threads=st)
        try:
            other = Raw(srv.port)
            for i in range(0, n, 5):
                other.call(_get(leaf(i)))
            r = Raw(srv.port)
            for i in range(0, n, 2):
                r.call(_get(leaf(i)))                 # the writer's own
            r.s.sendall(reqs)
            frames, replies = [], 0
            while replies < n:
                b = r._frame()
                frames.append(b)
                if int.from_bytes(b[:4], 'big', signed=True) != -1:
                    replies += 1
            got[st] = frames
            other.sync()
            notes[st] = list(other.notes)
            r.close()
            other.close()
            t = srv.timing()
        finally:
            srv.shutdown()
        assert (t['par_bursts'] > 0) == (st > 0), t
    xmap = {1000 + i: 'SET_DATA' for i in range(n)}

    def norm(body):
        rep = jute.decode_response(body, xmap)
        st = rep.get('stat')
        if st is not None:
            rep['stat'] = (st.czxid, st.mzxid, st.version, st.dataLength)
        return rep
    a = [norm(b) for b in got[0]]
    assert a == [norm(b) for b in got[4]]
    own = [x for x in a if x['xid'] == consts.XID_NOTIFICATION]
    assert len(own) == n // 2
    assert notes[0] == notes[4] and len(notes[0]) == n // 5

