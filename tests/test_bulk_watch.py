"""Bulk watches — the owner side of the node-wide fan-out (R1,
zkmi/parallel/fanout.py): ``Client.watch_bulk`` + ``bulk_get(watch=True)``
arm data watches whose NOTIFICATION frames the transport keeps (the native
loop's note sink, csrc/host/zk_loop.cpp; the Python loop's fallback in
zkmi/models/connection.py), ``take_notes`` hands them over as raw frames,
``bulk_set`` fires them, and a session that moves re-arms them with a
SET_WATCHES whose path vector is kept pre-encoded
(``jute.PackedStrings``), the server replaying what changed while it was
away.  Runs on the CPU (host codec), on both event loops, against the
native 3-member server.

Reference: lib/zk-session.js:853-854 (a watcher's events), :421-471
(SET_WATCHES resume), test/multi-node.test.js:233-350 (member failover)."""

import threading
import time

import pytest

from zkmi import codec
from zkmi import consts
from zkmi import jute
from zkmi.config import ClientConfig, RecoveryPolicy
from zkmi.models.client import Client
from zkmi.runtime import loop as L
from zkmi.runtime import nloop
from zkmi.server import fast

N = 600


def test_packed_strings_encode_like_a_list():
    paths = ['/a', '/b/ü', '/c' * 40]
    extra = ['/x', '/y']
    p = jute.PackedStrings.of(paths)
    assert len(p) == 3 and list(p) == paths
    both = extra + p
    assert list(both) == extra + paths
    for ev in ({'dataChanged': both},
               {'dataChanged': extra, 'childrenChanged': p}):
        pkt = {'xid': consts.XID_SET_WATCHES, 'opcode': 'SET_WATCHES',
               'relZxid': 77, 'events': ev}
        assert jute.packed_events(ev)
        plain = dict(pkt, events={k: list(v) for k, v in ev.items()})
        assert jute.encode_request(pkt) == codec.encode_request(plain)
        back = jute.decode_request(jute.encode_request(pkt))
        assert back['events']['dataChanged'] == list(ev['dataChanged'])


def _loops():
    out = ['asyncio']
    if nloop.available():
        out.append('native')
    return out


def _wait(fn, what, timeout=20.0):
    t_end = time.monotonic() + timeout
    while True:
        v = fn()
        if v:
            return v
        if time.monotonic() > t_end:
            raise AssertionError('timed out waiting for ' + what)
        time.sleep(0.005)


def _bulk(call, *args, **kw):
    done = threading.Event()
    box = {}

    def cb(err, res=None):
        box['err'], box['res'] = err, res
        done.set()
    call(*args, cb, **kw)
    assert done.wait(30), 'bulk batch timed out'
    assert box['err'] is None, box['err']
    return box['res']


def _note_paths(raw, k):
    frames, _, bad = codec.scan_frames(raw, 0, len(raw), consts.MAX_PACKET)
    assert bad < 0 and len(frames) == k
    out = []
    for o, ln in frames:
        pk = codec.decode_response(raw[o:o + ln], {})
        assert pk['xid'] == consts.XID_NOTIFICATION
        assert pk['type'] == 'DATA_CHANGED'
        out.append(pk['path'])
    return out


class _Notes(object):
    def __init__(self, client):
        self.c = client
        self.paths = []

    def until(self, n):
        def more():
            raw, k = self.c.take_notes()
            if k:
                self.paths += _note_paths(raw, k)
            return len(self.paths) >= n
        _wait(more, '%d notifications' % n)
        got, self.paths = self.paths, []
        return got


@pytest.mark.skipif(not fast.available(), reason='zk_fastserver not built')
@pytest.mark.parametrize('kind', _loops())
def test_bulk_watch_notes_and_failover_replay(kind, monkeypatch):
    monkeypatch.setenv('ZKMI_LOOP', kind)
    srv = fast.FastZKServer(members=3)
    lp = L.new_loop('bulk-watch-' + kind)
    connects = []
    cfg = ClientConfig(connect_policy=RecoveryPolicy(1000, 3, 5, 100),
                       default_policy=RecoveryPolicy(1000, 3, 5, 100))
    c = Client({'servers': [{'address': '127.0.0.1', 'port': p}
                            for p in srv.ports],
                'sessionTimeout': 8000, 'config': cfg, 'device': False,
                'loop': lp,
                'listeners': [('connect', lambda: connects.append(1))]})
    try:
        c.wait_connected(20)
        paths = ['/bw/p%04d' % k for k in range(N)]
        c.call_sync('create', '/bw', b'', {})
        res = _bulk(c.bulk, [{'opcode': 'CREATE', 'path': p, 'data': b'0'}
                             for p in paths])
        assert set(res.errors()) == {'OK'}
        c.watch_bulk(paths)
        c.watch_bulk(paths[:10])            # (already watched: no-op)
        res = _bulk(c.bulk_get, paths, watch=True)
        assert set(res.errors()) == {'OK'} and res.n == N
        notes = _Notes(c)
        raw, k = c.take_notes()
        assert k == 0 and raw == b''
        # a write fires each armed watch once; the notes are raw frames
        w1 = paths[::3]
        res = _bulk(c.bulk_set, w1, b'one')
        assert set(res.errors()) == {'OK'}
        assert sorted(notes.until(len(w1))) == sorted(w1)
        # fired watches stay quiet until re-armed
        _bulk(c.bulk_set, w1[:5], b'again')
        _bulk(c.bulk_get, w1, watch=True)
        raw, k = c.take_notes()
        assert k == 0
        w2 = paths[1::3]
        _bulk(c.bulk_set, w2 + w1[:7], b'two')
        assert sorted(notes.until(len(w2) + 7)) == sorted(w2 + w1[:7])
        _bulk(c.bulk_get, w2 + w1[:7], watch=True)
        # member down; writes while the session is away; the session moves,
        # SET_WATCHES (the pre-encoded bulk vector) replays exactly those
        port = c.loop.run(
            lambda: c.getSession().getConnection().server['port'])
        before = len(connects)
        w3 = paths[2::5]
        srv.outage(srv.ports.index(port), [(p, b'three') for p in w3])
        _wait(lambda: len(connects) > before, 'the failover')
        assert sorted(notes.until(len(w3))) == sorted(w3)
        assert c.loop.run(lambda: c.getSession().rearmed) >= N
        # and every watch is armed again on the new member
        _bulk(c.bulk_get, w3, watch=True)
        _bulk(c.bulk_set, paths, b'four')
        assert sorted(notes.until(N)) == sorted(paths)
        res = _bulk(c.bulk_get, paths[:3])
        assert [p['data'] for p in res.packets()[:3]] == [b'four'] * 3
    finally:
        try:
            c.close_sync(10)
        finally:
            lp.stop()
            srv.shutdown()


@pytest.mark.skipif(not fast.available(), reason='zk_fastserver not built')
@pytest.mark.parametrize('kind', _loops())
def test_watchers_keep_firing_with_bulk_watches(kind, monkeypatch):
    """With the note sink on, events for a watcher()'s path still reach the
    watcher (and stay out of the sink unless the path is also a bulk
    watch); bulk paths go to the sink only (the sink swallowed
    every notification of the connection)."""
    monkeypatch.setenv('ZKMI_LOOP', kind)
    srv = fast.FastZKServer(members=1)
    lp = L.new_loop('bulk-watch-mixed-' + kind)
    c = Client({'servers': [{'address': '127.0.0.1', 'port': srv.ports[0]}],
                'sessionTimeout': 8000, 'device': False, 'loop': lp})
    try:
        c.wait_connected(20)
        c.call_sync('create', '/mx', b'', {})
        for p in ('/mx/w', '/mx/b', '/mx/both'):
            c.call_sync('create', p, b'0', {})
        seen = {'/mx/w': [], '/mx/both': []}
        for p in seen:
            c.watcher(p).on('dataChanged',
                            lambda d, s, p=p: seen[p].append(d))
        _wait(lambda: all(v == [b'0'] for v in seen.values()), 'arming')
        c.watch_bulk(['/mx/b', '/mx/both'])
        _bulk(c.bulk_get, ['/mx/b', '/mx/both'], watch=True)
        notes = _Notes(c)
        for p in ('/mx/w', '/mx/b', '/mx/both'):
            c.call_sync('set', p, b'1', -1)
        # the sink: the bulk paths only
        assert sorted(notes.until(2)) == ['/mx/b', '/mx/both']
        # the watchers: fired and re-armed with the new data
        _wait(lambda: seen['/mx/w'][-1:] == [b'1'], 'the watcher event')
        _wait(lambda: seen['/mx/both'][-1:] == [b'1'], 'the shared event')
        raw, k = c.take_notes()
        assert k == 0
    finally:
        try:
            c.close_sync(10)
        finally:
            lp.stop()
            srv.shutdown()
