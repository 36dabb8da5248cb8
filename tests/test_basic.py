"""Single-server integration suite — the reference's test/basic.test.js
(37 tape tests against a real ZooKeeper), here against the in-process fake
server.  Scenario names follow the reference."""

import threading
import time

import pytest

from zkmi.server import FakeZKServer
from zkmi.errors import ZKError, ZKProtocolError

from zkhelpers import Box, Recorder, client, wait_for


@pytest.fixture
def zk():
    s = FakeZKServer(tick_ms=250)
    yield s
    s.shutdown()


@pytest.fixture
def zkc(zk):
    c = client(zk.servers())
    c.wait_connected(10)
    yield c
    c.close_sync(10)


# -- connect / ping (basic.test.js:36-120) --------------------------------

def test_simple_connect_and_ping(zk):
    # JS attaches listeners in the constructor's tick, before any event can
    # fire; with the client on its own loop thread the equivalent is the
    # ``listeners`` option (attached before the client starts)
    pinged = Box()
    closed = Box()
    box = {}

    def on_connect():
        assert wait_for(lambda: 'c' in box, 5)
        c = box['c']
        assert c.isConnected()
        c.ping(lambda err: (pinged(err), c.close()))
    c = box['c'] = client(zk.servers(), listeners=[('connect', on_connect),
                                                    ('close', closed)])
    assert pinged.wait()[0] is None
    closed.wait()
    assert not c.isConnected()


def test_double_ping_coalesces(zk, zkc):
    before = zk.run(lambda: zk.db.stats['requests'])
    got = []
    done = threading.Event()

    def both():
        def cb(err):
            got.append(err)
            if len(got) == 2:
                done.set()
        zkc.ping(cb)
        zkc.ping(cb)
    zkc.loop.run(both)
    assert done.wait(5) and got == [None, None]
    after = zk.run(lambda: zk.db.stats['requests'])
    assert after - before == 1        # one PING on the wire (xid -2)


def test_connect_ping_with_death_expires(zk):
    c = client(zk.servers(), session_timeout=1000)
    rec = Recorder(c)
    c.wait_connected(10)
    c.call_sync('ping')
    t1 = time.monotonic()
    zk.stop()
    rec.wait('expire', timeout=10)
    assert time.monotonic() - t1 >= 0.95
    c.close_sync(10)
    assert rec.events[:2] == ['session', 'connect']
    assert 'expire' in rec.events and rec.events[-1] == 'close'


# -- data API (basic.test.js:122-642) --------------------------------------

def test_list_and_get(zk, zkc):
    zk.cli_create('/foo', b'hi')
    kids, stat = zkc.call_sync('list', '/')
    assert sorted(kids) == ['foo', 'zookeeper']
    assert stat.numChildren == 2
    data, stat = zkc.call_sync('get', '/foo')
    assert data == b'hi' and stat.dataLength == 2 and stat.version == 0


def test_get_acl(zk, zkc):
    zk.cli_create('/foo', b'hi')
    acl = zkc.call_sync('getACL', '/foo')
    assert len(acl) == 1
    assert acl[0]['id'] == {'scheme': 'world', 'id': 'anyone'}
    assert sorted(acl[0]['perms']) == ['ADMIN', 'CREATE', 'DELETE', 'READ',
                                       'WRITE']


def test_delete_and_no_node(zk, zkc):
    zk.cli_create('/foo', b'hi')
    assert zkc.call_sync('delete', '/foo', 0) is None
    with pytest.raises(ZKError) as ei:
        zkc.call_sync('stat', '/foo')
    assert ei.value.code == 'NO_NODE'
    assert ei.value.message.startswith('NO_NODE: ')


def test_create_node(zk, zkc):
    assert zkc.call_sync('create', '/foo', b'hi there', {}) == '/foo'
    assert zk.cli_get('/foo') == b'hi there'
    with pytest.raises(ZKError) as ei:
        zkc.call_sync('create', '/foo', b'x', {})
    assert ei.value.code == 'NODE_EXISTS'


def test_create_empty_data(zk, zkc):
    assert zkc.call_sync('create', '/foonull', b'', {}) == '/foonull'
    data, stat = zkc.call_sync('get', '/foonull')
    assert data == b'' and stat.dataLength == 0
    zkc.call_sync('delete', '/foonull', -1)


def test_set_with_version_cas(zk, zkc):
    zkc.call_sync('create', '/v', b'a', {})
    assert zkc.call_sync('set', '/v', b'b', 0) is None
    with pytest.raises(ZKError) as ei:
        zkc.call_sync('set', '/v', b'c', 0)
    assert ei.value.code == 'BAD_VERSION'
    zkc.call_sync('set', '/v', b'd', None)           # -1 wildcard
    data, stat = zkc.call_sync('get', '/v')
    assert data == b'd' and stat.version == 2


def test_create_with_empty_parents_basic(zk, zkc):
    p = zkc.call_sync('createWithEmptyParents', '/hi/there', b'hi there', {})
    assert p == '/hi/there'
    assert zk.cli_get('/hi') == b'null'
    assert zk.cli_get('/hi/there') == b'hi there'


def test_create_with_empty_parents_no_overwrite(zk, zkc):
    zkc.call_sync('create', '/exist', b'exist', {})
    assert zkc.call_sync('createWithEmptyParents', '/exist/new', b'new',
                         {}) == '/exist/new'
    assert zkc.call_sync('get', '/exist')[0] == b'exist'
    assert zkc.call_sync('get', '/exist/new')[0] == b'new'


def test_create_with_empty_parents_existing(zk, zkc):
    zkc.call_sync('createWithEmptyParents', '/new/path', b'new', {})
    with pytest.raises(ZKError) as ei:
        zkc.call_sync('createWithEmptyParents', '/new/path', b'overwrite',
                      {})
    assert ei.value.code == 'NODE_EXISTS'
    assert zkc.call_sync('get', '/new/path')[0] == b'new'


def test_create_with_empty_parents_no_ephemeral_parents(zk, zkc):
    p = zkc.call_sync('createWithEmptyParents', '/no/ephem/parents/child',
                      b'ephemeral', {'flags': ['EPHEMERAL']})
    assert p == '/no/ephem/parents/child'
    for q in ('/no', '/no/ephem', '/no/ephem/parents'):
        assert zkc.call_sync('stat', q).ephemeralOwner == 0
    assert zkc.call_sync('stat', p).ephemeralOwner != 0


def test_create_with_empty_parents_no_sequential_parents(zk, zkc):
    p = zkc.call_sync('createWithEmptyParents', '/no/seq/parents/child',
                      b'sequence node', {'flags': ['SEQUENTIAL']})
    assert p.startswith('/no/seq/parents/child') and len(p) == len(
        '/no/seq/parents/child') + 10
    for q in ('/no', '/no/seq', '/no/seq/parents'):
        zkc.call_sync('stat', q)
    zkc.call_sync('stat', p)


def test_large_node(zk, zkc):
    d = bytes([5]) * 9000
    assert zkc.call_sync('create', '/bignode', d, {}) == '/bignode'
    out, stat = zkc.call_sync('get', '/bignode')
    assert len(out) == 9000 and out[5] == 5
    zkc.call_sync('delete', '/bignode', -1)


def test_sequential_naming(zk, zkc):
    zkc.call_sync('create', '/q', b'', {})
    a = zkc.call_sync('create', '/q/n-', b'', {'flags': ['SEQUENTIAL']})
    b = zkc.call_sync('create', '/q/n-', b'', {'flags': ['SEQUENTIAL']})
    assert a == '/q/n-0000000000' and b == '/q/n-0000000001'


def test_sync(zk, zkc):
    assert zkc.call_sync('sync', '/') is None


def test_ephemeral_deleted_on_close(zk):
    c = client(zk.servers())
    c.wait_connected(10)
    c.call_sync('create', '/eph', b'x', {'flags': ['EPHEMERAL']})
    assert zk.cli_exists('/eph')
    c.close_sync(10)
    assert wait_for(lambda: not zk.cli_exists('/eph'), 5)


# -- watchers (basic.test.js:644-981) --------------------------------------

def _collect(w, evt, out, fmt=lambda *a: a):
    w.on(evt, lambda *a: out.append(fmt(*a)))


def test_data_watcher(zk, zkc):
    zk.cli_create('/foo', b'hi there')
    seen = []
    _collect(zkc.watcher('/foo'), 'dataChanged', seen, lambda d, s: d)
    assert wait_for(lambda: seen == [b'hi there'], 5)
    zk.cli_set('/foo', b'hi')
    assert wait_for(lambda: seen == [b'hi there', b'hi'], 5)


def test_delete_while_watching(zk, zkc):
    zk.cli_create('/foo', b'hi')
    deleted = Box()
    zkc.watcher('/foo').on('deleted', deleted)
    stat = zkc.call_sync('stat', '/foo')
    zkc.call_sync('delete', '/foo', stat.version)
    deleted.wait()


def test_delete_while_watching_data(zk, zkc):
    zk.cli_create('/foobar', b'hi')
    fired = []
    w = zkc.watcher('/foobar')
    w.on('dataChanged', lambda d, s: fired.append('data'))
    deleted = Box()
    w.on('deleted', deleted)
    assert wait_for(lambda: fired == ['data'], 5)
    stat = zkc.call_sync('stat', '/foobar')
    zkc.call_sync('delete', '/foobar', stat.version)
    deleted.wait()
    assert fired == ['data']


def test_children_watcher(zk, zkc):
    zk.cli_create('/foobar', b'hi')
    seen = {}
    done = threading.Event()

    def on_kids(kids, stat):
        # latest cversion per shape, as basic.test.js:776-786 records them
        if 'foobar' in kids:
            seen['foobar'] = stat.cversion
        if 'foo' in kids:
            seen['foo'] = stat.cversion
        if kids == ['zookeeper']:
            seen['none'] = stat.cversion
        if 'foo' in seen and seen.get('none', -1) > seen['foo']:
            done.set()
    zkc.watcher('/').on('childrenChanged', on_kids)
    assert wait_for(lambda: 'foobar' in seen, 5)
    zkc.call_sync('delete', '/foobar', -1)
    zkc.call_sync('create', '/foo', b'hi', {})
    assert wait_for(lambda: 'foo' in seen, 5)
    zkc.call_sync('delete', '/foo', -1)
    assert done.wait(5)
    assert seen['foo'] > seen['foobar'] and seen['none'] > seen['foo']


def test_children_watcher_no_node(zk, zkc):
    seen = {}
    done = threading.Event()

    def on_kids(kids, stat):
        if len(kids) == 0:
            seen.setdefault('none', stat.cversion)
        if 'foo' in kids and 'foobar' in kids:
            seen.setdefault('all', stat.cversion)
            done.set()
    zkc.watcher('/parent').on('childrenChanged', on_kids)
    time.sleep(0.3)
    zkc.call_sync('create', '/parent', b'', {})
    assert wait_for(lambda: 'none' in seen, 5)
    zkc.call_sync('create', '/parent/foo', b'hi', {})
    zkc.call_sync('create', '/parent/foobar', b'hi', {})
    assert done.wait(5)
    assert seen['all'] > seen['none']


def test_deletion_watcher_sequence(zk, zkc):
    zkc.call_sync('create', '/delseq', b'hi', {})
    evts = []
    w = zkc.watcher('/delseq')
    w.on('deleted', lambda: evts.append('deleted'))
    w.on('created', lambda s: evts.append('created'))
    assert wait_for(lambda: evts == ['created'], 5)
    zkc.call_sync('delete', '/delseq', -1)
    assert wait_for(lambda: len(evts) >= 2, 5)
    zkc.call_sync('create', '/delseq', b'hi', {})
    assert wait_for(lambda: len(evts) >= 3, 5)
    zkc.call_sync('delete', '/delseq', -1)
    assert wait_for(lambda: len(evts) >= 4, 5)
    time.sleep(0.2)
    assert evts == ['created', 'deleted', 'created', 'deleted']


def test_data_watcher_sequence(zk, zkc):
    zkc.call_sync('create', '/dataseq', b'hi', {})
    evts = []
    zkc.watcher('/dataseq').on('dataChanged',
                               lambda d, s: evts.append(d.decode()))
    assert wait_for(lambda: evts == ['hi'], 5)
    zkc.call_sync('set', '/dataseq', b'hi2', -1)
    zkc.call_sync('delete', '/dataseq', -1)
    zkc.call_sync('create', '/dataseq', b'hi', {})
    assert wait_for(lambda: len(evts) >= 3, 5)
    zkc.call_sync('set', '/dataseq', b'hi2', -1)
    zkc.call_sync('delete', '/dataseq', -1)
    assert wait_for(lambda: len(evts) >= 4, 5)
    time.sleep(0.2)
    assert evts == ['hi', 'hi2', 'hi', 'hi2']


def test_watcher_once_throws(zkc):
    with pytest.raises(Exception):
        zkc.watcher('/x').once('created', lambda *a: None)


def test_notification_metric(zk, zkc):
    zk.cli_create('/m', b'1')
    seen = []
    zkc.watcher('/m').on('dataChanged', lambda d, s: seen.append(d))
    assert wait_for(lambda: len(seen) == 1, 5)
    zk.cli_set('/m', b'2')
    assert wait_for(lambda: len(seen) == 2, 5)
    c = zkc.collector.getCollector('zookeeper_notifications')
    assert c.get({'event': 'dataChanged'}) >= 1
    ev = zkc.collector.getCollector('zookeeper_events')
    assert ev.get({'evtype': 'session'}) == 1
    assert ev.get({'evtype': 'connect'}) >= 1
    assert 'zookeeper_events{evtype="session"} 1' in zkc.collector.collect()


# -- session resumption (basic.test.js:983-1342) ---------------------------

def _kill_socket(c, error=True):
    def go():
        conn = c.getSession().getConnection()
        sock = conn.zcf_socket
        assert sock.listenerCount('error') > 0
        if error:
            sock.inject_error(Exception('I killed it'))
        sock.destroy()
    c.loop.run(go)


@pytest.mark.parametrize('error', [True, False])
def test_session_resumption_with_watcher(zk, error):
    c1 = client(zk.servers())
    c2 = client(zk.servers())
    rec = Recorder(c1)
    c1.wait_connected(10)
    c2.wait_connected(10)
    created = []
    c2.watcher('/foo').on('created', lambda s: created.append(1))
    got = []
    c1.watcher('/foo').on('dataChanged', lambda d, s: got.append(d))
    assert c1.call_sync('create', '/foo', b'hi there', {}) == '/foo'
    assert wait_for(lambda: created and got == [b'hi there'], 5)
    stat = c2.call_sync('stat', '/foo')
    _kill_socket(c1, error)
    c2.call_sync('set', '/foo', b'hello again', stat.version)
    assert wait_for(lambda: b'hello again' in got, 10)
    c1.close_sync(10)
    c2.close_sync(10)
    assert rec.events == ['session', 'connect', 'disconnect', 'connect',
                          'close']


def test_session_resumption_new_watcher_race_39(zk):
    c1 = client(zk.servers())
    c2 = client(zk.servers())
    rec = Recorder(c1)
    c1.wait_connected(10)
    c2.wait_connected(10)
    counts = {}

    def inc(k):
        return lambda *a: counts.__setitem__(k, counts.get(k, 0) + 1)

    reconnected = threading.Event()

    def go():
        c1.once('connect', lambda: reconnected.set())
        c1.watcher('/race1').on('created', inc('race1'))
        conn = c1.getSession().getConnection()
        sock = conn.zcf_socket
        sock.inject_error(Exception('I killed it'))
        sock.destroy()
        c1.watcher('/race2').on('created', inc('race2'))
        c1.loop.call_soon(lambda: c1.watcher('/race3').on('created',
                                                          inc('race3')))
    c1.loop.run(go)
    assert reconnected.wait(10)
    for p in ('/race1', '/race2', '/race3'):
        c2.call_sync('create', p, b'hi there', {})
    assert wait_for(lambda: counts == {'race1': 1, 'race2': 1, 'race3': 1},
                    10), counts
    assert c1.loop.run(
        lambda: c1.getSession().listenerCount('stateChanged')) == 1
    c1.close_sync(10)
    c2.close_sync(10)
    assert rec.events == ['session', 'connect', 'disconnect', 'connect',
                          'close']


def test_session_resumption_existence_watch(zk):
    c1 = client(zk.servers())
    c2 = client(zk.servers())
    rec = Recorder(c2)
    c1.wait_connected(10)
    c2.wait_connected(10)
    created = Box()
    c2.watcher('/foo4').on('created', created)
    c2.call_sync('sync', '/foo4')
    _kill_socket(c2, error=False)
    c1.call_sync('create', '/foo4', b'hello again', {})
    created.wait(10)
    c1.close_sync(10)
    c2.close_sync(10)
    assert rec.events == ['session', 'connect', 'disconnect', 'connect',
                          'close']


def test_clean_close_cancelled_request_46(zk):
    c = client(zk.servers())
    rec = Recorder(c)
    c.wait_connected(10)
    res = Box()

    def go():
        conn = c.getSession().getConnection()
        sock = conn.zcf_socket
        sock.pause_reading()        # the reference test unpipes the socket
        c.create('/foo5', b'hello again', {}, lambda err, *a: (res(err),
                                                               c.close()))
        c.loop.call_soon(conn.close)
        c.loop.call_later(500, lambda: sock.inject_error(Exception('dead')))
    c.loop.run(go)
    err = res.wait(10)[0]
    assert isinstance(err, ZKProtocolError)
    assert 'Connection closed.' in str(err)
    rec.wait('close')
    assert rec.events == ['session', 'connect', 'disconnect', 'close']


# -- connect failures (basic.test.js:1391-1448) ----------------------------

def test_connect_refused_fails(zk):
    port = zk.port
    zk.stop()
    c = client([{'address': '127.0.0.1', 'port': port}])
    rec = Recorder(c)
    rec.wait('failed', timeout=20)
    c.close_sync(10)
    assert 'connect' not in rec.events
    ev = c.collector.getCollector('zookeeper_events')
    assert ev.get({'evtype': 'failed'}) == 1


def test_connect_immediate_close_fails(zk):
    zk.set_mode('close')
    c = client(zk.servers())
    rec = Recorder(c)
    rec.wait('failed', timeout=20)
    c.close_sync(10)
    assert 'connect' not in rec.events
    assert zk.accepted >= 1


def test_reconnect_after_server_restart(zk):
    c = client(zk.servers(), session_timeout=4000)
    rec = Recorder(c)
    c.wait_connected(10)
    zk.stop()
    rec.wait('disconnect', timeout=10)
    zk.start()
    rec.wait('connect', n=2, timeout=10)
    assert c.call_sync('ping') is None
    c.close_sync(10)
    assert rec.events[:4] == ['session', 'connect', 'disconnect', 'connect']


def test_expired_session_gets_new_session(zk):
    c = client(zk.servers(), session_timeout=1000)
    rec = Recorder(c)
    c.wait_connected(10)
    old = c.getSession().getSessionId()
    # make the server forget the session while the client is cut off
    zk.pause_reads()
    zk.drop_connections()
    zk.run(lambda: [zk.db.expire_session(s) for s in list(zk.db.sessions)])
    zk.resume_reads()
    rec.wait('session', n=2, timeout=15)
    assert c.getSession().getSessionId() != old
    assert 'expire' in rec.events
    c.close_sync(10)
