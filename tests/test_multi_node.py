"""3-server ensemble suite — the reference's test/multi-node.test.js (three
JVMs on one host), here as three fake endpoints sharing one database.  Adds
session migration (cueball decoherence) and reattach-revert coverage."""

import time

import pytest

from zkmi.server import FakeEnsemble, FakeZKServer

from zkhelpers import Box, Recorder, client, fast_config, wait_for


@pytest.fixture
def ens():
    e = FakeEnsemble(3, tick_ms=250)
    yield e
    e.shutdown()


def _backend_port(c):
    def go():
        conn = c.getSession().getConnection()   # None while (re)attaching
        return None if conn is None else conn.server['port']
    return c.loop.run(go)


@pytest.mark.parametrize('member', [0, 2])
def test_connect_and_ping(ens, member):
    c = client([ens[member].address])
    c.wait_connected(10)
    assert c.call_sync('ping') is None
    c.close_sync(10)


def test_write_visibility(ens):
    c1 = client([ens[0].address])
    c2 = client([ens[1].address])
    c1.wait_connected(10)
    c2.wait_connected(10)
    assert c1.call_sync('create', '/foo', b'hello world', {}) == '/foo'
    c1.call_sync('sync', '/foo')
    data, stat = c2.call_sync('get', '/foo')
    assert data == b'hello world' and stat.version == 0
    c1.close_sync(10)
    c2.close_sync(10)


def test_cross_server_data_watch(ens):
    c1 = client([ens[0].address])
    c2 = client([ens[1].address])
    c1.wait_connected(10)
    c2.wait_connected(10)
    c1.call_sync('create', '/foo', b'x', {})
    got = Box()
    c1.watcher('/foo').on('dataChanged', lambda d, s: d == b'testing' and
                          got(d, s))
    time.sleep(0.2)
    c2.call_sync('set', '/foo', b'testing', 0)
    c2.call_sync('sync', '/foo')
    d, s = got.wait()
    assert s.version > 0
    c1.close_sync(10)
    c2.close_sync(10)


def test_ephemeral_failover(ens):
    c1 = client(ens.servers(), session_timeout=3000)
    c2 = client([ens[2].address])
    rec1 = Recorder(c1)
    c1.wait_connected(10)
    c2.wait_connected(10)
    assert _backend_port(c1) == ens[0].port        # preference order
    created, deleted = [], []

    def on_created(stat):
        created.append(1)
        c2.watcher('/foo.ephem').on('deleted', lambda: deleted.append(1))
    c2.watcher('/foo.ephem').on('created', on_created)
    sid = c1.getSession().getSessionId()
    assert c1.call_sync('create', '/foo.ephem', b'hello world',
                        {'flags': ['EPHEMERAL']}) == '/foo.ephem'
    c1.call_sync('sync', '/foo.ephem')
    c2.call_sync('sync', '/foo.ephem')
    assert wait_for(lambda: created, 5) and not deleted
    ens[0].stop()                                 # kill server 1
    rec1.wait('connect', n=2, timeout=10)         # moved to another server
    assert _backend_port(c1) in (ens[1].port, ens[2].port)
    assert c1.getSession().getSessionId() == sid
    time.sleep(3.5)                               # > sessionTimeout
    assert created and not deleted
    assert c2.call_sync('get', '/foo.ephem')[0] == b'hello world'
    ens[0].start()
    time.sleep(0.5)
    assert c1.call_sync('get', '/foo.ephem')[0] == b'hello world'
    assert not deleted
    c1.close_sync(10)
    c2.close_sync(10)
    assert rec1.events[:4] == ['session', 'connect', 'disconnect', 'connect']
    # closing the owning session deletes the ephemeral
    assert wait_for(lambda: not ens[1].cli_exists('/foo.ephem'), 5)


def test_session_migration_decoherence(ens):
    """Every decoherence interval the set prefers another backend; the
    session is moved there (reattaching -> attached) without a disconnect
    and watches keep working (zk-session.js:265-339)."""
    cfg = fast_config(decoherence_interval_s=0.6)
    c = client(ens.servers(), config=cfg)
    rec = Recorder(c)
    c.wait_connected(10)
    first = _backend_port(c)
    sid = c.getSession().getSessionId()
    seen = []
    c.watcher('/mig').on('dataChanged', lambda d, s: seen.append(d))
    ens[0].cli_create('/mig', b'0')
    assert wait_for(lambda: seen == [b'0'], 5)
    assert wait_for(lambda: _backend_port(c) not in (first, None), 5)
    assert c.getSession().getSessionId() == sid
    assert 'disconnect' not in rec.events
    ens[0].cli_set('/mig', b'1')
    assert wait_for(lambda: seen == [b'0', b'1'], 5)
    c.close_sync(10)
    assert rec.events.count('session') == 1


def test_reattach_revert_on_unknown_session():
    """The preferred backend does not know the session (answers sid 0):
    the move is reverted and the session stays on the old connection."""
    a = FakeZKServer(tick_ms=250)
    b = FakeZKServer(tick_ms=250)           # separate db: unknown session
    try:
        cfg = fast_config(decoherence_interval_s=0.6)
        c = client(a.servers() + b.servers(), config=cfg)
        rec = Recorder(c)
        c.wait_connected(10)
        sid = c.getSession().getSessionId()
        assert wait_for(lambda: b.accepted >= 1, 5)
        time.sleep(0.5)
        assert c.getSession().getSessionId() == sid
        assert _backend_port(c) == a.port
        assert c.call_sync('ping') is None
        assert 'expire' not in rec.events
        c.close_sync(10)
    finally:
        a.shutdown()
        b.shutdown()
