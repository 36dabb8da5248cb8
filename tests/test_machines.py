"""The native session / connection / client machines
(csrc/host/zk_machines.cpp) against their Python oracle (the state
functions in zkmi/models/*.py, selected with ZKMI_PY_FSM=1).

Each scenario runs once per implementation; the state histories of the
client, its session and its connections and the client's events must come
out the same (lib/client.js:123-181, lib/zk-session.js:38-375,
lib/connection-fsm.js:27-351)."""

import pytest

from zkmi.models import connection as C
from zkmi.models import session as S
from zkmi.server import FakeZKServer

from zkhelpers import Recorder, client, wait_for

pytestmark = pytest.mark.skipif(S._zkmach is None,
                                reason='native machines not built')


@pytest.fixture
def zk():
    s = FakeZKServer(tick_ms=250)
    yield s
    s.shutdown()


def _mode(monkeypatch, native):
    if native:
        monkeypatch.delenv('ZKMI_PY_FSM', raising=False)
    else:
        monkeypatch.setenv('ZKMI_PY_FSM', '1')


def _histories(c, conns):
    """(client, session, [connections]) state histories, on the loop."""
    def go():
        return (list(c.fsm_history), list(c.session.fsm_history),
                [list(x.fsm_history) for x in conns])
    return c.loop.run(go)


def _scenario_reconnect(zk):
    """connect, a request, the socket killed (the session resumes on a new
    connection), a request, close."""
    c = client(zk.servers())
    rec = Recorder(c)
    c.wait_connected(10)
    conns = []
    c.loop.run(lambda: conns.append(c.getSession().getConnection()))
    assert c.call_sync('create', '/m', b'x', {}) == '/m'

    def kill():
        sock = c.getSession().getConnection().zcf_socket
        sock.inject_error(Exception('killed'))
        sock.destroy()
    c.loop.run(kill)
    rec.wait('connect', 2)
    c.loop.run(lambda: conns.append(c.getSession().getConnection()))
    assert c.call_sync('get', '/m')[0] == b'x'
    c.close_sync(10)
    assert wait_for(lambda: c.loop.run(lambda: conns[-1].getState()) ==
                    'closed', 10)
    return list(rec.events), _histories(c, conns)


def _scenario_expiry(zk):
    """the server expires the session: the client gets 'expire' and a new
    session."""
    c = client(zk.servers(), session_timeout=2000)
    rec = Recorder(c)
    c.wait_connected(10)
    sess = c.loop.run(lambda: c.getSession())
    # the expiry closes the session's connection itself (server side, in
    # the server's loop): dropping the connection first let the client's
    # reconnect race the expiry, and the histories differed by timing
    zk.run(lambda: [zk.db.expire_session(s) for s in list(zk.db.sessions)])
    rec.wait('expire', 1, 15)
    hist = c.loop.run(lambda: list(sess.fsm_history))
    c.close_sync(10)
    return list(rec.events), hist


@pytest.mark.parametrize('scenario', [_scenario_reconnect, _scenario_expiry])
def test_native_matches_oracle(zk, monkeypatch, scenario):
    out = {}
    for native in (True, False):
        _mode(monkeypatch, native)
        srv = FakeZKServer(tick_ms=250)      # a fresh tree each time
        try:
            out[native] = scenario(srv)
        finally:
            srv.shutdown()
    assert out[True] == out[False]


def test_native_is_the_default(zk, monkeypatch):
    _mode(monkeypatch, True)
    c = client(zk.servers())
    c.wait_connected(10)
    sess = c.loop.run(lambda: c.getSession())
    conn = c.loop.run(lambda: sess.getConnection())
    assert isinstance(sess, S.NativeZKSession)
    assert isinstance(conn, C.NativeZKConnectionFSM)
    assert type(c._fsm_core).__name__ == 'Machine'
    c.close_sync(10)
    _mode(monkeypatch, False)
    c = client(zk.servers())
    c.wait_connected(10)
    sess = c.loop.run(lambda: c.getSession())
    assert isinstance(sess, S.PyZKSession)
    assert isinstance(c.loop.run(lambda: sess.getConnection()),
                      C.PyZKConnectionFSM)
    c.close_sync(10)


def test_relays_do_not_accumulate(zk, monkeypatch):
    """A machine subscribes each peer once; moving to a new connection drops
    the old one's relays (no listener growth over reconnects)."""
    _mode(monkeypatch, True)
    c = client(zk.servers())
    rec = Recorder(c)
    c.wait_connected(10)
    for k in range(5):
        def kill():
            sock = c.getSession().getConnection().zcf_socket
            sock.inject_error(Exception('killed'))
            sock.destroy()
        c.loop.run(kill)
        rec.wait('connect', k + 2)
    sess = c.loop.run(lambda: c.getSession())
    conn = c.loop.run(lambda: sess.getConnection())
    # the session: its connection's four events and the expiry timer
    assert c.loop.run(lambda: sess._m.subscriptions) == 5
    # the connection: its socket's four events (the session's only while
    # handshaking)
    assert c.loop.run(lambda: conn._m.subscriptions) == 4
    assert c.loop.run(lambda: sess.listenerCount('stateChanged')) == 1
    c.close_sync(10)
