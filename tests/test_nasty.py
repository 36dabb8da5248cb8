"""Fault injection with misbehaving servers — the reference's
test/nasty.test.js (inline net.createServer fakes), here via the fake
server's fault hooks.  Time constants are scaled down ~10x."""

import binascii
import time

import pytest

from zkmi import jute
from zkmi.errors import ZKNotConnectedError
from zkmi.server import FakeZKServer
from zkmi.utils.log import create_logger

from zkhelpers import Box, Recorder, client, wait_for


def h(s):
    return binascii.unhexlify(s)


@pytest.fixture
def zk():
    s = FakeZKServer(tick_ms=250)
    yield s
    s.shutdown()


def _failed_with(zk, code):
    log = create_logger('nasty', level='warn', stream=open('/dev/null', 'w'))
    recs = log.capture()
    c = client(zk.servers(), log=log)
    rec = Recorder(c)
    rec.wait('failed', timeout=20)
    c.close_sync(10)
    assert 'connect' not in rec.events
    codes = [r.get('err', {}).get('code') for r in recs if 'err' in r]
    assert code in codes, codes


def test_bad_length_too_big_split(zk):
    # 0x40004000 > 16 MiB, the length split across two writes
    zk.set_mode('write', raw_writes=[(0, h('4000')), (100, h('4000'))])
    _failed_with(zk, 'BAD_LENGTH')


def test_bad_length_zero(zk):
    # a zero-length frame cannot hold a ConnectResponse -> BAD_DECODE
    zk.set_mode('write', raw_writes=[(0, h('000000000102'))])
    _failed_with(zk, 'BAD_DECODE')


def test_bad_length_negative(zk):
    zk.set_mode('write', raw_writes=[(0, h('fffffffe0102'))])
    _failed_with(zk, 'BAD_LENGTH')


def test_handshake_bad_version(zk):
    zk.set_mode('bad_version')
    _failed_with(zk, 'VERSION_INCOMPAT')


def test_handshake_unexpected_extra_packet(zk):
    cr = jute.frame(jute.encode_connect_response(
        {'protocolVersion': 0, 'timeOut': 30000, 'sessionId': 5,
         'passwd': b'\0' * 16}))
    zk.set_mode('write', raw_writes=[(50, cr + cr)])
    _failed_with(zk, 'UNEXPECTED_PACKET')


def test_argument_assertions(zk):
    c = client(zk.servers())
    with pytest.raises(TypeError):
        c.list(5, lambda *a: None)
    with pytest.raises(TypeError):
        c.list('/foo')                                   # no callback
    with pytest.raises(TypeError):
        c.create('/foo', 'not-bytes', {}, lambda *a: None)
    with pytest.raises(TypeError):
        c.delete('/foo', '1', lambda *a: None)
    with pytest.raises(TypeError):
        c.create('/foo', b'', {'flags': 'EPHEMERAL'}, lambda *a: None)
    with pytest.raises(ValueError):
        c.create('/foo', b'', {'flags': ['BOGUS']}, lambda *a: None)
    with pytest.raises(TypeError):
        c.getACL(None, lambda *a: None)
    c.close_sync(10)


def test_options_validation():
    from zkmi import Client
    with pytest.raises(TypeError):
        Client(address='127.0.0.1')                       # port required
    with pytest.raises(TypeError):
        Client(servers=[{'address': '127.0.0.1', 'port': 'x'}])
    with pytest.raises(TypeError):
        Client(address='127.0.0.1', port=1, sessionTimeout='5')


def test_calling_before_ready_not_connected(zk):
    zk.stop()
    c = client(zk.servers())
    res = Box()
    c.list('/', res)
    err = res.wait()[0]
    assert err.code == 'CONNECTION_LOSS'
    assert isinstance(err, ZKNotConnectedError)
    c.close_sync(10)


def test_calling_during_handshake(zk):
    zk.set_mode('hang')
    c = client(zk.servers())
    rec = Recorder(c)
    assert wait_for(lambda: zk.accepted >= 1, 5)
    res = Box()
    c.list('/', res)
    err = res.wait()[0]
    assert err.code == 'CONNECTION_LOSS'
    assert err.name == 'ZKNotConnectedError'
    c.close_sync(10)
    assert 'connect' not in rec.events


def test_attach_and_send_cr_race():
    """Two hanging backends; one closes and relistens while the set retries
    (nasty.test.js:40-103).  Several connections race to attach to the one
    session; the client must not crash (loop error fixture) and must close."""
    a = FakeZKServer(tick_ms=250)
    b = FakeZKServer(tick_ms=250, loop=a.loop, db=a.db)
    a.set_mode('hang')
    b.set_mode('hang')
    try:
        c = client(a.servers() + b.servers())
        rec = Recorder(c)
        time.sleep(1.0)
        a.stop()
        time.sleep(1.3)
        a.start()
        time.sleep(1.0)
        c.close_sync(10)
        assert 'connect' not in rec.events
        assert a.accepted + b.accepted >= 2
    finally:
        a.stop()
        b.stop()
        a.shutdown()


def test_failed_then_recovers_when_server_appears(zk):
    port = zk.port
    zk.stop()
    c = client([{'address': '127.0.0.1', 'port': port}])
    rec = Recorder(c)
    rec.wait('failed', timeout=20)
    zk.start()                    # cueball keeps retrying in monitor mode
    rec.wait('connect', timeout=20)
    assert c.call_sync('ping') is None
    c.close_sync(10)
    assert rec.events[:3] == ['failed', 'session', 'connect']
