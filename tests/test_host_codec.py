"""Native C++ host codec (csrc/host/zk_host_codec.cpp) against the
pure-Python Jute oracle: randomized byte/record parity, error behaviour."""

import os
import random
import sys

import pytest

from zkmi import jute
from zkmi.errors import ZKDecodeError
from zkmi.utils import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope='module')
def native():
    if os.environ.get('ZKMI_HOST_CODEC_PATH'):
        # the sanitizer build (tools/sanitize_host.sh), loaded by zkmi.codec
        from zkmi import codec
        assert codec.IMPL == 'native'
        return codec._zkhost
    sys.path.insert(0, os.path.join(ROOT, 'tools'))
    import build_native
    build_native.build_host()
    from zkmi import _zkhost
    _zkhost.init(jute.Stat, ZKDecodeError)
    return _zkhost


def test_encode_request_parity(native):
    r = synth.rng(3)
    for xid in range(3000):
        p = synth.rand_request(r, xid, maxdata=300)
        assert native.encode_request(dict(p)) == jute.encode_request(p), p
    sw = {'xid': -8, 'opcode': 'SET_WATCHES', 'relZxid': 0x517,
          'events': {'dataChanged': ['/d'], 'createdOrDestroyed': [],
                     'childrenChanged': ['/c', '/x']}}
    assert native.encode_request(sw) == jute.encode_request(sw)


def test_decode_response_parity(native):
    r = synth.rng(4)
    xmap = {}
    for xid in range(3000):
        rep = synth.rand_notification(r) if r.random() < 0.1 else \
            synth.rand_reply(r, xid, maxdata=300)
        if rep['xid'] >= 0:
            xmap[rep['xid']] = rep['opcode']
        body = jute.encode_response(rep)
        a = native.decode_response(body, xmap)
        b = jute.decode_response(body, xmap)
        assert a == b


def test_decode_errors(native):
    with pytest.raises(ZKDecodeError):
        native.decode_response(b'\0' * 8, {})
    with pytest.raises(ZKDecodeError):
        native.decode_response(b'\0\0\0\x05' + b'\0' * 12, {})   # no xid
    # truncated GET_DATA body
    body = jute.encode_response({'xid': 1, 'zxid': 2, 'err': 'OK',
                                 'opcode': 'GET_DATA', 'data': b'abc',
                                 'stat': jute.Stat()})
    with pytest.raises(ZKDecodeError):
        native.decode_response(body[:-5], {1: 'GET_DATA'})
    with pytest.raises(ValueError):
        native.encode_request({'xid': 1, 'opcode': 'CREATE', 'path': '/a',
                               'data': b'', 'acl': [], 'flags': ['NOPE']})


def test_scan_frames_parity(native):
    r = random.Random(9)
    s = b''.join(jute.frame(bytes(r.getrandbits(8) for _ in range(
        r.randint(0, 200)))) for _ in range(300))
    for cut in (len(s), len(s) - 3, len(s) - 50):
        assert native.scan_frames(s, 0, cut, 1 << 24) == \
            jute.scan_frames(s, 0, cut)
    bad = s + b'\xff\xff\xff\xfe\x01'
    assert native.scan_frames(bad, 0, None, 1 << 24) == \
        jute.scan_frames(bad)
    assert native.frame(b'xyz') == jute.frame(b'xyz')


def test_active_codec_is_native_when_built(native):
    import importlib
    import zkmi.codec as C
    importlib.reload(C)
    assert C.IMPL == 'native'
