"""Golden wire vectors and the reference's packet capture
(test/streams.test.js:21-82) against the Jute codec, plus framing edge cases.
Every byte string here was produced by the reference's own ZKBuffer."""

import base64
import binascii

import pytest

from zkmi import consts, jute
from zkmi import codec
from zkmi.errors import ZKDecodeError
from zkmi.streams import ZKDecoder, ZKEncoder


def h(s):
    return binascii.unhexlify(s.replace(' ', '').replace('\n', ''))


WORLD_ALL = [{'id': {'scheme': 'world', 'id': 'anyone'},
              'perms': ['read', 'write', 'create', 'delete', 'admin']}]

GOLDEN = [
    ({'xid': -2, 'opcode': 'PING'}, '00000008 fffffffe 0000000b'),
    ({'xid': 7, 'opcode': 'CLOSE_SESSION'}, '00000008 00000007 fffffff5'),
    ({'xid': 3, 'opcode': 'GET_DATA', 'path': '/foo', 'watch': True},
     '00000011 00000003 00000004 00000004 2f666f6f 01'),
    ({'xid': 4, 'opcode': 'EXISTS', 'path': '/foo', 'watch': False},
     '00000011 00000004 00000003 00000004 2f666f6f 00'),
    ({'xid': 5, 'opcode': 'CREATE', 'path': '/a', 'data': b'hi',
      'acl': WORLD_ALL, 'flags': ['EPHEMERAL', 'SEQUENTIAL']},
     '00000033 00000005 00000001 00000002 2f61 00000002 6869 00000001 '
     '0000001f 00000005 776f726c64 00000006 616e796f6e65 00000003'),
    ({'xid': 6, 'opcode': 'CREATE', 'path': '/a', 'data': b'', 'acl': [],
      'flags': []},
     '0000001a 00000006 00000001 00000002 2f61 ffffffff 00000000 00000000'),
    ({'xid': 8, 'opcode': 'SET_DATA', 'path': '/a', 'data': b'x',
      'version': -1},
     '00000017 00000008 00000005 00000002 2f61 00000001 78 ffffffff'),
    ({'xid': 9, 'opcode': 'DELETE', 'path': '/a', 'version': 0},
     '00000012 00000009 00000002 00000002 2f61 00000000'),
    ({'xid': 10, 'opcode': 'SYNC', 'path': '/a'},
     '0000000e 0000000a 00000009 00000002 2f61'),
    ({'xid': 11, 'opcode': 'GET_ACL', 'path': '/a'},
     '0000000e 0000000b 00000006 00000002 2f61'),
    ({'xid': -8, 'opcode': 'SET_WATCHES', 'relZxid': 0x517,
      'events': {'dataChanged': ['/d'], 'createdOrDestroyed': ['/e'],
                 'childrenChanged': ['/c']}},
     '0000002e fffffff8 00000065 0000000000000517 00000001 00000002 2f64 '
     '00000001 00000002 2f65 00000001 00000002 2f63'),
]


@pytest.mark.parametrize('impl', ['python', 'active'])
@pytest.mark.parametrize('pkt,hexs', GOLDEN)
def test_request_golden(pkt, hexs, impl):
    enc = jute.encode_request if impl == 'python' else codec.encode_request
    fr = jute.frame if impl == 'python' else codec.frame
    assert fr(enc(dict(pkt))) == h(hexs)
    # server-mode decode round-trips (readRequest, zk-buffer.js:58-95)
    back = jute.decode_request(h(hexs)[4:])
    assert back['xid'] == pkt['xid'] and back['opcode'] == pkt['opcode']
    if 'path' in pkt:
        assert back['path'] == pkt['path']


def test_connect_request_golden():
    got = jute.frame(jute.encode_connect_request(
        {'protocolVersion': 0, 'lastZxidSeen': 0, 'timeOut': 30000,
         'sessionId': 0, 'passwd': b'\0' * 8}))
    assert got == h('00000024 00000000 0000000000000000 00007530 '
                    '0000000000000000 00000008 0000000000000000')


# test/streams.test.js:21-27 — a captured `zkCli ls /` exchange.
CAPTURE1 = [
    ('send', 'AAAALQAAAAAAAAAAAAAAAAAAdTAAAAAAAAAAAAAAABAAAAAAAAAAAAAAAAAA'
             'AAAAAA=='),
    ('recv', 'AAAAJQAAAAAAAHUwAVWjqFbbAAAAAAAQh19uvwgo25o9B6hUkSvqKQA='),
    ('send', 'AAAADgAAAAEAAAAIAAAAAS8A'),
    ('recv', 'AAAAKAAAAAEAAAAAAAAFFwAAAAAAAAACAAAACXpvb2tlZXBlcgAAAANmb28='),
]


@pytest.mark.parametrize('impl', ['python', 'active'])
def test_decode_capture1(impl):
    dec_resp = jute.decode_response if impl == 'python' else \
        codec.decode_response
    bufs = [base64.b64decode(d) for _, d in CAPTURE1]
    for b in bufs:
        (n,) = __import__('struct').unpack('>i', b[:4])
        assert n == len(b) - 4
    cr = jute.decode_connect_request(bufs[0][4:])
    assert cr == {'protocolVersion': 0, 'lastZxidSeen': 0, 'timeOut': 30000,
                  'sessionId': 0, 'passwd': b'\0' * 16}
    cresp = jute.decode_connect_response(bufs[1][4:])
    assert cresp['protocolVersion'] == 0 and cresp['timeOut'] == 30000
    assert cresp['sessionId'] == int.from_bytes(
        base64.b64decode('AVWjqFbbAAA='), 'big')
    assert cresp['passwd'] == base64.b64decode('h19uvwgo25o9B6hUkSvqKQ==')
    req = jute.decode_request(bufs[2][4:])
    assert req == {'xid': 1, 'opcode': 'GET_CHILDREN', 'path': '/',
                   'watch': False}
    rep = dec_resp(bufs[3][4:], {1: 'GET_CHILDREN'})
    assert rep == {'xid': 1, 'opcode': 'GET_CHILDREN', 'err': 'OK',
                   'zxid': 0x517, 'children': ['zookeeper', 'foo']}


@pytest.mark.parametrize('impl', ['python', 'active'])
def test_decoded_examples(impl):
    dec_resp = jute.decode_response if impl == 'python' else \
        codec.decode_response
    n = dec_resp(h('ffffffff ffffffffffffffff 00000000 00000003 00000003 '
                   '00000004 2f666f6f'), {})
    assert n == {'xid': -1, 'zxid': -1, 'err': 'OK', 'opcode':
                 'NOTIFICATION', 'type': 'DATA_CHANGED',
                 'state': 'SYNC_CONNECTED', 'path': '/foo'}
    e = dec_resp(h('00000005 0000000000000520 ffffff92'), {5: 'CREATE'})
    assert e == {'xid': 5, 'zxid': 0x520, 'err': 'NODE_EXISTS',
                 'opcode': 'CREATE'}


def test_reply_must_match_request():
    with pytest.raises(ZKDecodeError):
        jute.decode_response(h('00000009 0000000000000001 00000000'), {})


def test_stat_and_perms_roundtrip():
    st = jute.Stat(1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11)
    assert len(st.to_bytes()) == consts.STAT_SIZE
    assert jute.JuteReader(st.to_bytes()).read_stat() == st
    # readPerms fixed: decode follows the mask bits.
    for mask, names in [(31, ['READ', 'WRITE', 'CREATE', 'DELETE', 'ADMIN']),
                        (1, ['READ']), (2, ['WRITE']), (30, ['WRITE',
                        'CREATE', 'DELETE', 'ADMIN'])]:
        w = jute.JuteWriter()
        w.write_int(mask)
        assert jute.JuteReader(w.getvalue()).read_perms() == names
    assert jute.perms_to_mask(['read', 'ADMIN']) == 17
    with pytest.raises(ValueError):
        jute.perms_to_mask(['bogus'])


def test_empty_buffer_rules():
    w = jute.JuteWriter()
    w.write_buffer(b'')
    assert w.getvalue() == h('ffffffff')           # written as -1
    assert jute.JuteReader(h('fffffffe')).read_buffer() == b''   # neg -> ''
    with pytest.raises(ZKDecodeError):
        jute.JuteReader(h('00000005 6162')).read_buffer()
    with pytest.raises(ZKDecodeError):
        jute.JuteReader(h('02')).read_bool()


def test_decoder_carry_and_chunking():
    frames = [jute.frame(jute.encode_response(
        {'xid': i, 'zxid': i, 'err': 'OK', 'opcode': 'SYNC'}))
        for i in range(50)]
    stream = b''.join(frames)
    d = ZKDecoder()
    got = []
    # byte-at-a-time and odd chunk sizes both work (length split across
    # writes, test/nasty.test.js:124-145)
    i = 0
    sizes = [1, 2, 3, 7, 64, 5]
    k = 0
    while i < len(stream):
        n = sizes[k % len(sizes)]
        k += 1
        bodies, err = d.feed(stream[i:i + n])
        assert err is None
        got += bodies
        i += n
    assert got == [f[4:] for f in frames]
    assert d.pending() == 0


@pytest.mark.parametrize('bad', ['4000', 'fffffffe0102', '7fffffff'])
def test_decoder_bad_length_stalls(bad):
    d = ZKDecoder()
    good = jute.frame(b'abc')
    bodies, err = d.feed(good + h(bad))
    assert bodies == [b'abc'] or bad == '4000'
    if bad == '4000':          # 2 bytes: not a full length yet
        assert err is None
        bodies, err = d.feed(h('4000'))       # 0x40004000 > 16 MiB
    assert err is not None and err.code == 'BAD_LENGTH'
    assert d.dead
    assert d.feed(good) == ([], None)          # stalled, like the reference


def test_encoder_records_xid_map():
    m = {}
    e = ZKEncoder(m)
    e.request({'xid': 12, 'opcode': 'GET_DATA', 'path': '/x',
               'watch': False})
    assert m == {12: 'GET_DATA'}


def test_consts_tables():
    assert consts.OP_CODES['GET_CHILDREN2'] == 12
    assert consts.ERR_LOOKUP[-110] == 'NODE_EXISTS'
    assert consts.STATE['SYNC_CONNECTED'] == 3
    assert consts.SPECIAL_XIDS[-8] == 'SET_WATCHES'
    for k, v in consts.ERR_CODES.items():
        if k != 'OK':
            assert k in consts.ERR_TEXT


def test_kernel_opcode_table_matches():
    """csrc/kernels/zk_common.h mirrors the opcode/xid constants."""
    import os
    import re
    src = open(os.path.join(os.path.dirname(__file__), '..', 'csrc',
                            'kernels', 'zk_common.h')).read()
    for name, val in consts.OP_CODES.items():
        m = re.search(r'OP_%s = (-?\d+)' % name, src)
        assert m is not None and int(m.group(1)) == val, name
    for name, val in [('NOTIFICATION', -1), ('PING', -2),
                      ('SET_WATCHES', -8)]:
        m = re.search(r'XID_%s = (-?\d+)' % name, src)
        assert int(m.group(1)) == val
