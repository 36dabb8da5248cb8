"""Property / fuzz tests of the host codec (zkmi.codec: the native C++
extension when built, else the oracle) against the pure-Python Jute oracle.
Arbitrary bytes must never crash the decoder, and wherever the oracle
decodes, the native codec must produce the identical packet; wherever the
oracle rejects, it must reject too.  tools/sanitize_host.sh runs these under
ASan/UBSan."""

from hypothesis import given, settings, strategies as st, HealthCheck

from zkmi import codec, consts, jute
from zkmi.errors import ZKDecodeError

OPS = [op for op in ('GET_DATA', 'EXISTS', 'SET_DATA', 'CREATE', 'DELETE',
                     'GET_CHILDREN', 'GET_CHILDREN2', 'GET_ACL', 'SYNC',
                     'PING', 'SET_WATCHES', 'CLOSE_SESSION')]
REJECT = (ZKDecodeError, ValueError, KeyError, UnicodeDecodeError,
          IndexError, OverflowError)

SETTINGS = settings(max_examples=400, deadline=None,
                    suppress_health_check=[HealthCheck.too_slow])


def _outcome(fn, *a):
    try:
        return ('ok', fn(*a))
    except REJECT as e:
        return ('err', type(e).__name__)


@SETTINGS
@given(body=st.binary(min_size=0, max_size=200),
       op=st.sampled_from(OPS), xid=st.integers(0, 5))
def test_decode_response_arbitrary_bytes(body, op, xid):
    xmap = {xid: op}
    # put the xid in front most of the time so the body reaches the
    # per-opcode decoders
    data = xid.to_bytes(4, 'big') + body[4:] if len(body) >= 4 else body
    a = _outcome(codec.decode_response, data, xmap)
    b = _outcome(jute.decode_response, data, xmap)
    assert a[0] == b[0], (a, b)
    if a[0] == 'ok':
        assert a[1] == b[1]


@SETTINGS
@given(data=st.binary(min_size=0, max_size=300),
       maxp=st.sampled_from([16, 64, consts.MAX_PACKET]))
def test_scan_frames_arbitrary_bytes(data, maxp):
    assert codec.scan_frames(data, 0, len(data), maxp) == \
        jute.scan_frames(data, 0, len(data), maxp)


path_st = st.text(alphabet=st.characters(min_codepoint=32,
                                         max_codepoint=0x2FF),
                  min_size=1, max_size=40).map(lambda s: '/' + s)


@SETTINGS
@given(xid=st.integers(0, 2**31 - 1), path=path_st,
       data=st.binary(max_size=100), version=st.integers(-1, 2**31 - 1),
       op=st.sampled_from(['GET_DATA', 'EXISTS', 'SET_DATA', 'DELETE',
                           'CREATE', 'GET_CHILDREN2', 'SYNC', 'GET_ACL']),
       flags=st.lists(st.sampled_from(['EPHEMERAL', 'SEQUENTIAL']),
                      unique=True),
       watch=st.booleans())
def test_encode_request_parity(xid, path, data, version, op, flags, watch):
    p = {'xid': xid, 'opcode': op, 'path': path, 'data': data,
         'version': version, 'flags': flags, 'watch': watch,
         'acl': jute.DEFAULT_ACL}
    assert codec.encode_request(dict(p)) == jute.encode_request(p)
    # and the oracle's server-side decoder reads it back
    back = jute.decode_request(jute.encode_request(p))
    assert back['xid'] == xid and back['opcode'] == op
