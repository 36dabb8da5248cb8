"""Persistent doorbell codec (csrc/kernels/doorbell.hip via
zkmi/ops/doorbell.py) against the Jute oracle: request encode and reply
decode byte/record parity, lifecycle (stop, deadline).  Needs an MI355X."""

import time

import pytest

from zkmi import jute
from zkmi.utils import synth

pytestmark = pytest.mark.gpu

ENC_OPS = ('GET_DATA', 'EXISTS', 'GET_CHILDREN', 'GET_CHILDREN2', 'GET_ACL',
           'SYNC', 'DELETE', 'PING', 'CLOSE_SESSION')
DEC_OPS = ('GET_DATA', 'EXISTS', 'SET_DATA', 'DELETE', 'SYNC')


def test_doorbell_encode_parity(gpu):
    from zkmi.ops.doorbell import DoorbellCodec
    r = synth.rng(11)
    with DoorbellCodec(max_seconds=30) as db:
        n = 0
        for xid in range(4000):
            p = synth.rand_request(r, xid)
            if p['opcode'] not in ENC_OPS:
                continue
            assert db.encode_request(p) == jute.frame(jute.encode_request(p))
            n += 1
        assert db.served == n


def test_doorbell_decode_parity(gpu):
    from zkmi.ops.doorbell import DoorbellCodec
    r = synth.rng(12)
    with DoorbellCodec(max_seconds=30) as db:
        for xid in range(3000):
            rep = synth.rand_reply(r, xid, maxdata=300)
            if rep['opcode'] not in DEC_OPS:
                continue
            body = jute.encode_response(rep)
            want = jute.decode_response(body, {xid: rep['opcode']})
            assert db.decode_response(body, rep['opcode']) == want


def test_doorbell_rejects_and_stops(gpu):
    from zkmi.ops.doorbell import DoorbellCodec
    with DoorbellCodec(max_seconds=30) as db:
        with pytest.raises(ValueError):          # not a doorbell opcode
            db.encode_request({'xid': 1, 'opcode': 'CREATE', 'path': '/a',
                               'data': b'', 'acl': [], 'flags': []})
        with pytest.raises(ValueError):          # body left to the host
            db.decode_response(jute.encode_response(
                {'xid': 2, 'zxid': 1, 'err': 'OK', 'opcode': 'CREATE',
                 'path': '/a'}), 'CREATE')
        # the ring keeps working after rejected records
        p = {'xid': 3, 'opcode': 'PING'}
        assert db.encode_request(p) == jute.frame(jute.encode_request(p))
    # the in-kernel deadline ends an idle wave on its own
    db = DoorbellCodec(max_seconds=0.5)
    time.sleep(1.0)
    with pytest.raises(RuntimeError):
        db.encode_request({'xid': 4, 'opcode': 'PING'})
    db.close()
