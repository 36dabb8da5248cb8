"""Random ZooKeeper packets for codec parity tests and synthetic streams."""

import random

from .. import jute

_REQ_OPS = ['GET_DATA', 'EXISTS', 'GET_CHILDREN', 'GET_CHILDREN2', 'CREATE',
            'DELETE', 'SET_DATA', 'GET_ACL', 'SYNC', 'PING', 'CLOSE_SESSION']


def rand_path(rng, maxdepth=4):
    d = rng.randint(1, maxdepth)
    return ''.join('/' + ''.join(rng.choice('abcdefghij0123456789_-')
                                 for _ in range(rng.randint(1, 12)))
                   for _ in range(d))


def rand_bytes(rng, maxlen):
    n = rng.choice([0, 1, rng.randint(0, maxlen)])
    return bytes(rng.getrandbits(8) for _ in range(n))


def rand_acl(rng):
    acl = []
    for _ in range(rng.randint(0, 2)):
        perms = [p for p in ('read', 'write', 'create', 'delete', 'admin')
                 if rng.random() < 0.6] or ['read']
        acl.append({'perms': perms,
                    'id': {'scheme': rng.choice(['world', 'digest', 'ip']),
                           'id': rng.choice(['anyone', 'u:x', '10.0.0.1'])}})
    return acl


def rand_request(rng, xid, maxdata=64):
    op = rng.choice(_REQ_OPS)
    p = {'xid': xid, 'opcode': op}
    if op in ('PING', 'CLOSE_SESSION'):
        return p
    p['path'] = rand_path(rng)
    if op in ('GET_DATA', 'EXISTS', 'GET_CHILDREN', 'GET_CHILDREN2'):
        p['watch'] = rng.random() < 0.5
    elif op == 'CREATE':
        p['data'] = rand_bytes(rng, maxdata)
        p['acl'] = rand_acl(rng)
        p['flags'] = [f for f in ('EPHEMERAL', 'SEQUENTIAL')
                      if rng.random() < 0.4]
    elif op == 'DELETE':
        p['version'] = rng.randint(-1, 10)
    elif op == 'SET_DATA':
        p['data'] = rand_bytes(rng, maxdata)
        p['version'] = rng.randint(-1, 10)
    return p


def rand_stat(rng):
    r = lambda: rng.randint(-2**40, 2**40)  # noqa: E731
    i = lambda: rng.randint(-2**20, 2**20)  # noqa: E731
    return jute.Stat(r(), r(), r(), r(), i(), i(), i(), r(), i(), i(), r())


_REPLY_OPS = ['GET_DATA', 'EXISTS', 'SET_DATA', 'CREATE', 'GET_CHILDREN',
              'GET_CHILDREN2', 'GET_ACL', 'DELETE', 'SYNC']


def rand_reply(rng, xid, maxdata=64):
    """Returns (reply_dict_for_encode, opcode_for_xid_map)."""
    op = rng.choice(_REPLY_OPS)
    rep = {'xid': xid, 'zxid': rng.randint(0, 2**48), 'opcode': op,
           'err': 'OK' if rng.random() < 0.85 else rng.choice(
               ['NO_NODE', 'NODE_EXISTS', 'BAD_VERSION'])}
    if op == 'GET_DATA':
        rep['data'] = rand_bytes(rng, maxdata)
        rep['stat'] = rand_stat(rng)
    elif op in ('EXISTS', 'SET_DATA'):
        rep['stat'] = rand_stat(rng)
    elif op == 'CREATE':
        rep['path'] = rand_path(rng)
    elif op in ('GET_CHILDREN', 'GET_CHILDREN2'):
        rep['children'] = [rand_path(rng, 1)[1:]
                           for _ in range(rng.randint(0, 5))]
        rep['stat'] = rand_stat(rng)
    elif op == 'GET_ACL':
        rep['acl'] = [{'perms': ['READ', 'ADMIN'],
                       'id': {'scheme': 'world', 'id': 'anyone'}}]
        rep['stat'] = rand_stat(rng)
    return rep


def rand_notification(rng):
    return {'xid': -1, 'zxid': -1, 'err': 'OK', 'opcode': 'NOTIFICATION',
            'type': rng.choice(['CREATED', 'DELETED', 'DATA_CHANGED',
                                'CHILDREN_CHANGED']),
            'state': 'SYNC_CONNECTED', 'path': rand_path(rng)}


def rng(seed=0):
    return random.Random(seed)
