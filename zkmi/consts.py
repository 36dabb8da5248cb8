"""L0 — ZooKeeper protocol constants.

Parity: ``lib/zk-consts.js:13-138`` of the reference (perm masks, create flags,
error codes + text, opcodes, notification types, keeper states, special xids).
The same numbers are mirrored for native code in ``csrc/kernels/zk_common.h``
(HIP kernels) and ``csrc/host/zk_host_codec.cpp``; ``tests/test_proto.py``
checks the tables agree.
"""

PERM_MASKS = {
    'READ': 1 << 0,
    'WRITE': 1 << 1,
    'CREATE': 1 << 2,
    'DELETE': 1 << 3,
    'ADMIN': 1 << 4,
}
PERM_ALL = 0x1f

CREATE_FLAGS = {
    'EPHEMERAL': 1 << 0,
    'SEQUENTIAL': 1 << 1,
}

ERR_CODES = {
    'OK': 0,
    'SYSTEM_ERROR': -1,
    'RUNTIME_INCONSISTENCY': -2,
    'DATA_INCONSISTENCY': -3,
    'CONNECTION_LOSS': -4,
    'MARSHALLING_ERROR': -5,
    'UNIMPLEMENTED': -6,
    'OPERATION_TIMEOUT': -7,
    'BAD_ARGUMENTS': -8,
    'API_ERROR': -100,
    'NO_NODE': -101,
    'NO_AUTH': -102,
    'BAD_VERSION': -103,
    'NO_CHILDREN_FOR_EPHEMERALS': -108,
    'NODE_EXISTS': -110,
    'NOT_EMPTY': -111,
    'SESSION_EXPIRED': -112,
    'INVALID_CALLBACK': -113,
    'INVALID_ACL': -114,
    'AUTH_FAILED': -115,
}
ERR_LOOKUP = {v: k for k, v in ERR_CODES.items()}

ERR_TEXT = {
    'SYSTEM_ERROR': 'An unknown system error occurred on the ZooKeeper server',
    'RUNTIME_INCONSISTENCY': 'A runtime inconsistency was found, and the '
                             'request aborted for safety',
    'DATA_INCONSISTENCY': 'A data inconsistency was found, and the request '
                          'aborted for safety',
    'CONNECTION_LOSS': 'Connection to the ZooKeeper server has been lost',
    'MARSHALLING_ERROR': 'Error while marshalling or unmarshalling data',
    'UNIMPLEMENTED': 'ZooKeeper request unimplemented',
    'OPERATION_TIMEOUT': 'ZooKeeper operation timed out',
    'BAD_ARGUMENTS': 'Bad arguments to ZooKeeper request',
    'API_ERROR': '',
    'NO_NODE': 'The specified ZooKeeper path does not exist',
    'NO_AUTH': 'Request requires authentication and your ZooKeeper '
               'connection is anonymous',
    'BAD_VERSION': 'A specific version of an object was named in the '
                   'request, but this was not the latest version on the '
                   'server. The object may have been changed by another '
                   'client.',
    'NO_CHILDREN_FOR_EPHEMERALS': 'Ephemeral nodes cannot have children',
    'NODE_EXISTS': 'The specified ZooKeeper path already exists, and the '
                   'requested operation requires creating a new node',
    'NOT_EMPTY': 'The specified ZooKeeper node has children and thus '
                 'cannot be destroyed',
    'SESSION_EXPIRED': 'ZooKeeper session expired',
    'INVALID_CALLBACK': '',
    'INVALID_ACL': 'The given ZooKeeper ACL was found to be invalid on the '
                   'server side',
    'AUTH_FAILED': 'ZooKeeper authentication failed',
}

OP_CODES = {
    'NOTIFICATION': 0,
    'CREATE': 1,
    'DELETE': 2,
    'EXISTS': 3,
    'GET_DATA': 4,
    'SET_DATA': 5,
    'GET_ACL': 6,
    'SET_ACL': 7,
    'GET_CHILDREN': 8,
    'SYNC': 9,
    'PING': 11,
    'GET_CHILDREN2': 12,
    'CHECK': 13,
    'MULTI': 14,
    'AUTH': 100,
    'SET_WATCHES': 101,
    'SASL': 102,
    'CREATE_SESSION': -10,
    'CLOSE_SESSION': -11,
    'ERROR': -1,
}
OP_CODE_LOOKUP = {v: k for k, v in OP_CODES.items()}

NOTIFICATION_TYPE = {
    'CREATED': 1,
    'DELETED': 2,
    'DATA_CHANGED': 3,
    'CHILDREN_CHANGED': 4,
}
NOTIFICATION_TYPE_LOOKUP = {v: k for k, v in NOTIFICATION_TYPE.items()}

STATE = {
    'DISCONNECTED': 0,
    'SYNC_CONNECTED': 3,
    'AUTH_FAILED': 4,
    'CONNECTED_READ_ONLY': 5,
    'SASL_AUTHENTICATED': 6,
    'EXPIRED': -122,
}
STATE_LOOKUP = {v: k for k, v in STATE.items()}

XID_NOTIFICATION = -1
XID_PING = -2
XID_AUTHENTICATION = -4
XID_SET_WATCHES = -8

SPECIAL_XIDS = {
    XID_NOTIFICATION: 'NOTIFICATION',
    XID_PING: 'PING',
    XID_AUTHENTICATION: 'AUTH',
    XID_SET_WATCHES: 'SET_WATCHES',
}

# Framing limit (reference lib/zk-streams.js:23).
MAX_PACKET = 16 * 1024 * 1024

# Size in bytes of a serialized Stat record (Appendix A of SURVEY.md).
STAT_SIZE = 68

DEFAULT_PORT = 2181
DEFAULT_SESSION_TIMEOUT = 30000
