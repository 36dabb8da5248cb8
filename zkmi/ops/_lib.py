"""ctypes binding to ``libzkmi_hip.so`` (csrc/kernels).

The library is compiled in-tree by ``tools/build_native.py`` (called from
``__graft_entry__.build``).  ``torch`` must be imported first so that the
HIP runtime the library links (``libamdhip64.so.7``) resolves to the copy
torch already loaded — one runtime, one set of streams.

On a machine with a GPU a missing or unloadable library is an error
(:func:`lib` raises); there is no silent CPU fallback for the batch codec.
"""

import ctypes
import os

import torch  # noqa: F401  (must precede the HIP library load)

_HERE = os.path.dirname(os.path.abspath(__file__))
# ZKMI_HIP_LIB: an alternative build of the same library (A/B runs)
LIB_PATH = os.environ.get('ZKMI_HIP_LIB') or os.path.join(_HERE,
                                                          'libzkmi_hip.so')

P = ctypes.c_void_p
I64 = ctypes.c_int64
I32 = ctypes.c_int32


class ZkReqBatch(ctypes.Structure):
    _fields_ = [(n, P) for n in (
        'opcode', 'xid', 'arg', 'path_off', 'path_len', 'data_off',
        'data_len', 'acl_id', 'path_arena', 'data_arena', 'acl_off',
        'acl_len', 'acl_arena')]


class ZkNodeStore(ctypes.Structure):
    _fields_ = [('slab', P), ('slot_off', P), ('data_len', P),
                ('slot_cap', P), ('cap', I64)]


# wire-format node slot layout (csrc/kernels/zk_batch.h)
SLOT_STAT = 0
SLOT_LEN = 72
SLOT_DATA = 76


class ZkRespBatch(ctypes.Structure):
    _fields_ = [(n, P) for n in (
        'opcode', 'xid', 'err', 'node', 'zxid', 'path_off', 'path_len',
        'path_arena', 'aux', 'slot')]


class ZkReplyOut(ctypes.Structure):
    _fields_ = [(n, P) for n in (
        'xid', 'err', 'opcode', 'status', 'zxid', 'stat64', 'stat32',
        'pay_off', 'pay_len', 'aux0', 'aux1')] + [('cap', I64)]


class ZkReqOut(ctypes.Structure):
    _fields_ = [(n, P) for n in (
        'xid', 'opcode', 'status', 'path_off', 'path_len', 'data_off',
        'data_len', 'arg', 'vec_off', 'vec_count', 'rel_zxid')] + \
        [('cap', I64)]


class ZkTree(ctypes.Structure):
    _fields_ = [('ht', P), ('mask', I64),
                ('node_path_off', P), ('node_path_len', P),
                ('node_parent', P), ('path_arena', P), ('path_cap', I64),
                ('slab_cap', I64), ('counters', P), ('store', ZkNodeStore),
                ('free_list', P), ('free_cap', I64), ('cver', P),
                ('nchild', P), ('pzxid', P), ('dirty', P), ('dirty_list', P),
                ('node_pw', P)]


class ZkSessionTable(ctypes.Structure):
    _fields_ = [('sid', P), ('passwd', P), ('timeout', P), ('state', P),
                ('next', P), ('cap', I64)]


# session handshake outcomes (csrc/kernels/session.hip SC_*)
SC_NEW, SC_RESUMED, SC_EXPIRED, SC_REFUSED, SC_BAD, SC_FULL = range(6)
CR_RESP_BYTES = 41


# ZkTree counters (csrc/kernels/tree.hip TC_*)
TC_NODES, TC_ZXID, TC_PATH_TOP, TC_SLAB_TOP = 0, 1, 2, 3
TC_FREE_HEAD, TC_FREE_TAIL, TC_FREE_PUB, TC_DIRTY = 4, 5, 6, 7
TC_DONE, TC_N = 8, 9
HT_WORDS = 2     # int64 words per hash entry {key, val}


_SIGS = {
    'zk_scan_workspace': (I64, [I64]),
    'zk_scan_set_mode': (I32, [I32]),
    'zk_scan_excl_i64': (I32, [P, P, I64, P, P, P]),
    'zk_scan_excl_i32': (I32, [P, P, I64, P, P, P]),
    'zk_encode_requests': (I32, [P, I64, P, P, P, P, P, I64, P, I64, P, P]),
    'zk_encode_requests2': (I32, [P, I64, P, P, P, P, P, I64, P, I64, P, I32,
                                  P]),
    'zk_encode_set_watches': (I32, [P, P, P, I64, I64, I64, I64, P, P, P, P,
                                    P, I64, P, P]),
    'zk_encode_responses': (I32, [P, P, P, I64, P, P, P, P, P, I64, P, P]),
    'zk_encode_responses2': (I32, [P, P, P, I64, P, P, P, P, P, I64, P, I32,
                                   I32, P]),
    'zk_frame_scan_workspace': (I64, [I64]),
    'zk_frame_scan': (I32, [P, I64, I64, P, I64, P, P, I64, P, P]),
    'zk_frame_scan2': (I32, [P, I64, I64, P, I64, P, P, I64, P, I32, P]),
    'zk_frame_scan3': (I32, [P, P, I64, I64, P, I64, P, P, I64, P, I32,
                             P]),
    'zk_frame_scan_stats': (I32, [P, I64, I32, P, P]),
    'zk_frame_scan_dbg': (I32, [P, I64]),
    'zk_decode_replies': (I32, [P, P, P, P, I64, P, I64, P, P]),
    'zk_expand_strings': (I32, [P, P, P, P, I64, P, P, P]),
    'zk_expand_acl': (I32, [P, P, P, P, I64, P, P, P, P, P, P]),
    'zk_decode_requests': (I32, [P, P, P, P, I64, P, P]),
    'zk_encode_connect_requests': (I32, [P, P, P, P, P, P, P, I64, P, P, P,
                                         P, P, P]),
    'zk_decode_connect_responses': (I32, [P, P, P, I64, P, P, P, P, P, P,
                                          P]),
    'zk_tree_build': (I32, [P, I64, I64, P]),
    'zk_tree_fill': (I32, [P, I64, I64, P, I64, P]),
    'zk_tree_serve': (I32, [P, P, P, P, I64, P, P, P, P, P, P, P, P, P, P,
                            I64, I64, P]),
    'zk_tree_expire': (I32, [P, I64, I64, P, P]),
    'zk_route_workspace': (I64, [I64, I32]),
    'zk_session_connect': (I32, [P, P, P, P, I64, P, I64, ctypes.c_uint64,
                                 I32, I32, P, P, P, P, P]),
    'zk_session_close': (I32, [P, P, I64, P]),
    'zk_route_requests': (I32, [I64, I32, P, P, P, P, P, P, P, P, P, P, P, P,
                                P]),
    'zk_bench_gen_get': (I32, [I64, ctypes.c_uint64, I64, I64, I32, P, P,
                               P, P, P, P]),
    'zk_bench_check_get': (I32, [I64, P, P, P, P, P, P, P, P, P, P, P]),
    'zk_bench_check_notif': (I32, [I64, I64, P, I64, I64, P, P, P, P, P, P,
                                   P, P, P, P, P, P, P]),
}

_lib = None


def lib():
    """Load (once) and return the HIP kernel library."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                'zkmi HIP library not built: run `python tools/'
                'build_native.py` (or __graft_entry__.build())')
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
        # ZKMI_SCAN=shfl selects the shuffle scan engine instead of the
        # MFMA byte-plane one (csrc/kernels/scan.hip)
        L.zk_scan_set_mode(0 if os.environ.get('ZKMI_SCAN') == 'shfl' else 1)
    return _lib


SCAN_SHFL, SCAN_MFMA, SCAN_MFMA_W1, SCAN_MFMA_W4 = 0, 1, 2, 3


def set_scan_mode(mode):
    """Select the prefix-scan engine used by every encoder; returns the
    previous mode."""
    return lib().zk_scan_set_mode(mode)


def available():
    return os.path.exists(LIB_PATH)


def check(rc, what):
    if rc != 0:
        raise RuntimeError('%s failed (hip error %d)' % (what, rc))


def ptr(t):
    """Device pointer of a tensor (or None)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_ptr(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)
