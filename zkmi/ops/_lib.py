"""The HIP batch codec as PyTorch-ROCm operators: ``torch.ops.zkmi.*``.

``zkmi/ops/libzkmi_torch.so`` (csrc/torch/zkmi_ops.cpp) registers the ops
with ``TORCH_LIBRARY(zkmi, ...)``; the kernels themselves live in
``zkmi/ops/libzkmi_hip.so`` (csrc/kernels/*.hip, gfx950), which the op
library links.  Both are compiled in-tree by ``tools/build_native.py``
(called from ``__graft_entry__.build``).  Every op checks dtype, device,
contiguity and lengths of its tensors before a pointer reaches a kernel,
runs on the current HIP stream and raises on a launch error.

On a machine with a GPU a missing library is an error (:func:`lib`
raises); there is no silent CPU fallback for the batch codec.  So is a
kernel library built from other sources than this tree's
(``zkmi/ops/_srchash.py``): its embedded source hash must match.
"""

import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, 'libzkmi_torch.so')
HIP_LIB_PATH = os.path.join(_HERE, 'libzkmi_hip.so')

# wire-format node slot layout (csrc/kernels/zk_abi.h)
SLOT_STAT = 0
SLOT_LEN = 72
SLOT_DATA = 76

# session handshake outcomes (csrc/kernels/session.hip SC_*)
SC_NEW, SC_RESUMED, SC_EXPIRED, SC_REFUSED, SC_BAD, SC_FULL = range(6)
CR_RESP_BYTES = 41

# ZkTree counters (csrc/kernels/tree.hip TC_*)
TC_NODES, TC_ZXID, TC_PATH_TOP, TC_SLAB_TOP = 0, 1, 2, 3
TC_FREE_HEAD, TC_FREE_TAIL, TC_FREE_PUB, TC_DIRTY = 4, 5, 6, 7
TC_SESS, TC_N = 8, 9
# serve / expire `session` argument: the one in counters[TC_SESS]
SESS_DEV = -2
HT_WORDS = 8     # int64 words per hash entry: key, val, lengths, path head

SCAN_SHFL, SCAN_MFMA, SCAN_MFMA_W1, SCAN_MFMA_W4 = 0, 1, 2, 3
SCAN_MFMA_FORCE = 4      # the multi-block MFMA path at any n (tests)

_ops = None


def lib():
    """Load (once) the operator library and return ``torch.ops.zkmi``."""
    global _ops
    if _ops is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                'zkmi operator library not built: run `python tools/'
                'build_native.py` (or __graft_entry__.build())')
        check_build()
        torch.ops.load_library(LIB_PATH)
        _ops = torch.ops.zkmi
        # the MFMA byte-plane scan engine (csrc/kernels/scan.hip); the
        # shuffle engine stays selectable (scan_set_mode) for the tests
        _ops.scan_set_mode(SCAN_MFMA)
    return _ops


def built_hash():
    """The source hash embedded in ``libzkmi_hip.so`` (None if absent)."""
    try:
        f = ctypes.CDLL(HIP_LIB_PATH).zkmi_hip_src_hash
    except (OSError, AttributeError):
        return None
    f.restype = ctypes.c_char_p
    return f().decode()


def check_build():
    """Raise unless the kernel library was compiled from this tree's kernel
    sources and flags (``ZKMI_ALLOW_STALE_BUILD=1`` skips the check for
    A/B runs that swap libraries on purpose)."""
    from . import _srchash
    if os.environ.get('ZKMI_ALLOW_STALE_BUILD') == '1':
        return
    want, got = _srchash.hip_hash(), built_hash()
    if got != want:
        raise RuntimeError(
            'zkmi/ops/libzkmi_hip.so was built from other sources (hash %s, '
            'tree %s): run `python tools/build_native.py`' % (got, want))


def set_scan_mode(mode):
    """Select the prefix-scan engine used by every encoder; returns the
    previous mode."""
    return lib().scan_set_mode(mode)


def available():
    return os.path.exists(LIB_PATH) and os.path.exists(HIP_LIB_PATH)
