"""Host codec dispatch for the interactive (one-record-at-a-time) path.

Uses the native C++ host codec (``csrc/host/zk_host_codec.cpp``, built
in-tree as ``zkmi/_zkhost*.so``) when present, else the pure-Python oracle in
:mod:`zkmi.jute`.  Both expose identical functions and produce identical
objects; ``tests/test_host_codec.py`` checks byte/record parity.

``ZKMI_HOST_CODEC=python`` forces the oracle (used by the parity tests).
"""

import os

from . import jute

IMPL = 'python'

encode_request = jute.encode_request
decode_response = jute.decode_response
encode_connect_request = jute.encode_connect_request
decode_connect_response = jute.decode_connect_response
decode_connect_request = jute.decode_connect_request
encode_connect_response = jute.encode_connect_response
decode_request = jute.decode_request
encode_response = jute.encode_response
scan_frames = jute.scan_frames
frame = jute.frame
# C entry point of the native reply decoder (a capsule the native loop's
# reply router calls); None without the native codec
DECODE_REPLY_C = None
ENCODE_REQUEST_C = None

def _load_native():
    """The in-tree extension, or the one at ``ZKMI_HOST_CODEC_PATH`` (the
    sanitizer build, tools/sanitize_host.sh)."""
    path = os.environ.get('ZKMI_HOST_CODEC_PATH')
    if path:
        import importlib.util
        spec = importlib.util.spec_from_file_location('_zkhost', path)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        return mod
    try:
        from . import _zkhost as mod  # built by __graft_entry__.build
    except ImportError:
        return None
    return mod


if os.environ.get('ZKMI_HOST_CODEC', 'native') != 'python':
    _zkhost = _load_native()
    if _zkhost is not None:
        from .errors import ZKDecodeError
        _zkhost.init(jute.Stat, ZKDecodeError)
        encode_request = _zkhost.encode_request
        decode_response = _zkhost.decode_response
        scan_frames = _zkhost.scan_frames
        frame = _zkhost.frame
        DECODE_REPLY_C = _zkhost._C_decode_reply
        ENCODE_REQUEST_C = _zkhost._C_encode_request
        IMPL = 'native'
