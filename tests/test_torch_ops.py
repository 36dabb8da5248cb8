"""torch.ops.zkmi (csrc/torch/zkmi_ops.cpp): the HIP codec registered as a
PyTorch operator library.  The ops check every tensor before a pointer
reaches a kernel: wrong dtype, wrong device, non-contiguous or too-short
tensors raise instead of corrupting memory.  The CPU cases run here (the
checks fire before any HIP call); the GPU cases on an MI355X."""

import pytest
import torch

from zkmi.ops import _lib

pytestmark = pytest.mark.skipif(not _lib.available(),
                                reason='operator library not built')

OPS = ('scan_excl', 'encode_requests', 'encode_set_watches',
       'encode_connect_requests', 'encode_responses', 'frame_scan',
       'decode_replies', 'expand_strings', 'expand_acl', 'decode_requests',
       'decode_connect_responses', 'tree_fill', 'tree_build', 'tree_serve',
       'tree_expire', 'bench_gen_get', 'bench_check_get',
       'bench_check_notif', 'route_requests', 'session_connect',
       'session_close')


def test_ops_registered_with_schemas():
    ops = _lib.lib()
    for name in OPS:
        schema = str(getattr(ops, name).default._schema)
        assert schema.startswith('zkmi::' + name + '('), schema
    # outputs are declared mutable
    assert 'Tensor(a!)[] out' in str(ops.decode_replies.default._schema)


def _frame_args(dev, foff_dtype=torch.int64, buf=None):
    buf = torch.zeros(64, dtype=torch.uint8, device=dev) if buf is None \
        else buf
    ws = torch.empty(_lib.lib().frame_scan_workspace(64), dtype=torch.uint8,
                     device=dev)
    return (buf, None, 64, 1 << 24, ws,
            torch.empty(16, dtype=foff_dtype, device=dev),
            torch.empty(16, dtype=torch.int32, device=dev),
            torch.empty(4, dtype=torch.int64, device=dev), 256)


def test_host_tensors_rejected_on_cpu():
    """Host tensors never reach a kernel (on a GPU-less host the op fails
    either on the tensor check or on the HIP stream lookup)."""
    ops = _lib.lib()
    with pytest.raises(RuntimeError):
        ops.frame_scan(*_frame_args('cpu'))
    with pytest.raises(RuntimeError):
        ops.scan_excl(torch.zeros(4, dtype=torch.int32),
                      torch.zeros(4, dtype=torch.int64),
                      torch.zeros(1, dtype=torch.int64),
                      torch.zeros(64, dtype=torch.int64))


@pytest.mark.gpu
def test_bad_tensors_raise_on_gpu(gpu):
    ops = _lib.lib()
    # wrong dtype of the frame offsets
    with pytest.raises(RuntimeError, match='frame_off must be Long'):
        ops.frame_scan(*_frame_args(gpu, foff_dtype=torch.int32))
    # a length past the buffer
    a = list(_frame_args(gpu))
    a[2] = 65
    with pytest.raises(RuntimeError, match='past the buffer'):
        ops.frame_scan(*a)
    # non-contiguous input
    a = list(_frame_args(gpu, buf=torch.zeros(128, dtype=torch.uint8,
                                              device=gpu)[::2]))
    with pytest.raises(RuntimeError, match='contiguous'):
        ops.frame_scan(*a)
    # a reply table too short for the frame table
    from zkmi.ops import batch as B
    buf = torch.zeros(64, dtype=torch.uint8, device=gpu)
    ft = B.frame_scan(buf, 64, cap=16)
    xt = B.XidTable(bits=10, device=gpu)
    short = B.alloc_replies(8, gpu)
    with pytest.raises(RuntimeError, match='needs 16'):
        ops.decode_replies(buf, ft.off, ft.length, ft.count, xt.tab, xt.mask,
                           short.tensors())
    # the xid table smaller than its mask says
    with pytest.raises(RuntimeError, match='xid_tab'):
        ops.decode_replies(buf, ft.off, ft.length, ft.count, xt.tab[:100],
                           xt.mask, B.alloc_replies(16, gpu).tensors())
    # an int64 request-batch field where int32 is expected
    rb = B.pack_requests([{'xid': 1, 'opcode': 'PING'}], gpu)
    rb.xid = rb.xid.to(torch.int64)
    with pytest.raises(RuntimeError, match='batch.xid must be Int'):
        B.encode_requests(rb)


@pytest.mark.gpu
def test_ops_run_on_the_current_stream(gpu):
    """A scan issued under ``torch.cuda.stream(s)`` is ordered on ``s``."""
    from zkmi.ops import batch as B
    s = torch.cuda.Stream(gpu)
    x = torch.arange(1 << 20, dtype=torch.int64, device=gpu)
    with torch.cuda.stream(s):
        base, total = B.exclusive_scan(x)
    s.synchronize()
    n = 1 << 20
    assert int(total.item()) == n * (n - 1) // 2
    assert int(base[-1].item()) == (n - 1) * (n - 2) // 2
