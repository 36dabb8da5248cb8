"""Device prefix scan (csrc/kernels/scan.hip): both engines — the MFMA
byte-plane scan and the shuffle scan — against a plain torch int64 cumsum.
Sizes cover one wave, partial segments, one block, the multi-level
recursion; value ranges cover 1-4 byte planes and the >32-bit fallback."""

import pytest
import torch

from zkmi.ops import _lib

pytestmark = pytest.mark.gpu


@pytest.fixture(params=[_lib.SCAN_MFMA_W1, _lib.SCAN_MFMA_W4,
                        _lib.SCAN_MFMA_FORCE, _lib.SCAN_SHFL],
                ids=['mfma_w1', 'mfma_w4', 'mfma_force', 'shfl'])
def mode(request, gpu):
    old = _lib.set_scan_mode(request.param)
    yield request.param
    _lib.set_scan_mode(old)


def _ref(x):
    x64 = x.to(torch.int64).cpu()
    inc = torch.cumsum(x64, 0)
    return inc - x64, int(inc[-1]) if len(x64) else 0


@pytest.mark.parametrize('n', [1, 63, 64, 1000, 1024, 1025, 4095, 4096,
                               4097, 65537, 1 << 20, 4096 * 4096 + 3])
@pytest.mark.parametrize('hi', [200, 60000, 1 << 20, (1 << 31) - 1])
def test_scan_i32(mode, gpu, n, hi):
    from zkmi.ops import batch as B
    if n > (1 << 20) and hi != 60000:
        pytest.skip('one large case is enough')
    g = torch.Generator().manual_seed(n ^ hi)
    x = torch.randint(0, hi, (n,), generator=g, dtype=torch.int32)
    base, total = B.exclusive_scan(x.to(gpu))
    ref, tot = _ref(x)
    assert torch.equal(base.cpu(), ref)
    assert int(total.item()) == tot


@pytest.mark.parametrize('n', [5, 4096 * 3 + 17, 300000])
def test_scan_i64_wide_and_negative(mode, gpu, n):
    """Waves holding values >= 2^32 or < 0 take the lane-serial path; the
    rest of the grid stays on MFMA.  The mix must still be exact."""
    from zkmi.ops import batch as B
    g = torch.Generator().manual_seed(n)
    x = torch.randint(0, 1 << 16, (n,), generator=g, dtype=torch.int64)
    x[::5000] = (1 << 40) + 7
    x[3::7001] = -12345
    base, total = B.exclusive_scan(x.to(gpu))
    ref, tot = _ref(x)
    assert torch.equal(base.cpu(), ref)
    assert int(total.item()) == tot


def test_scan_zero_and_sparse(mode, gpu):
    from zkmi.ops import batch as B
    x = torch.zeros(70000, dtype=torch.int32)
    x[12345] = 255
    x[12346] = 256
    x[69999] = (1 << 24) + 1
    base, total = B.exclusive_scan(x.to(gpu))
    ref, tot = _ref(x)
    assert torch.equal(base.cpu(), ref)
    assert int(total.item()) == tot


@pytest.mark.parametrize('n', [2048, 16384, 65536])
def test_scan_mfma_forced_small(gpu, n):
    """The multi-block MFMA path forced below the one-workgroup threshold
    (round 5's crash: the host recursed on one block forever): block
    levels down to one block, each scanned on MFMA."""
    from zkmi.ops import batch as B
    old = _lib.set_scan_mode(_lib.SCAN_MFMA_FORCE)
    try:
        g = torch.Generator().manual_seed(n)
        x = torch.randint(0, 50000, (n,), generator=g, dtype=torch.int64)
        base, total = B.exclusive_scan(x.to(gpu))
        ref, tot = _ref(x)
        assert torch.equal(base.cpu(), ref)
        assert int(total.item()) == tot
    finally:
        _lib.set_scan_mode(old)


@pytest.mark.parametrize('mfma', [True, False], ids=['mfma', 'shfl'])
@pytest.mark.parametrize('n', [1, 100, 2048, 2049, 4096, 16384, 65541])
def test_scan_small_one_workgroup(gpu, n, mfma):
    """The one-workgroup scan of the encoders' block sums (K10 / K13: 2048
    of them per 512K-record connection of the GET step) on the MFMA
    byte-plane engine and on the shuffle engine, against torch.cumsum;
    values of 1-3 byte planes plus a few past 2^32 (the lane-serial path
    of their wave)."""
    L = _lib.lib()
    g = torch.Generator().manual_seed(n + mfma)
    x = torch.randint(0, 60000, (n,), generator=g, dtype=torch.int64)
    if n > 1000:
        x[777] = (1 << 33) + 5
    xd = x.to(gpu)
    base = torch.empty(n, dtype=torch.int64, device=gpu)
    total = torch.empty(1, dtype=torch.int64, device=gpu)
    L.scan_small(xd, base, total, mfma)
    ref, tot = _ref(x)
    assert torch.equal(base.cpu(), ref)
    assert int(total.item()) == tot
