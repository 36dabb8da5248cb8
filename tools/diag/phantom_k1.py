"""Diagnostic: K1 on create replies with a phantom-chain region (zxids
0x2Exxxx, see tests/test_frame_repair.py), scanned a few times; run under
rocprofv3 --kernel-trace for the per-kernel split."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..',
                                'tests'))
from test_frame_repair import _create_replies  # noqa: E402
from zkmi.ops import batch as B  # noqa: E402

dev = torch.device('cuda', 0)
n = 1 << 20
for tag, z0 in (('clean', 0x500000), ('phantom', 0x2E0000 - 500000)):
    buf, starts = _create_replies(n, zxid0=z0)
    d = torch.from_numpy(buf).to(dev)
    sc = B.FrameScanner(n + 16, dev, window=256)
    for k in range(4):
        t0 = time.perf_counter()
        ft = sc.scan(d, len(buf))
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        print(tag, k, 'ms %.3f' % ms, ft.host_result(), sc.chain_stats(),
              flush=True)

# ZKMI_FS_DBG=1: fs_link's phase clock of the last scan (100 MHz ticks)
if os.environ.get('ZKMI_FS_DBG'):
    from zkmi.ops import _lib
    tiles = (len(buf) + 4095) // 4096
    row = _lib.lib().frame_scan_dbg(tiles + 1).numpy()[tiles]
    names = ['chases', 'barrier', 'link check', 'finish']
    print('fs_link phases us:', {nm: (int(row[i + 1]) - int(row[i])) / 100.0
                                 for i, nm in enumerate(names)},
          'exact chase starts at +%.1f us, takes %.1f us' % (
              (int(row[6]) - int(row[0])) / 100.0,
              (int(row[7]) - int(row[6])) / 100.0))
