"""Diagnostic: the 0-1024 B GET pipeline at a K1 window below its largest
frame (ZKMI_FS_WINDOW_MAX), every reply stream's frame table checked
against a host framing of the same bytes; the first mismatch is reported
with its tile and the scanner's chain statistics."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
from zkmi.bench import synthetic as S  # noqa: E402

dev = torch.device('cuda', 0)
batch = 1 << 19
tree = S.GpuTree(1_000_000, 100, device=dev, seed=0, data_dist=(0, 1024))
pipe = S.GetPipeline(tree, batch, seed=1)
print('reply window', pipe.rwindow, flush=True)
for step in range(int(os.environ.get('STEPS', '12'))):
    acc = pipe.step()
    torch.cuda.synchronize()
    ok = int(acc.item())
    st = pipe.rscanner.chain_stats()
    idx, rep, rx, ft = pipe.last
    r = ft.host_result()
    n = int(r['consumed'])
    raw = rx[:n].cpu().numpy()
    # host framing (vectorised hops are not possible: walk in python)
    b = raw.tobytes()
    offs = []
    p = 0
    while p + 4 <= n:
        ln = int.from_bytes(b[p:p + 4], 'big')
        offs.append(p + 4)
        p += 4 + ln
    offs = np.asarray(offs, np.int64)
    got = ft.off[:r['frames']].cpu().numpy()
    same = len(got) == len(offs) and np.array_equal(got, offs)
    print('step', step, 'ok', ok, 'of', batch, 'frames', r['frames'],
          len(offs), 'same', same, st, flush=True)
    if not same:
        m = min(len(got), len(offs))
        bad = np.nonzero(got[:m] != offs[:m])[0]
        i0 = int(bad[0]) if len(bad) else m
        print('first mismatch frame', i0, 'got', got[i0:i0 + 3],
              'want', offs[i0:i0 + 3], 'tile', offs[i0] // 4096,
              'n bad', len(bad), flush=True)
        if os.environ.get('SAVE'):
            np.savez_compressed('gpurun_out/var_k1_bad.npz', raw=raw,
                                got=got, want=offs)
        sys.exit(1)
