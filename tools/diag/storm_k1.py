"""Diagnostic: the reply stream of the storm workload's FIRST step (the
one whose link repair ran long) — K1 chain statistics, the repair time,
and a prefix of the stream saved for offline analysis."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
from zkmi.bench import synthetic as S  # noqa: E402
from zkmi.ops import batch as B  # noqa: E402

dev = torch.device('cuda', 0)
batch = 1 << 20
tree = S.GpuTree(1_000_000, 100, device=dev, seed=0,
                 spare=(batch * 3 + 8192) / 1e6 + 0.05)
t0 = time.perf_counter()
pipe = S.StormPipeline(tree, batch, seed=0)
torch.cuda.synchronize()
print('init s', round(time.perf_counter() - t0, 3))
d = pipe.drv
# chain counters of the scans run so far (create_dirs + the first step)
print('reply scanner', d.rscanner.chain_stats(), 'request scanner',
      d.server.scanner.chain_stats(), flush=True)
def rescan(out, n, sc, tag):
    if hasattr(sc, 'last_cap'):
        sc.chain_stats()
    t0 = time.perf_counter()
    ft = sc.scan(out, n)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) * 1e3
    print(tag, 'scan ms', round(el, 3), ft.host_result(), sc.chain_stats(),
          flush=True)


for k in range(3):
    pipe.step(validate=False)
    torch.cuda.synchronize()
    print('step', k, 'reply scanner', d.rscanner.chain_stats(),
          'request scanner', d.server.scanner.chain_stats(), flush=True)
    out, total, _, _ = d.server.result
    n = int(total.item())
    if k == 0:
        keep = out[:n].clone()
        np.savez_compressed('gpurun_out/storm_step0_reply.npz',
                            raw=keep.cpu().numpy())
        # the same stream again: the pipeline's own scanner (reused
        # workspace), a fresh one, and the pipeline's scanner once more
        rescan(out, n, d.rscanner, 'step0 again, pipeline scanner')
        rescan(keep, n, B.FrameScanner(batch + 16, dev, window=d.rwindow),
               'step0 copy, fresh scanner')
        rescan(out, n, d.rscanner, 'step0 third, pipeline scanner')
        print('pipeline scanner window', d.rwindow, 'cap', d.rscanner.cap,
              'ws_for', d.rscanner.ws_for, 'buf numel', out.numel(),
              flush=True)
rb, rep = pipe.last
# re-scan the reply stream of that first step from the server's buffer
out, total, _, _ = d.server.result
n = int(total.item())
print('reply stream bytes', n, 'frames', int(rep.count.item()), flush=True)
for nospec in (False, True):
    sc = B.FrameScanner(batch + 16, dev, window=d.rwindow)
    sc.scan(out, n, nospec=nospec)
    torch.cuda.synchronize()
    sc.chain_stats()
    t0 = time.perf_counter()
    ft = sc.scan(out, n, nospec=nospec)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) * 1e3
    print('nospec', nospec, 'window', d.rwindow, 'scan ms', round(el, 3),
          ft.host_result(), sc.chain_stats(), flush=True)
raw = out[:min(n, 8 << 20)].cpu().numpy()
os.makedirs('gpurun_out', exist_ok=True)
np.save('gpurun_out/storm_first_reply.npy', raw)
ft = d.rscanner.table
off = ft.off[:200].cpu().numpy()
print('first frame bodies', off[:10].tolist(),
      'lens', ft.length[:10].cpu().tolist())
print(bytes(raw[:160]).hex())
