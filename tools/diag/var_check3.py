"""Diagnostic: find a broken reply stream of the variable-size GET
pipeline and show where the host framer and the expected replies differ."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
from zkmi import jute  # noqa: E402
from zkmi.bench import synthetic as S  # noqa: E402


def main():
    dev = torch.device('cuda', 0)
    tree = S.GpuTree(1_000_000, 0, device=dev, data_dist=(0, 1024))
    p = S.GetPipeline(tree, 1 << 18)
    for step in range(6):
        ok = int(p.step().item())
        idx, rep, rx, ft = p.last
        n = p.batch
        if ok == n:
            print('step', step, 'ok', flush=True)
            continue
        r = ft.host_result()
        print('step', step, 'ok', ok, r, flush=True)
        total = int(p.server.last_rec_off[n - 1].item()) + 4 + int(
            rx[int(p.server.last_rec_off[n - 1].item()):][:4].cpu().numpy()
            .view('>i4')[0])
        hb = rx[:total].cpu().numpy().tobytes()
        frames, cons, bad = jute.scan_frames(hb)
        print('host frames', len(frames), 'consumed', cons, 'of', total,
              'bad', bad, flush=True)
        ro = p.server.last_rec_off[:n].cpu().numpy()
        hs = np.array([o - 4 for o, _ in frames[:n]])
        k = np.nonzero(hs[:min(len(hs), n)] != ro[:min(len(hs), n)])[0]
        print('rec_off vs host first diff', k[:3].tolist(), flush=True)
        dl = tree.data_len[idx].cpu().numpy()
        sizes = 4 + 16 + 4 + dl + 68
        exp = np.zeros(n, np.int64)
        np.cumsum(sizes[:-1], out=exp[1:])
        k2 = np.nonzero(exp != ro)[0]
        print('rec_off vs expected sizes first diff', k2[:3].tolist(),
              flush=True)
        # first frame whose length word disagrees with its expected size
        lw = np.array([int.from_bytes(hb[o:o + 4], 'big', signed=True)
                       for o in ro[:n]])
        k3 = np.nonzero(lw != sizes - 4)[0]
        print('length words wrong', len(k3), k3[:5].tolist(), flush=True)
        if len(k3):
            j = int(k3[0])
            print('  record', j, 'off', ro[j], 'len word', lw[j], 'want',
                  sizes[j] - 4, 'dl', dl[j], 'block', j // 256, 'in block',
                  j % 256, flush=True)
            o = int(ro[j])
            print('  bytes', hb[o - 8:o + 24].hex(), flush=True)
        xidw = np.array([int.from_bytes(hb[o + 4:o + 8], 'big', signed=True)
                         for o in ro[:n]])
        want_x = p.xid[:n].cpu().numpy()
        k4 = np.nonzero(xidw != want_x)[0]
        print('xid words wrong', len(k4), k4[:5].tolist(), flush=True)
        break


if __name__ == '__main__':
    main()
