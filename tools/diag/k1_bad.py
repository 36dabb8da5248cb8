"""Diagnostic: rescan a reply stream K1 got wrong and dump the per-tile
records around the first wrong frame."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
from zkmi import jute  # noqa: E402
from zkmi.ops import batch as B  # noqa: E402
from zkmi.bench import synthetic as S  # noqa: E402

FT_S, FT_LMAX = 4096, 1024


def plan(n):
    tiles = (n + FT_S - 1) // FT_S if n > 0 else 1
    o = 0
    offs = {}
    for name, b in (('list', tiles * FT_LMAX * 2),
                    ('pre', tiles * FT_LMAX * 2),
                    ('sx', tiles * 8), ('lbw', (2 * tiles + 4) * 8),
                    ('rent', tiles * 8), ('rexit', tiles * 8),
                    ('rmeta', tiles * 8), ('rcnt', tiles * 4),
                    ('base', tiles * 8)):
        offs[name] = o
        o += (b + 255) & ~255
    return tiles, offs


def main():
    dev = torch.device('cuda', 0)
    tree = S.GpuTree(1_000_000, 0, device=dev, data_dist=(0, 1024))
    p = S.GetPipeline(tree, 1 << 18)
    p.step()
    idx, rep, rx, ft = p.last
    n = p.batch
    ro = p.server.last_rec_off[:n].cpu().numpy()
    total = int(ro[-1]) + 4 + int(rx[int(ro[-1]):int(ro[-1]) + 4].cpu()
                                   .numpy().view('>i4')[0])
    buf = rx[:total].clone()
    sc = B.FrameScanner(n + 1024, dev, window=2048)
    t = sc.scan(buf, total)
    r = t.host_result()
    print('rescan', r, sc.chain_stats(), flush=True)
    got = t.off[:r['frames']].cpu().numpy() - 4
    truth = set(ro.tolist())
    bad = [k for k, g in enumerate(got) if int(g) not in truth]
    print('wrong frames', len(bad), flush=True)
    if not bad:
        return
    k = bad[0]
    g = int(got[k])
    tile = g // FT_S
    tiles, o = plan(sc.last_cap)
    ws = sc.ws.cpu().numpy()

    def arr(name, dt, cnt):
        return np.frombuffer(ws[o[name]:o[name] + cnt * np.dtype(dt).itemsize]
                             .tobytes(), dt)
    rent = arr('rent', np.int64, tiles)
    rexit = arr('rexit', np.int64, tiles)
    rmeta = arr('rmeta', np.int64, tiles)
    rcnt = arr('rcnt', np.int32, tiles)
    sx = arr('sx', np.int64, tiles)
    for tt in range(max(tile - 2, 0), min(tile + 2, tiles)):
        m = int(rmeta[tt])
        tr = sorted(x - tt * FT_S for x in truth
                    if tt * FT_S <= x < (tt + 1) * FT_S)
        print('tile', tt, 'entry', rent[tt] - tt * FT_S, 'exit',
              rexit[tt] - (tt + 1) * FT_S, 'cnt', m & 0x7ff, 'np',
              (m >> 11) & 0x7ff, 'js', ((m >> 22) & 0x7ff) - 1, 'term',
              (m >> 33) & 1, 'surv m', rcnt[tt], 'send', sx[tt] -
              (tt + 1) * FT_S, 'true starts', tr, flush=True)
        lst = arr('list', np.uint16, tiles * FT_LMAX)[tt * FT_LMAX:tt *
                                                       FT_LMAX + rcnt[tt]]
        pre = arr('pre', np.uint16, tiles * FT_LMAX)[tt * FT_LMAX:tt *
                                                      FT_LMAX + 16]
        print('   survivor list', lst[:40].tolist(), 'pre', pre.tolist(),
              flush=True)
    print('first wrong frame at', g, 'tile rel', g - tile * FT_S, flush=True)


if __name__ == '__main__':
    main()
