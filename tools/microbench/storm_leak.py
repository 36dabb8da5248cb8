"""Storm leak hunt (small tree): after every expiry, any node still owned
by the expired session is located in the hash index from its home slot,
with what lies between (tree.hip 64-byte entries: key, val, ...)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from zkmi.bench.synthetic import GpuTree, StormPipeline  # noqa: E402

M64 = (1 << 64) - 1


def path_hash(p):
    n = len(p)
    h = (0x9E3779B97F4A7C15 ^ n) & M64
    i = 0
    while i + 8 <= n:
        w = int.from_bytes(p[i:i + 8], 'little')
        h = ((h ^ w) * 0xFF51AFD7ED558CCD) & M64
        h ^= h >> 32
        i += 8
    if i < n:
        w = int.from_bytes(p[i:], 'little')
        h = ((h ^ w) * 0xFF51AFD7ED558CCD) & M64
        h ^= h >> 32
    h ^= h >> 33
    h = (h * 0xC4CEB9FE1A85EC53) & M64
    h ^= h >> 33
    return h


dev = torch.device('cuda', 0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
tree = GpuTree(20000, 37, fanout=100, device=dev, spare=1.5)
pipe = StormPipeline(tree, n, ndirs=64)
for s in range(steps):
    ok = int(pipe.step().item())
    if ok == n:
        continue
    print('step', s, 'ok', ok, pipe.diagnose()['removed'], flush=True)
    torch.cuda.synchronize()
    cnt = tree.counters.cpu().tolist()
    nn = cnt[0]
    eph = tree.eph[:nn].cpu().numpy()
    par = tree.node_parent[:nn].cpu().numpy()
    prev = int(pipe.prev_sid.item())
    left = np.nonzero((eph == prev) & (par != -2))[0]
    print('expired session', hex(prev), 'nodes left', len(left))
    ht = tree.ht.view(-1, 8).cpu().numpy()
    mask = tree.hcap - 1
    arena = tree.path_arena.cpu().numpy().tobytes()
    po = tree.node_path_off.cpu().numpy()
    pl = tree.node_path_len.cpu().numpy()
    for v in left[:5]:
        p = arena[po[v]:po[v] + pl[v]]
        key = (path_hash(p) | 1)
        keys = ht[:, 0].astype(np.uint64)
        where = np.nonzero(keys == np.uint64(key))[0]
        home = key & mask
        print(' node', v, p, 'home', home, 'entries with key', where,
              'vals', [int(ht[w, 1]) for w in where])
        for w in where:
            d = int((w - home) & mask)
            seg = [int((home + k) & mask) for k in range(d + 1)]
            empt = [x for x in seg if ht[x, 0] == 0]
            print('  at', w, 'dist', d, 'val', int(ht[w, 1]),
                  'empties between', empt[:8], flush=True)
            lo = max(0, len(seg) - 6)
            print('  last slots', [(x, int(ht[x, 0]) & 0xffffff,
                                    int(ht[x, 1])) for x in seg[lo:]])
    break
else:
    print('no leak in', steps, 'steps')
