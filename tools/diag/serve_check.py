"""Diagnostic: run the GET pipeline's server half step by step and check
the serve kernel's reply descriptors on the host before the reply encode."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
from zkmi.ops import _lib  # noqa: E402
from zkmi.ops import batch as B  # noqa: E402
from zkmi.bench import synthetic as S  # noqa: E402


def main():
    dev = torch.device('cuda', 0)
    tree = S.GpuTree(20000, 37, fanout=100, device=dev)
    n = 8192
    ht = tree.ht.view(-1, _lib.HT_WORDS).cpu()
    live = ht[:, 1] >= 0
    print('entries', int(live.sum()), flush=True)
    p = S.GetPipeline(tree, n)
    g = p._phases(True, torch.zeros(1, dtype=torch.int64, device=dev))
    next(g)                       # request encode issued
    torch.cuda.synchronize()
    print('encode ok', flush=True)
    srv = p.server
    tx = p.tx
    L = _lib.lib()
    # the server half by hand; the paused generator holds `total`
    total = g.gi_frame.f_locals['total']
    ntx = int(total.item())
    ft = B.frame_scan(tx, ntx, cap=srv.cap_frames, window=srv.window)
    rt = B.decode_requests(tx, ft, out=srv.rt)
    torch.cuda.synchronize()
    print('scan+decode ok, frames', int(ft.count.item()), flush=True)
    r = srv.resp
    r.count = ft.count
    r.slot.fill_(-7)
    L.tree_serve(tree.tensors, tx, rt.tensors(), ft.count, srv.cap_frames,
                 [r.opcode, r.xid, r.err, r.node, r.zxid, r.path_off,
                  r.path_len, r.slot, srv.presized[0], srv.presized[1]],
                 0, int(time.time() * 1000))
    torch.cuda.synchronize()
    print('serve ok', flush=True)
    err = r.err[:n].cpu()
    slot = r.slot[:n].cpu()
    node = r.node[:n].cpu()
    sizes = srv.presized[0][:n].cpu()
    nb = (n + 255) // 256
    bsum = srv.presized[1][:nb].cpu()
    print('err!=0', int((err != 0).sum()), 'slot', int(slot.min()),
          int(slot.max()), 'node', int(node.min()), int(node.max()),
          'sizes', int(sizes.min()), int(sizes.max()),
          'bsum ok', bool((bsum == sizes.view(nb, 256).sum(1)).all()),
          flush=True)
    want = tree.slot_off[node.to(dev)].cpu()
    good = bool((want == slot).all())
    print('slot==slot_off[node]', good, flush=True)
    if not good:
        return
    p2 = S.GetPipeline(tree, n)
    for _ in range(3):
        acc = p2.step()
        print('step ok', int(acc.item()), flush=True)


if __name__ == '__main__':
    main()
