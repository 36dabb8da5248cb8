"""Per-tile timing of fs_tile (ZKMI_FS_DBG=1): survivor walk, wait for the
tile before's exit, join walk; for the benchmark's request and reply
streams."""
import os
import sys

os.environ['ZKMI_FS_DBG'] = '1'
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from zkmi.ops import _lib  # noqa: E402
from zkmi.ops import batch as B  # noqa: E402
from zkmi.bench import synthetic as S  # noqa: E402


def dump(name, scanner, nbytes):
    torch.cuda.synchronize()
    tiles = (scanner.last_cap + 4095) // 4096
    a = _lib.lib().frame_scan_dbg(tiles).numpy()
    nt = (nbytes + 4095) // 4096
    a = a[:nt]
    t0 = a[:, 0].min()
    clk = 100.0    # wall_clock64 MHz
    stage = (a[:, 6] - a[:, 0]) / clk
    front = (a[:, 7] - a[:, 6]) / clk
    surv = (a[:, 1] - a[:, 7]) / clk
    wait = (a[:, 2] - a[:, 1]) / clk
    walk = (a[:, 3] - a[:, 2]) / clk
    end = (a[:, 3] - t0) / clk
    start = (a[:, 0] - t0) / clk
    print(name, 'tiles', nt)
    for k, v in (('start', start), ('stage', stage), ('frontier', front),
                 ('survivor', surv), ('wait', wait),
                 ('walk', walk), ('end', end), ('np', a[:, 4]),
                 ('surv', a[:, 5])):
        print('  %-9s p50 %8.2f p90 %8.2f max %8.2f mean %8.2f' % (
            k, np.percentile(v, 50), np.percentile(v, 90), v.max(),
            v.mean()))


def main():
    dev = torch.device('cuda', 0)
    # K1DBG_DIST=lo-hi: variable payloads (uniform lo..hi bytes)
    dist = os.environ.get('K1DBG_DIST')
    dd = tuple(int(x) for x in dist.split('-')) if dist else None
    data = int(os.environ.get('K1DBG_DATA', '100'))
    tree = S.GpuTree(1_000_000, data, device=dev, data_dist=dd)
    pipe = S.GetPipeline(tree, 1 << 19)
    for _ in range(2):
        pipe.step()
    torch.cuda.synchronize()
    # the reply scan ran last
    _, rep, rx, ft = pipe.last
    nrx = int(ft.result[1].item())
    dump('reply', pipe.rscanner, nrx)
    tx_len = int(pipe.server.scanner.table.result[1].item())
    pipe.server.scanner.scan(pipe.tx, tx_len)
    dump('request', pipe.server.scanner, tx_len)


if __name__ == '__main__':
    main()
