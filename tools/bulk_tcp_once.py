"""One bulk_get-over-TCP measurement (bench.measure_bulk_tcp) against the
native server: ops/s and phase times for 1 and 8 connections.

    python tools/bulk_tcp_once.py [--batch 1048576] [--iters 3]
"""

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=1 << 20)
    ap.add_argument('--iters', type=int, default=3)
    ap.add_argument('--nodes', type=int, default=1_000_000)
    a = ap.parse_args()
    srv = bench.start_fast_server(a.nodes, 100)
    import torch
    dev = torch.device('cuda', 0)
    try:
        one = bench.measure_bulk_tcp(srv.port, a.nodes, a.batch, a.iters,
                                     dev, 1, srv)
        k = bench.measure_bulk_tcp(srv.port, a.nodes, a.batch, a.iters, dev, 8)
    finally:
        srv.shutdown()
    print(json.dumps({'ops_s_1conn': round(one[0]), 'phases_1conn': one[2],
                      'ops_s_8conn': round(k[0])},
                     default=float))


if __name__ == '__main__':
    main()
