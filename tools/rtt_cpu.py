"""Interactive-path timing on the host (no GPU): event-loop get() round
trips and pipelined get() throughput against the native server.

    python tools/rtt_cpu.py [--n 20000] [--window 256]
"""

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=20000)
    ap.add_argument('--window', type=int, default=256)
    ap.add_argument('--nodes', type=int, default=1000,
                    help='znodes preloaded in the native server')
    ap.add_argument('--torch-gpu', action='store_true',
                    help='start the server, then initialise the GPU in this '
                         'process first (as bench.py does)')
    a = ap.parse_args()
    srv = bench.start_fast_server(a.nodes, 100)
    if a.torch_gpu:
        import torch
        torch.ones(1, device='cuda').sum().item()
    if srv is None:
        raise SystemExit('native server not built')
    try:
        ev50, ev99 = bench.measure_rtt_async(srv.port, n=a.n)
        ops = bench.measure_pipelined(srv.port, n=a.n * 10, window=a.window)
        b50, b99 = bench.measure_rtt(srv.port, n=a.n // 4)
    finally:
        srv.shutdown()
    print(json.dumps({'evloop_p50_us': round(ev50, 2),
                      'evloop_p99_us': round(ev99, 2),
                      'blocking_p50_us': round(b50, 2),
                      'blocking_p99_us': round(b99, 2),
                      'pipelined_get_ops_s': round(ops),
                      'window': a.window, 'nodes': a.nodes,
                      'torch_gpu': a.torch_gpu}))


if __name__ == '__main__':
    main()
