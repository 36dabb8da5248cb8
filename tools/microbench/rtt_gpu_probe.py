"""Why the event-loop get() round trip is slower after the GPU work: the
same measurement (bench.measure_rtt_async, native server, loopback) at
each stage of a bench process's life, and with the suspects removed.

  stage 0  before the process touches the GPU
  stage 1  after torch initialised the GPU (one tiny kernel)
  stage 2  after a 1M-node tree, a GET pipeline and its graph replays
  stage 3  the same, after gc.collect() + gc.freeze() (the long-lived
           objects out of the collector's generations)
  stage 4  the same with the collector off

  python tools/microbench/rtt_gpu_probe.py [--n 20000] [--steps 300]
"""
import argparse
import gc
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))))

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=20000)
    ap.add_argument('--steps', type=int, default=300)
    a = ap.parse_args()
    srv = bench.start_fast_server(1000, 100)
    out = {}

    def stage(name):
        p50, p99 = bench.measure_rtt_async(srv.port, n=a.n)
        out[name] = {'p50_us': round(p50, 2), 'p99_us': round(p99, 2),
                     'threads': threading.active_count(),
                     'gc_counts': gc.get_count()}
        print(name, out[name], flush=True)
    try:
        stage('0_pre_gpu')
        import torch
        torch.ones(1, device='cuda').sum().item()
        stage('1_gpu_init')
        from zkmi.bench import synthetic as S
        dev = torch.device('cuda', 0)
        tree = S.GpuTree(1000000, 100, device=dev, seed=0)
        pipe = S.GetPipeline(tree, 1 << 20, seed=0, streams=2)
        acc = torch.zeros(64, dtype=torch.int64, device=dev)
        for _ in range(3):
            pipe.step(acc=acc)
        g = pipe.capture(acc)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            g.replay()
        torch.cuda.synchronize()
        print('replays %.3f ms/step' % ((time.perf_counter() - t0) * 1e3 /
                                       a.steps), flush=True)
        stage('2_after_gpu_work')
        gc.collect()
        gc.freeze()
        stage('3_gc_frozen')
        gc.disable()
        stage('4_gc_off')
        gc.enable()
    finally:
        srv.shutdown()
    print(json.dumps(out))


if __name__ == '__main__':
    main()
