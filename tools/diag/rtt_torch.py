"""rtt_cmp.py inside a process that has initialised the GPU (as bench.py's
RTT measurement is): does the HIP runtime's presence change the blocking
get() round trip?"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))))
import bench  # noqa: E402
from zkmi.server.fast import FastZKServer  # noqa: E402

srv = FastZKServer(1000, 100)
try:
    print('before GPU: blocking', bench.measure_rtt(srv.port, 2000))
    import torch
    x = torch.ones(1 << 20, device='cuda')
    torch.cuda.synchronize()
    print('after GPU init: blocking', bench.measure_rtt(srv.port, 2000))
    print('after GPU init: evloop  ', bench.measure_rtt_async(srv.port, 2000))
    print('threads:', len(os.listdir('/proc/self/task')), 'torch threads',
          torch.get_num_threads())
finally:
    srv.shutdown()
