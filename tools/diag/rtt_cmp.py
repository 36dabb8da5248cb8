"""Interactive get() RTT against the native server: blocking call_sync and
event-loop chained callbacks (bench.measure_rtt / measure_rtt_async)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))))
import bench  # noqa: E402
from zkmi.server.fast import FastZKServer  # noqa: E402

srv = FastZKServer(1000, 100)
try:
    print('blocking', bench.measure_rtt(srv.port, 3000))
    print('evloop  ', bench.measure_rtt_async(srv.port, 3000))
finally:
    srv.shutdown()
