"""bench.py's round-trip measurements against the native fast server (CPU
only: the client, its event loop and the server; no GPU)."""

import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(
    __file__))))


def _server():
    from zkmi.server.fast import FastZKServer
    try:
        return FastZKServer(100, 16)
    except (OSError, RuntimeError) as e:      # binary not built here
        pytest.skip('zk_fastserver unavailable: %s' % e)


def test_rtt_blocking_and_event_loop():
    import bench
    srv = _server()
    try:
        p50, p99 = bench.measure_rtt(srv.port, 200)
        e50, e99 = bench.measure_rtt_async(srv.port, 200, warm=20)
    finally:
        srv.shutdown()
    assert 0 < p50 <= p99
    assert 0 < e50 <= e99
