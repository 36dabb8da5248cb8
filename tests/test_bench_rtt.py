"""bench.py's round-trip measurements against the native fast server (the
client, its event loop and the server; the bulk TCP split needs the GPU
codec path)."""

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


def test_server_wire_clock():
    """The server's wire clock counts a client's traffic and resets."""
    import time
    from zkmi import Client
    srv = _server()
    try:
        srv.timing(reset=True)
        t0 = time.perf_counter()
        c = Client(address='127.0.0.1', port=srv.port)
        c.wait_connected(10)
        for _ in range(20):
            c.call_sync('get', '/bench/d000000/n000000001')
        # (the server stamps a send after send() returns: the client may
        # have the reply before that; read the clock once it settled)
        time.sleep(0.05)
        w = srv.timing()
        t1 = time.perf_counter()
        c.close_sync(10)
        srv.timing(reset=True)
        z = srv.timing()
    finally:
        srv.shutdown()
    # the same clock as perf_counter
    assert t0 * 1e9 <= w['first_rx'] <= w['last_tx'] <= t1 * 1e9
    assert w['bursts'] >= 21 and w['sends'] >= 21
    assert w['rx_bytes'] > 0 and w['tx_bytes'] > 0
    assert w['serve_ns'] > 0 and w['recv_ns'] > 0 and w['send_ns'] > 0
    assert all(v == 0 for v in z.values())


@pytest.mark.gpu
def test_bulk_tcp_wire_split():
    """The bulk TCP phases split the wire + server time by the server's own
    clock: the pieces are non-negative and add up inside the span."""
    import torch
    import bench
    srv = _server()
    try:
        w0 = srv.timing()
        assert set(w0) == set(srv.CLOCK)
        ops, ms, ph = bench.measure_bulk_tcp(srv.port, 100, 256, 2,
                                             torch.device('cuda', 0), 1, srv)
        w = srv.timing()
    finally:
        srv.shutdown()
    assert ops > 0 and ms > 0
    sp = ph['wire_split_ms']
    assert sp['server_span'] >= 0 and sp['client_capture'] >= 0
    assert sp['client_send'] >= 0
    # serve + socket time happen inside the server's span (one connection)
    assert sp['server_serve'] + sp['server_socket'] <= \
        sp['server_span'] + 1.0
    # (medians over the attributed batches: their sum is near, not at, the
    # median of the sums)
    assert abs(sp['client_send'] + sp['server_span'] +
               sp['client_capture'] - sp['send_to_capture']) < \
        0.05 * sp['send_to_capture'] + 0.01
    assert w['rx_bytes'] > 0 and w['tx_bytes'] > w['rx_bytes']
    assert w['first_rx'] <= w['last_tx']
