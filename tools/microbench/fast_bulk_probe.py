"""The native server's side of bench.py's bulk_tcp (one connection, a batch
of GET_DATA of random existing nodes in one send) without the GPU client:
the requests are pre-encoded on the host, the replies only counted.
Prints the server's wire clock: bursts, how many went to the helper
threads, and the time serving them.

  python tools/microbench/fast_bulk_probe.py [--batch 1048576] [--iters 3]
"""
import argparse
import os
import socket
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))))

import numpy as np  # noqa: E402

from zkmi import jute  # noqa: E402
from zkmi.server import fast  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--batch', type=int, default=1 << 20)
ap.add_argument('--iters', type=int, default=3)
ap.add_argument('--nodes', type=int, default=1_000_000)
ap.add_argument('--serve-threads', type=int, default=None)
a = ap.parse_args()


def frames(idx, x0):
    """GET_DATA (no watch) frames of /bench/dDDDDDD/nNNNNNNNN, vectorised."""
    n = len(idx)
    s = np.char.add(np.char.add('/bench/d', np.char.zfill(
        (idx // 1000).astype(str), 6)), np.char.add('/n', np.char.zfill(
            idx.astype(str), 9)))
    plen = len(s[0])
    body = 4 + 4 + 4 + plen + 1
    out = np.zeros((n, 4 + body), np.uint8)
    out[:, 0:4] = np.frombuffer(body.to_bytes(4, 'big'), np.uint8)
    xid = (np.arange(n, dtype=np.int64) + x0).astype('>i4')
    out[:, 4:8] = xid.view(np.uint8).reshape(n, 4)
    out[:, 8:12] = np.frombuffer((4).to_bytes(4, 'big'), np.uint8)
    out[:, 12:16] = np.frombuffer(plen.to_bytes(4, 'big'), np.uint8)
    out[:, 16:16 + plen] = np.frombuffer(''.join(s.tolist()).encode(),
                                         np.uint8).reshape(n, plen)
    return out.tobytes()


srv = fast.FastZKServer(preload=a.nodes, data_bytes=100,
                        serve_threads=a.serve_threads)
try:
    sk = socket.create_connection(('127.0.0.1', srv.port))
    sk.sendall(jute.frame(jute.encode_connect_request(
        {'timeOut': 30000, 'sessionId': 0, 'passwd': b'\0' * 16})))
    hdr = b''
    while len(hdr) < 4:
        hdr += sk.recv(4 - len(hdr))
    need = int.from_bytes(hdr, 'big')
    while need:
        need -= len(sk.recv(need))
    rng = np.random.default_rng(0)
    rep_len = 4 + 16 + 4 + 100 + 68
    for it in range(a.iters + 1):
        req = frames(rng.integers(0, a.nodes, a.batch), 1 + it * a.batch)
        srv.timing(reset=True)
        t0 = time.perf_counter()
        sk.sendall(req)
        left = a.batch * rep_len
        while left:
            left -= len(sk.recv(min(left, 1 << 22)))
        el = time.perf_counter() - t0
        w = srv.timing()
        if it == 0:
            continue                      # (warm-up)
        print('batch %d: %.1f ms (%.2f M ops/s) | bursts %d, parallel %d '
              '(%.1f ms) | serve %.1f ms, recv+send %.1f ms, blocked %.1f ms'
              % (it, el * 1e3, a.batch / el / 1e6, w['bursts'],
                 w['par_bursts'], w['par_ns'] * 1e-6, w['serve_ns'] * 1e-6,
                 (w['recv_ns'] + w['send_ns']) * 1e-6,
                 w['blocked_ns'] * 1e-6), flush=True)
    sk.close()
finally:
    srv.shutdown()
