"""The native server's side of bench.py's bulk_tcp (one connection, a batch
of GET_DATA of random existing nodes in one send) without the GPU client:
the requests are pre-encoded on the host, the replies only counted.
Prints the server's wire clock: bursts, how many went to the helper
threads, and the time serving them.

  python tools/microbench/fast_bulk_probe.py [--batch 1048576] [--iters 3]

``--set`` sends SET_DATA of distinct paths instead (config 4's bulk write,
``--batch 4096``), after the session armed a data watch on every path it
will write (``--watch``): each reply then comes behind its notification.
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
ap.add_argument('--set', action='store_true')
ap.add_argument('--watch', action='store_true')
a = ap.parse_args()


def frames(idx, x0, op=4, tail=b'\0'):
    """GET_DATA (no watch) frames of /bench/dDDDDDD/nNNNNNNNN, vectorised
    (op / tail: another opcode and what follows the path)."""
    n = len(idx)
    s = np.char.add(np.char.add('/bench/d', np.char.zfill(
        (idx // 1000).astype(str), 6)), np.char.add('/n', np.char.zfill(
            idx.astype(str), 9)))
    plen = len(s[0])
    body = 4 + 4 + 4 + plen + len(tail)
    out = np.zeros((n, 4 + body), np.uint8)
    out[:, 0:4] = np.frombuffer(body.to_bytes(4, 'big'), np.uint8)
    xid = (np.arange(n, dtype=np.int64) + x0).astype('>i4')
    out[:, 4:8] = xid.view(np.uint8).reshape(n, 4)
    out[:, 8:12] = np.frombuffer(op.to_bytes(4, 'big'), np.uint8)
    out[:, 12:16] = np.frombuffer(plen.to_bytes(4, 'big'), np.uint8)
    out[:, 16:16 + plen] = np.frombuffer(''.join(s.tolist()).encode(),
                                         np.uint8).reshape(n, plen)
    out[:, 16 + plen:] = np.frombuffer(tail, np.uint8)
    return out.tobytes()


def read_frames(sk, k):
    """Read k frames; returns how many were notifications (xid -1)."""
    buf = b''
    notes = 0
    while k:
        chunk = sk.recv(1 << 22)
        if not chunk:
            raise ConnectionError('closed')
        buf += chunk
        o = 0
        while k and len(buf) - o >= 8:
            n = int.from_bytes(buf[o:o + 4], 'big')
            if len(buf) - o < 4 + n:
                break
            if buf[o + 4:o + 8] == b'\xff\xff\xff\xff':
                notes += 1
            else:
                k -= 1
            o += 4 + n
        buf = buf[o:]
    return notes


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
    x0 = 1
    for it in range(a.iters + 1):
        notes = 0
        if a.set:
            idx = rng.permutation(a.nodes)[:a.batch]
            if a.watch:                       # data watches, one burst
                sk.sendall(frames(idx, x0, 4, b'\1'))
                x0 += a.batch
                read_frames(sk, a.batch)
            req = frames(idx, x0, 5, (4).to_bytes(4, 'big') + b'data' +
                         (-1).to_bytes(4, 'big', signed=True))
        else:
            req = frames(rng.integers(0, a.nodes, a.batch), x0)
        x0 += a.batch
        srv.timing(reset=True)
        t0 = time.perf_counter()
        sk.sendall(req)
        if a.set:
            notes = read_frames(sk, a.batch)
        else:
            left = a.batch * rep_len
            while left:
                left -= len(sk.recv(min(left, 1 << 22)))
        el = time.perf_counter() - t0
        w = srv.timing()
        if it == 0:
            continue                      # (warm-up)
        print('batch %d: %.2f ms (%.2f M ops/s, %d notes) | bursts %d, '
              'parallel %d '
              '(%.1f ms) | serve %.1f ms, recv+send %.1f ms, blocked %.1f ms'
              % (it, el * 1e3, a.batch / el / 1e6, notes, w['bursts'],
                 w['par_bursts'], w['par_ns'] * 1e-6, w['serve_ns'] * 1e-6,
                 (w['recv_ns'] + w['send_ns']) * 1e-6,
                 w['blocked_ns'] * 1e-6), flush=True)
    sk.close()
finally:
    srv.shutdown()
