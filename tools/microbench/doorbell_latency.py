"""Single-record codec latency on one MI355X: the persistent doorbell wave
(csrc/kernels/doorbell.hip) vs one batch-kernel launch per record (K10 with
n = 1 and a stream sync) vs the native host codec.  Prints p50 / p99 in us
for a GET_DATA request encode and a GET_DATA reply decode."""

import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))

import torch  # noqa: E402

from zkmi import codec, jute  # noqa: E402
from zkmi.ops import batch as B  # noqa: E402
from zkmi.ops.doorbell import DoorbellCodec  # noqa: E402


def lat(fn, n=3000, warm=300):
    for _ in range(warm):
        fn()
    ts = []
    for _ in range(n):
        t = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t) * 1e6)
    ts.sort()
    return statistics.median(ts), ts[int(0.99 * len(ts))]


def main():
    pkt = {'xid': 7, 'opcode': 'GET_DATA', 'path': '/bench/d000123/n000123456',
           'watch': False}
    rep = {'xid': 7, 'zxid': 99, 'err': 'OK', 'opcode': 'GET_DATA',
           'data': b'x' * 100, 'stat': jute.Stat(1, 2, 3, 4, 5, 6, 7, 0, 100,
                                                 0, 9)}
    body = jute.encode_response(rep)
    dev = torch.device('cuda', 0)
    rows = []
    with DoorbellCodec(max_seconds=60) as db:
        rows.append(('doorbell encode', lat(lambda: db.encode_request(pkt))))
        rows.append(('doorbell decode',
                     lat(lambda: db.decode_response(body, 'GET_DATA'))))
    xt = B.XidTable(bits=10, device=dev)

    def launch_encode():
        rb = B.pack_requests([pkt], device=dev)
        out, _, total, _ = B.encode_requests(rb, xt)
        torch.cuda.synchronize()
    rows.append(('kernel-launch encode (K10, n=1)', lat(launch_encode, 500,
                                                        50)))
    rows.append(('host codec encode (%s)' % codec.IMPL,
                 lat(lambda: codec.frame(codec.encode_request(pkt)))))
    rows.append(('host codec decode (%s)' % codec.IMPL,
                 lat(lambda: codec.decode_response(body, {7: 'GET_DATA'}))))
    for name, (p50, p99) in rows:
        print('%-36s p50 %8.2f us   p99 %8.2f us' % (name, p50, p99),
              flush=True)


if __name__ == '__main__':
    main()
