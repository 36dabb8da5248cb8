"""Run the fake ZooKeeper as its own process: ``python -m zkmi.server
[--host H] [--port P] [--tick-ms T]``.

Prints ``PORT <n>`` once listening and serves until stdin reaches EOF (the
parent closing the pipe).  A separate process gives the client benchmarks
a server that does not share the client's interpreter lock, as a real
ZooKeeper would not (bench.py's RTT measurement uses it).
"""

import argparse
import sys

from .fakezk import FakeZKServer


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--host', default='127.0.0.1')
    ap.add_argument('--port', type=int, default=0)
    ap.add_argument('--tick-ms', type=int, default=2000)
    a = ap.parse_args()
    srv = FakeZKServer(host=a.host, port=a.port, tick_ms=a.tick_ms)
    sys.stdout.write('PORT %d\n' % srv.port)
    sys.stdout.flush()
    try:
        sys.stdin.read()
    finally:
        srv.shutdown()


if __name__ == '__main__':
    main()
