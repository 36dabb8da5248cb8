"""Run the fake ZooKeeper as its own process: ``python -m zkmi.server
[--host H] [--port P] [--tick-ms T] [--ensemble N]``.

Prints ``PORT <n>`` (one server) or ``PORTS <p1> ... <pN>`` (``--ensemble
N``: N endpoints sharing one database, the 3-JVM ensemble of
``test/multi-node.test.js``) once listening, and serves until stdin reaches
EOF (the parent closing the pipe).  A separate process gives the client
benchmarks a server that does not share the client's interpreter lock, as a
real ZooKeeper would not (bench.py's RTT measurement uses it).

With ``--ensemble`` stdin also carries one fault command per line, each
answered by one line (``OK <detail>`` or ``ERR <reason>``):

  ``outage <i> [<path>=<hexdata> ...]``  kill member i, then apply the sets
                                         in the same loop turn (answers the
                                         zxid after them)
  ``start <i>``                          restart member i on its old port
"""

import argparse
import sys

from .fakezk import FakeEnsemble, FakeZKServer


def _command(ens, line):
    f = line.split()
    if not f:
        return 'ERR empty'
    if f[0] == 'outage':
        sets = []
        for kv in f[2:]:
            p, _, h = kv.partition('=')
            sets.append((p, bytes.fromhex(h)))
        return 'OK %d' % ens.outage(int(f[1]), sets)
    if f[0] == 'start':
        ens[int(f[1])].start()
        return 'OK %d' % ens[int(f[1])].port
    return 'ERR unknown command %r' % f[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--host', default='127.0.0.1')
    ap.add_argument('--port', type=int, default=0)
    ap.add_argument('--tick-ms', type=int, default=2000)
    ap.add_argument('--ensemble', type=int, default=0)
    a = ap.parse_args()
    if a.ensemble:
        ens = FakeEnsemble(a.ensemble, tick_ms=a.tick_ms)
        sys.stdout.write('PORTS %s\n' % ' '.join(
            str(m.port) for m in ens.members))
        sys.stdout.flush()
        try:
            for line in sys.stdin:
                try:
                    out = _command(ens, line)
                except Exception as e:          # noqa: BLE001
                    out = 'ERR %s: %s' % (type(e).__name__, e)
                sys.stdout.write(out + '\n')
                sys.stdout.flush()
        finally:
            ens.shutdown()
        return
    srv = FakeZKServer(host=a.host, port=a.port, tick_ms=a.tick_ms)
    sys.stdout.write('PORT %d\n' % srv.port)
    sys.stdout.flush()
    try:
        sys.stdin.read()
    finally:
        srv.shutdown()


if __name__ == '__main__':
    main()
