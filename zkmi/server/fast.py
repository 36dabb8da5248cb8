"""The native benchmark server (``csrc/host/zk_fastserver.cpp``) as a child
process: the ZooKeeper wire protocol's data plane (handshake, ping, get,
exists, set, create, delete, sync, children) from a pool of epoll threads
(one connection per worker, round robin), so a pipelined client benchmark
measures the client, not a Python server.  The
full contract (watches, ensembles, fault hooks) stays with
:class:`~zkmi.server.fakezk.FakeZKServer`."""

import os
import subprocess

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BINARY = os.path.join(_ROOT, 'bin', 'zk_fastserver')


def available():
    return os.path.exists(BINARY)


class FastZKServer(object):
    """``FastZKServer(preload=N, data_bytes=B)`` starts the server with the
    synthetic ``/bench`` tree of N leaves (GpuTree's layout)."""

    def __init__(self, preload=0, data_bytes=100, fanout=1000, port=0,
                 threads=None):
        if not available():
            raise RuntimeError('zk_fastserver not built '
                               '(tools/build_native.py)')
        # a sanitizer runtime preloaded into the caller (tools/
        # sanitize_host.sh) is not for this uninstrumented program
        env = {k: v for k, v in os.environ.items() if k != 'LD_PRELOAD'}
        self.p = subprocess.Popen(
            [BINARY, '--port', str(port), '--preload', str(preload),
             '--data-bytes', str(data_bytes), '--fanout', str(fanout)] +
            (['--threads', str(threads)] if threads else []),
            stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True,
            env=env)
        f = self.p.stdout.readline().split()
        if len(f) != 2 or f[0] != 'PORT':
            self.p.kill()
            raise RuntimeError('zk_fastserver did not start: %r' % f)
        self.port = int(f[1])

    @property
    def address(self):
        return {'address': '127.0.0.1', 'port': self.port}

    def servers(self):
        return [self.address]

    def shutdown(self):
        try:
            self.p.stdin.close()
            self.p.wait(10)
        except Exception:                       # noqa: BLE001
            self.p.kill()
