"""The native benchmark server (``csrc/host/zk_fastserver.cpp``) as a child
process: the ZooKeeper wire protocol (handshake, ping, get, exists, set,
create, delete, sync, children, watches and SET_WATCHES) from a pool of
epoll threads (one connection per worker, round robin), so a pipelined
client benchmark measures the client, not a Python server.  ``members=M``
serves M ports over one tree with fakezk's ensemble fault commands
(:meth:`FastZKServer.outage`, :meth:`FastZKServer.start`).  ACLs, expiry and
the connection-level fault modes stay with
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
                 threads=None, members=1, serve_threads=None):
        if not available():
            raise RuntimeError('zk_fastserver not built '
                               '(tools/build_native.py)')
        # a sanitizer runtime preloaded into the caller (tools/
        # sanitize_host.sh) is not for this uninstrumented program (only
        # those entries go; anything else preloaded stays)
        env = dict(os.environ)
        if env.get('LD_PRELOAD'):
            keep = [x for x in env['LD_PRELOAD'].replace(':', ' ').split()
                    if 'san.so' not in os.path.basename(x)]
            if keep:
                env['LD_PRELOAD'] = ' '.join(keep)
            else:
                del env['LD_PRELOAD']
        # transparent huge pages for the node heap (THP in madvise mode):
        # a GET or SET is a handful of dependent misses into ~0.5 GB of
        # nodes, paths and data per 1M znodes, each a TLB miss on 4 KiB
        # pages (ZKMI_FAST_HUGEPAGES=0: off)
        if os.environ.get('ZKMI_FAST_HUGEPAGES', '1') == '1':
            tun = env.get('GLIBC_TUNABLES', '')
            env['GLIBC_TUNABLES'] = (tun + ':' if tun else '') + \
                'glibc.malloc.hugetlb=1'
        self.p = subprocess.Popen(
            [BINARY, '--port', str(port), '--preload', str(preload),
             '--data-bytes', str(data_bytes), '--fanout', str(fanout)] +
            (['--threads', str(threads)] if threads else []) +
            (['--serve-threads', str(serve_threads)]
             if serve_threads is not None else []) +
            (['--members', str(members)] if members > 1 else []),
            stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True,
            env=env)
        f = self.p.stdout.readline().split()
        if len(f) < 2 or f[0] not in ('PORT', 'PORTS'):
            self.p.kill()
            raise RuntimeError('zk_fastserver did not start: %r' % f)
        self.ports = [int(x) for x in f[1:]]
        self.port = self.ports[0]

    def _cmd(self, line):
        self.p.stdin.write(line + '\n')
        self.p.stdin.flush()
        ans = self.p.stdout.readline().split(None, 1)
        if not ans or ans[0] != 'OK':
            raise RuntimeError('zk_fastserver command %r: %r' % (line, ans))
        return ans[1].strip() if len(ans) > 1 else ''

    def outage(self, i, sets=()):
        """Member ``i`` down (its connections and port close; sessions
        stay, their watches go), then ``sets`` = [(path, data)] applied,
        firing watches.  Returns the zxid after them."""
        return int(self._cmd('outage %d %s' % (i, ' '.join(
            '%s=%s' % (p, d.hex()) for p, d in sets))))

    def start(self, i):
        """Member ``i`` listens on its port again; returns the port."""
        return int(self._cmd('start %d' % i))

    CLOCK = ('first_rx', 'last_rx', 'first_tx', 'last_tx', 'recv_ns',
             'serve_ns', 'send_ns', 'blocked_ns', 'rx_bytes', 'tx_bytes',
             'bursts', 'sends', 'recvs', 'par_bursts', 'par_ns')

    def timing(self, reset=False):
        """The server's wire clock since the last reset (CLOCK_MONOTONIC ns,
        the clock of ``time.perf_counter``): first / last recv that returned
        bytes and send that moved bytes; ns spent in recv(), serving frames,
        send() and with replies blocked on a full socket; bytes, bursts,
        send and recv calls.  ``reset=True`` zeroes it (returns None)."""
        if reset:
            self._cmd('timing reset')
            return None
        v = [int(x) for x in self._cmd('timing').split()]
        return dict(zip(self.CLOCK, v))

    @property
    def address(self):
        return {'address': '127.0.0.1', 'port': self.port}

    def servers(self):
        return [{'address': '127.0.0.1', 'port': p} for p in self.ports]

    def shutdown(self):
        try:
            self.p.stdin.close()
            self.p.wait(10)
        except Exception:                       # noqa: BLE001
            self.p.kill()
