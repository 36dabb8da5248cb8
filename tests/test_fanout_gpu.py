"""R1 on the GPU: the interactive DistributedWatcher API
(zkmi/parallel/group.py) over FrameFanout with RCCL (``nccl``, world 1 on
the one-GPU box) — the owner's events travel as wire frames and are decoded
by K1 + K2-K8 on the device, not by the host codec.

Reference: lib/zk-session.js:853-854 (one watcher's events to every
listener)."""

import socket
import time

import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_group_fanout_decodes_on_the_gpu():
    import torch
    import torch.distributed as dist
    from zkhelpers import client
    from zkmi.parallel import SessionGroup
    from zkmi.server import FakeZKServer
    zk = FakeZKServer(tick_ms=250)
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    dist.init_process_group('nccl', init_method='tcp://127.0.0.1:%d'
                            % _free_port(), rank=0, world_size=1,
                            device_id=dev)
    c = None
    try:
        c = client([{'address': '127.0.0.1', 'port': zk.port}],
                   session_timeout=4000)
        c.wait_connected(10)
        g = SessionGroup(c)
        assert g.fan.dev is not None and g.fan.coll.type == 'cuda'
        c.call_sync('create', '/gf', b'a', {})
        seen = []
        g.watcher('/gf').on('dataChanged',
                            lambda d, s: seen.append((d, s.version)))

        def tick_until(n):
            t_end = time.monotonic() + 20
            while len(seen) < n:
                assert time.monotonic() < t_end, seen
                g.tick()
                time.sleep(0.01)
        tick_until(1)
        c.call_sync('set', '/gf', b'bb', -1)
        tick_until(2)
        assert seen == [(b'a', 0), (b'bb', 1)]
        assert g.fan.stats['decoded_gpu'] == 4
        assert g.fan.stats['decoded_host'] == 0
    finally:
        if c is not None:
            c.close_sync(10)
        dist.destroy_process_group()
        zk.shutdown()
