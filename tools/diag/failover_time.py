"""Where a config-4 failover's time goes: one session with N bulk watches on
a 3-member native ensemble; member down; time to the reconnect, the
resumeWatches call and the SET_WATCHES reply.  Usage:
python tools/diag/failover_time.py [N] [cuda]"""

import sys
import threading
import time

import torch

from zkmi.models import session as S
from zkmi.parallel.ensemble import EnsembleControl
from zkmi.models.client import Client
from zkmi.config import ClientConfig, RecoveryPolicy

N = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
dev = sys.argv[2] if len(sys.argv) > 2 else None

ctl = EnsembleControl(3)
marks = {}
orig = S.ZKSession.resumeWatches


def timed(self):
    t0 = time.perf_counter()
    orig(self)
    marks['resume_call_ms'] = (time.perf_counter() - t0) * 1e3
    marks['resume_at'] = t0


S.ZKSession.resumeWatches = timed
ev = threading.Event()
n_conn = [0]


def on_connect():
    n_conn[0] += 1
    marks['connect_at'] = time.perf_counter()
    ev.set()


cfg = ClientConfig(ping_floor_ms=500, ping_timeout_floor_ms=2000,
                   connect_policy=RecoveryPolicy(1000, 3, 5, 100),
                   default_policy=RecoveryPolicy(1000, 3, 5, 100),
                   codec_device=dev)
c = Client({'servers': [{'address': '127.0.0.1', 'port': p}
                        for p in ctl.ports],
            'sessionTimeout': 8000, 'config': cfg,
            'device': torch.device(dev) if dev else False,
            'listeners': [('connect', on_connect)]})
c.wait_connected(20)
paths = ['/ens/p%05d' % k for k in range(N)]
c.call_sync('create', '/ens', b'', {})
done = threading.Event()
c.bulk([{'opcode': 'CREATE', 'path': p, 'data': b'x',
         'acl': [{'perms': ['READ', 'WRITE', 'CREATE', 'DELETE', 'ADMIN'],
                  'id': {'scheme': 'world', 'id': 'anyone'}}]}
        for p in paths], lambda e, r=None: done.set())
done.wait(60)
c.watch_bulk(paths)
done.clear()
c.bulk_get(paths, lambda e, r=None: done.set(), watch=True)
done.wait(60)
for rep in range(3):
    port = c.loop.run(lambda: c.getSession().getConnection().server['port'])
    m = ctl.ports.index(port)
    ev.clear()
    if rep:
        ctl.start(down)
    t0 = time.perf_counter()
    ctl.outage(m, [(p, b'w%d' % rep) for p in paths[:4096]])
    down = m
    t1 = time.perf_counter()
    ev.wait(30)
    t2 = time.perf_counter()
    got = 0
    while got < 4096 and time.perf_counter() - t2 < 10:
        _, k = c.take_notes()
        got += k
        time.sleep(0.0002)
    t3 = time.perf_counter()
    print('outage %.2f ms, to connect %.2f ms (resume call %.2f ms, starts '
          '%.2f ms after outage), notes %d in %.2f ms after connect'
          % ((t1 - t0) * 1e3, (t2 - t1) * 1e3, marks['resume_call_ms'],
             (marks['resume_at'] - t1) * 1e3, got, (t3 - t2) * 1e3))
c.close_sync(10)
ctl.close()
