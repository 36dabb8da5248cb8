"""BASELINE config 4: a 3-server ensemble, one ZooKeeper session per rank,
failover of a rank's server and the watch replay fanned out over the node.

Reference behaviour this reproduces at node scale:

* ephemeral failover — kill the server a session lives on, the session
  moves to another member without expiring (``test/multi-node.test.js:
  233-350``, ``lib/zk-session.js:265-339``);
* watch resume — the reattached session re-arms its watches with one
  SET_WATCHES at ``relZxid = lastZxid`` and the server replays every change
  it missed (``lib/zk-session.js:421-471``);
* watch fan-out — one server watch per path, its events delivered to every
  listener (``lib/zk-session.js:853-854``), here to every rank of the node.

Per rank: a :class:`~zkmi.Client` on the ensemble (rank ``r`` prefers
member ``r % n``), with ``ClientConfig.codec_device`` set on a GPU so its
(re)connects run K9 (ConnectRequest / ConnectResponse) and its watch resume
K11 (SET_WATCHES) on the device (:mod:`zkmi.models.gpucodec`).  Each path
has one owner rank (``crc32(path) % world``) that holds the only server
watch on it; owners forward the events their watchers emit with
:class:`WireFanout` (R1).

:class:`WireFanout` ships events as the ZooKeeper wire frames the owner's
session received — a NOTIFICATION frame (xid -1, type, state, path) and the
re-arm's GET_DATA reply (data + Stat) — so the node-wide stream is decoded
by the same kernels as a connection's RX stream: one size exchange, one
padded ``all_gather_into_tensor`` on the collective device (GPU tensors
over RCCL/xGMI with ``nccl``), then K1 frame scan + K2-K8 reply decode on
the GPU of every rank and one device-to-host copy of the decoded table.
Without a GPU (gloo rehearsal on CPU) the gathered frames are decoded by
the host codec instead.
"""

import collections
import subprocess
import sys
import threading
import time
import zlib

import numpy as np
import torch
import torch.distributed as dist

from .. import codec
from .. import consts
from .. import jute

KMAX = 1 << 16            # events one rank forwards per exchange
_GET_DATA = consts.OP_CODES['GET_DATA']


def owner_of(path, world):
    return zlib.crc32(path.encode('utf-8')) % world


class WireFanout(object):
    """R1 over the node: every rank's watch events, as wire frames, to every
    rank (collective: all ranks call :meth:`exchange` together)."""

    def __init__(self, group=None, decode_device=None):
        on = dist.is_available() and dist.is_initialized()
        self.group = group
        self.world = dist.get_world_size(group) if on else 1
        self.rank = dist.get_rank(group) if on else 0
        backend = dist.get_backend(group) if on else None
        if decode_device is None and torch.cuda.is_available():
            decode_device = torch.device('cuda', torch.cuda.current_device())
        self.dev = torch.device(decode_device) if decode_device else None
        # collective tensors live where the backend moves them: HBM for
        # RCCL, host memory for gloo
        self.coll = self.dev if backend in (None, 'nccl') and self.dev \
            else torch.device('cpu')
        self.stats = collections.Counter()
        self.xt = None
        if self.dev is not None and self.dev.type == 'cuda':
            from ..ops import batch as B
            self.B = B
            bits = max(10, (self.world * KMAX - 1).bit_length())
            self.xt = B.XidTable(bits=bits, device=self.dev)
            x = torch.arange(self.world * KMAX, dtype=torch.int64,
                             device=self.dev)
            self.xt.tab[x & self.xt.mask] = (x << 32) | _GET_DATA

    # -- encode (owner side) -------------------------------------------------

    def encode(self, events):
        """``events`` = [(path, data, Stat)] -> framed NOTIFICATION +
        GET_DATA reply per event (xid = rank << 16 | k)."""
        parts = []
        base = self.rank << 16
        for k, (path, data, stat) in enumerate(events):
            parts.append(codec.frame(jute.encode_response({
                'xid': consts.XID_NOTIFICATION, 'zxid': -1, 'err': 'OK',
                'opcode': 'NOTIFICATION', 'type': 'DATA_CHANGED',
                'state': 'SYNC_CONNECTED', 'path': path})))
            parts.append(codec.frame(jute.encode_response({
                'xid': base | k, 'zxid': stat.mzxid, 'err': 'OK',
                'opcode': 'GET_DATA', 'data': data, 'stat': stat})))
        return b''.join(parts)

    # -- the collective -------------------------------------------------------

    def exchange(self, events):
        """Send this rank's ``events`` (at most :data:`KMAX`), receive every
        rank's: returns [(src_rank, path, data, Stat)] in rank order."""
        if len(events) > KMAX:
            raise ValueError('at most %d events per exchange' % KMAX)
        payload = self.encode(events)
        W = self.world
        if W == 1:
            sizes = [len(payload)]
            rx = None
        else:
            # the one size exchange (a single host read of W sizes)
            n = torch.tensor([len(payload)], dtype=torch.int64,
                             device=self.coll)
            st = torch.empty(W, dtype=torch.int64, device=self.coll)
            dist.all_gather_into_tensor(st, n, group=self.group)
            sizes = st.cpu().tolist()
            mx = max(max(sizes), 1)
            buf = torch.zeros(mx, dtype=torch.uint8, device=self.coll)
            if payload:
                buf[:len(payload)].copy_(torch.frombuffer(
                    bytearray(payload), dtype=torch.uint8))
            rx = torch.empty(W * mx, dtype=torch.uint8, device=self.coll)
            dist.all_gather_into_tensor(rx, buf, group=self.group)
        self.stats['exchanges'] += 1
        self.stats['bytes'] += sum(sizes)
        if self.xt is not None:
            return self._decode_gpu(payload, rx, sizes)
        return self._decode_host(payload, rx, sizes)

    def _segments(self, payload, rx, sizes):
        mx = max(max(sizes), 1)
        if rx is None:
            return [torch.frombuffer(bytearray(payload or b'\0'),
                                     dtype=torch.uint8)[:len(payload)]]
        return [rx[r * mx:r * mx + s] for r, s in enumerate(sizes) if s]

    def _decode_gpu(self, payload, rx, sizes):
        B = self.B
        dev = self.dev
        total = sum(sizes)
        if total == 0:
            return []
        segs = self._segments(payload, rx, sizes)
        # close the padding gaps on the device (rank order kept)
        stream = torch.cat([s.to(dev, non_blocking=True) for s in segs])
        ft = B.frame_scan(stream, total, cap=total // 32 + 1,
                          window=B.frame_window(512))
        rep = B.decode_replies(stream, ft, self.xt)
        cap = ft.off.numel()
        cols = torch.cat([
            ft.result.to(torch.int64),
            rep.xid.to(torch.int64), rep.opcode.to(torch.int64),
            rep.status.to(torch.int64), rep.err.to(torch.int64),
            rep.pay_off, rep.pay_len.to(torch.int64),
            rep.aux0.to(torch.int64), rep.aux1.to(torch.int64),
            rep.stat64.reshape(-1), rep.stat32.to(torch.int64).reshape(-1)])
        host = cols.cpu().numpy()                   # one D2H for the table
        hb = stream.cpu().numpy().tobytes()        # one for the bytes
        nfr, bad = int(host[0]), int(host[2])
        if bad or int(host[3]):
            raise RuntimeError('fan-out stream: bad frame')
        c = host[4:]
        xid, op, st, err, po, pl, a0, a1 = (c[k * cap:(k + 1) * cap]
                                            for k in range(8))
        s64 = c[8 * cap:14 * cap].reshape(6, cap)
        s32 = c[14 * cap:19 * cap].reshape(5, cap)
        out = []
        notif = consts.OP_CODES['NOTIFICATION']
        for i in range(0, nfr, 2):
            j = i + 1
            if j >= nfr or op[i] != notif or op[j] != _GET_DATA or \
                    st[i] or st[j] or err[i] or err[j]:
                raise RuntimeError('fan-out stream: unpaired frame %d' % i)
            path = hb[po[i]:po[i] + pl[i]].decode('utf-8')
            data = hb[po[j]:po[j] + pl[j]]
            stat = jute.Stat(int(s64[0, j]), int(s64[1, j]), int(s64[2, j]),
                             int(s64[3, j]), int(s32[0, j]), int(s32[1, j]),
                             int(s32[2, j]), int(s64[4, j]), int(s32[3, j]),
                             int(s32[4, j]), int(s64[5, j]))
            out.append((int(xid[j]) >> 16, path, data, stat))
        self.stats['decoded_gpu'] += len(out)
        return out

    def _decode_host(self, payload, rx, sizes):
        out = []
        for seg in self._segments(payload, rx, sizes):
            raw = bytes(seg.numpy().tobytes()) if seg.numel() else b''
            frames, _, bad = codec.scan_frames(raw, 0, len(raw),
                                               consts.MAX_PACKET)
            if bad >= 0:
                raise RuntimeError('fan-out stream: bad frame')
            bodies = [raw[o:o + n] for o, n in frames]
            for i in range(0, len(bodies), 2):
                nb, rb = bodies[i], bodies[i + 1]
                xid = int.from_bytes(rb[0:4], 'big', signed=True)
                n = codec.decode_response(nb, {})
                r = codec.decode_response(rb, {xid: 'GET_DATA'})
                out.append((xid >> 16, n['path'], r['data'], r['stat']))
        self.stats['decoded_host'] += len(out)
        return out


class EnsembleControl(object):
    """The fake ensemble as a child process (``python -m zkmi.server
    --ensemble N``), driven over its stdin fault-command channel."""

    def __init__(self, n=3, tick_ms=250):
        self.p = subprocess.Popen(
            [sys.executable, '-m', 'zkmi.server', '--ensemble', str(n),
             '--tick-ms', str(tick_ms)],
            stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
        f = self.p.stdout.readline().split()
        if not f or f[0] != 'PORTS':
            self.p.kill()
            raise RuntimeError('ensemble did not start: %r' % f)
        self.ports = [int(x) for x in f[1:]]

    def _cmd(self, line):
        self.p.stdin.write(line + '\n')
        self.p.stdin.flush()
        ans = self.p.stdout.readline().split(None, 1)
        if not ans or ans[0] != 'OK':
            raise RuntimeError('ensemble command %r: %r' % (line, ans))
        return ans[1].strip() if len(ans) > 1 else ''

    def outage(self, i, sets):
        return int(self._cmd('outage %d %s' % (i, ' '.join(
            '%s=%s' % (p, d.hex()) for p, d in sets))))

    def start(self, i):
        self._cmd('start %d' % i)

    def close(self):
        try:
            self.p.stdin.close()
            self.p.wait(10)
        except Exception:                           # noqa: BLE001
            self.p.kill()


def _bcast_ints(vals, n, src, device):
    t = torch.zeros(n, dtype=torch.int64, device=device)
    if vals is not None:
        t[:len(vals)] = torch.tensor(vals, dtype=torch.int64)
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.broadcast(t, src)
    return t.cpu().tolist()


class EnsembleWorkload(object):
    """Collective: every rank constructs it and calls :meth:`step` together.

    ``n_paths`` znodes ``/ens/pNNNNN``; a step sets ``writes`` of them
    (each exactly once, new data ``s<step>``) and ticks the fan-out until
    every rank received every resulting event.  Every ``failover_every``-th
    step the writes are made by the ensemble itself while the member rank 0
    is on is down (:meth:`EnsembleControl.outage`): rank 0's session (and
    any other session on that member) fails over, resumes its watches with
    SET_WATCHES and the server replays the missed changes, which the owners
    forward like any other event.  :meth:`verify` checks that every rank saw
    every event (initial arm, live and replayed) exactly once.

    ``ctl`` is the :class:`EnsembleControl` on rank 0 (None elsewhere);
    the member ports are broadcast from rank 0."""

    def __init__(self, ctl=None, n_members=3, n_paths=256, writes=64,
                 failover_every=4, session_timeout=8000, codec_device=None,
                 group=None, seed=0, coll_device=None):
        from ..models.client import Client
        from ..config import ClientConfig, RecoveryPolicy
        on = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if on else 1
        self.rank = dist.get_rank(group) if on else 0
        self.ctl = ctl
        self.group = group
        backend = dist.get_backend(group) if on else None
        if coll_device is None:
            coll_device = torch.device(
                'cuda', torch.cuda.current_device()) \
                if backend == 'nccl' else torch.device('cpu')
        self.coll = cd = torch.device(coll_device)
        ports = _bcast_ints(ctl.ports if ctl else None, n_members, 0, cd)
        self.ports = ports
        n = len(ports)
        me = self.rank % n
        servers = [{'address': '127.0.0.1', 'port': ports[(me + k) % n]}
                   for k in range(n)]
        cfg = ClientConfig(
            ping_floor_ms=500, ping_timeout_floor_ms=2000,
            connect_policy=RecoveryPolicy(1000, 3, 50, 400),
            default_policy=RecoveryPolicy(1000, 3, 100, 800),
            codec_device=str(codec_device) if codec_device else None)
        self.connects = 0
        self._lk = threading.Lock()
        # signalled by every event an owner's watcher emits: the fan-out
        # waits on it instead of polling on a timer
        self._ev = threading.Condition(self._lk)
        self._connected = threading.Event()

        def on_connect():
            with self._lk:
                self.connects += 1
            self._connected.set()
        self.client = Client({'servers': servers,
                              'sessionTimeout': session_timeout,
                              'config': cfg,
                              'listeners': [('connect', on_connect)]})
        self.client.wait_connected(20)
        self.paths = ['/ens/p%05d' % k for k in range(n_paths)]
        self.writes = min(writes, n_paths)
        self.failover_every = failover_every
        self.seed = seed
        self.fan = WireFanout(group, decode_device=codec_device)
        self.pending = []
        self.seen = collections.Counter()
        self.expected = set()
        self.replayed = set()
        self.step_no = 0
        self.failovers = 0
        self.down = None
        if self.rank == 0:
            self._create_tree()
        self._barrier()
        self.mine = [p for p in self.paths
                     if owner_of(p, self.world) == self.rank]
        for p in self.mine:
            self.client.watcher(p).on(
                'dataChanged', lambda d, s, p=p: self._on_event(p, d, s))
        self.expected.update((p, b'init') for p in self.paths)
        self._deliver_until(len(self.paths), mine=len(self.mine))

    # -- plumbing -------------------------------------------------------------

    def _barrier(self):
        if self.world > 1:
            dist.barrier(group=self.group)

    def _create_tree(self):
        c = self.client
        c.call_sync('create', '/ens', b'', {})
        left = [len(self.paths)]
        done = threading.Event()
        errs = []

        def cb(err, *_):
            if err is not None:
                errs.append(err)
            left[0] -= 1
            if left[0] == 0:
                done.set()

        def go():
            for p in self.paths:
                c.create(p, b'init', {}, cb)
        c.loop.run(go)
        if not done.wait(60) or errs:
            raise RuntimeError('ensemble tree create failed: %r' % errs[:3])

    def _on_event(self, path, data, stat):
        with self._lk:
            self.pending.append((path, data, stat))
            self._ev.notify_all()

    def _deliver_until(self, want, timeout=60.0, mine=None):
        """Tick the fan-out until every rank has received ``want`` events
        (collective; the stop decision is all-reduced).  Returns the number
        this rank received.  ``mine``: the events this rank's watchers will
        emit — each round first waits (on the event condition, no polling)
        until they are all pending or a tick (5 ms) passes, so a step is
        usually ONE exchange."""
        got = 0
        t_end = time.monotonic() + timeout
        # [not done, timed out], all-reduced with MAX: every rank stops
        # together, and a rank's timeout makes every rank raise (none is
        # left waiting in the next collective)
        flag = torch.zeros(2, dtype=torch.int64, device=self.coll)
        sent = 0
        while True:
            with self._lk:
                if mine is not None:
                    self._ev.wait_for(
                        lambda: sent + len(self.pending) >= mine, 0.005)
                batch = self.pending[:KMAX]
                del self.pending[:KMAX]
            sent += len(batch)
            for src, path, data, stat in self.fan.exchange(batch):
                self.seen[(path, data)] += 1
                got += 1
            flag[0] = 0 if got >= want else 1
            flag[1] = 1 if time.monotonic() > t_end else 0
            if self.world > 1:
                dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=self.group)
            busy, late = flag.tolist()
            if not busy:
                return got
            if late:
                raise RuntimeError('fan-out: %d of %d events after %.0f s '
                                   '(on this rank or another)'
                                   % (got, want, timeout))

    def _choose(self, s):
        rng = np.random.default_rng(self.seed * 1000003 + s)
        return [self.paths[k] for k in rng.choice(len(self.paths),
                                                  self.writes,
                                                  replace=False)]

    def _member(self):
        def go():
            conn = self.client.getSession().getConnection()
            return -1 if conn is None else conn.server['port']
        port = self.client.loop.run(go)
        return self.ports.index(port) if port in self.ports else -1

    # -- one step -------------------------------------------------------------

    def step(self):
        """One step (collective); returns the events this rank received."""
        s = self.step_no
        self.step_no += 1
        data = b's%d' % s
        chosen = self._choose(s)
        self.expected.update((p, data) for p in chosen)
        fail = self.failover_every and (s % self.failover_every ==
                                        self.failover_every - 1)
        if fail:
            before = self.connects
            mine_m = self._member()
            self._barrier()
            m = None
            if self.rank == 0:
                m = mine_m
                if self.down is not None:
                    self.ctl.start(self.down)       # the last victim is back
                self.ctl.outage(m, [(p, data) for p in chosen])
                self.down = m
            m = _bcast_ints([m] if m is not None else None, 1, 0,
                            self.coll)[0]
            self.replayed.update((p, data) for p in chosen)
            self.failovers += 1
            # every session on the killed member reconnects and replays
            if mine_m == m:
                t_end = time.monotonic() + 30
                while self.connects <= before:
                    if time.monotonic() > t_end:
                        raise RuntimeError('rank %d: no failover' % self.rank)
                    time.sleep(0.005)
        else:
            mine = chosen[self.rank::self.world]
            self._set_all(mine, data)
        self._barrier()
        mine = sum(1 for p in chosen if owner_of(p, self.world) == self.rank)
        return self._deliver_until(len(chosen), mine=mine)

    def _set_all(self, paths, data):
        if not paths:
            return
        c = self.client
        left = [len(paths)]
        done = threading.Event()
        errs = []

        def cb(err, *_):
            if err is not None:
                errs.append(err)
            left[0] -= 1
            if left[0] == 0:
                done.set()

        def go():
            for p in paths:
                c.set(p, data, -1, cb)
        c.loop.run(go)
        if not done.wait(30) or errs:
            raise RuntimeError('set failed: %r' % errs[:3])

    def rearmed(self):
        """Watches this rank's session re-armed through SET_WATCHES."""
        return self.client.loop.run(lambda: self.client.getSession().rearmed)

    def verify(self):
        """Every expected (path, data) seen exactly once on this rank, and
        nothing else.  Returns a problem description or None."""
        extra = [k for k in self.seen if k not in self.expected]
        dup = [k for k, v in self.seen.items() if v != 1]
        miss = [k for k in self.expected if self.seen.get(k, 0) == 0]
        if extra or dup or miss:
            return {'missing': miss[:5], 'dup': dup[:5], 'extra': extra[:5],
                    'n_missing': len(miss), 'n_dup': len(dup)}
        return None

    def close(self):
        try:
            self.client.close_sync(10)
        except Exception:                           # noqa: BLE001
            pass
