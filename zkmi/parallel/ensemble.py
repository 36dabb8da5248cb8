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

The ensemble is the native server with ``--members 3`` (one tree, three
ports, fakezk's fault commands; ``csrc/host/zk_fastserver.cpp``) in a child
process started before anything touches the GPU.  Per rank: a
:class:`~zkmi.Client` on the ensemble (rank ``r`` prefers member ``r % n``)
whose (re)connects run K9 and its watch resume K11 on the GPU
(``ClientConfig.codec_device``).  Each path has one owner rank
(``owner_of``) holding the only server watch on it, as a bulk watch
(:meth:`~zkmi.Client.watch_bulk`): the native loop keeps the notification
frames, the owner re-arms them with ONE bulk GET_DATA(watch) per tick (K10
encode on the GPU, replies captured in pinned memory, K1 + K2-K8 decode),
and forwards the raw notification + reply frames with
:class:`~zkmi.parallel.fanout.FrameFanout` (R1).  Every rank decodes the
node's stream on its GPU and counts each (path, version) event in HBM; no
event becomes a Python object on the way.  Writes go out as bulk SET_DATA
batches.  Without a GPU (the gloo rehearsal on CPU) the same flow runs on
the host codec.

Exactly once: a watch's catch-up can reach its owner twice.  When the
client's connection set moves a session again while the first resume's
SET_WATCHES is still unanswered (e.g. back to its preferred member as soon
as that member restarts), the second SET_WATCHES carries the same relZxid
— the catch-up notifications carry no zxid that could have advanced it —
and the member replays the same changes.  A ZooKeeper client drops such a
repeat because the fired watch is gone from its watch table; bulk watches
stay armed on the client, so the owner drops it by version instead: the
re-arm read of a change it already forwarded returns a version no newer
than the one it forwarded (:meth:`EnsembleWorkload._rearm`).
"""

import collections
import threading
import time

import numpy as np
import torch
import torch.distributed as dist

from .. import codec
from .. import consts
from ..errors import ZKProtocolError
from .fanout import FrameFanout, XID_FWD, notification_frames, owner_of, \
    path_ids

__all__ = ['EnsembleControl', 'EnsembleWorkload', 'owner_of']

_DIGITS = 5                      # paths are /ens/pNNNNN


def _phased(t):
    """A bulk call's phase clock has every mark the split needs (the
    'captured' mark exists only when the native transport captured the
    batch; a per-frame or non-native path has none)."""
    return bool(t.get('submit')) and all(
        k in t for k in ('encoded', 'captured', 'finished'))


class EnsembleControl(object):
    """The ensemble as a child process — the native server with ``n``
    members (``zkmi.server.fast``), or with ``native=False`` the Python
    fake ensemble (``python -m zkmi.server --ensemble N``) — driven over its
    stdin fault-command channel: :meth:`outage`, :meth:`start`."""

    def __init__(self, n=3, tick_ms=250, native=True):
        from ..server import fast
        self.native = native and fast.available()
        if self.native:
            self.srv = fast.FastZKServer(members=n)
            self.ports = list(self.srv.ports)
            return
        import subprocess
        import sys
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
        """Member ``i`` down, then ``sets`` = [(path, data)] applied while
        its sessions are detached; returns the zxid after them."""
        if self.native:
            return self.srv.outage(i, sets)
        return int(self._cmd('outage %d %s' % (i, ' '.join(
            '%s=%s' % (p, d.hex()) for p, d in sets))))

    def start(self, i):
        if self.native:
            self.srv.start(i)
        else:
            self._cmd('start %d' % i)

    def close(self):
        if self.native:
            self.srv.shutdown()
            return
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


def _batch_prior_max(key, val):
    """For each entry i: the largest ``val`` of the entries before it in the
    batch with the same ``key`` (-1: none) — a segmented exclusive running
    max on the device: a stable sort by key, then one cummax over
    ``segment * 2**32 + val`` (segments ascend, so the max never crosses
    into the next segment; val in [-1, 2**31))."""
    n = key.numel()
    if n == 0:
        return val.clone()
    ks, order = torch.sort(key, stable=True)
    seg = torch.cumsum((ks[1:] != ks[:-1]).to(torch.int64), 0)
    seg = torch.cat([seg.new_zeros(1), seg])
    v = val[order] + 1                        # >= 0
    run = torch.cummax(seg * (1 << 32) + v, 0).values - seg * (1 << 32)
    prior = torch.cat([run.new_zeros(1), run[:-1]])
    start = torch.cat([torch.ones(1, dtype=torch.bool, device=key.device),
                       ks[1:] != ks[:-1]])
    prior = torch.where(start, torch.zeros_like(prior), prior) - 1
    out = torch.empty_like(prior)
    out[order] = prior
    return out


def _patch_xids(raw):
    """Host path: reply frames with their xids set to XID_FWD."""
    b = bytearray(raw)
    frames, _, _ = codec.scan_frames(bytes(b), 0, len(b), consts.MAX_PACKET)
    x = XID_FWD.to_bytes(4, 'big')
    for o, _ in frames:
        b[o:o + 4] = x
    return bytes(b)


class EnsembleWorkload(object):
    """Collective: every rank constructs it and calls :meth:`step` together.

    ``n_paths`` znodes ``/ens/pNNNNN``; a step sets ``writes`` of them (each
    exactly once) and ticks the fan-out until every rank received every
    resulting event.  Every ``failover_every``-th step the writes are made
    by the ensemble itself while the member rank 0 is on is down
    (:meth:`EnsembleControl.outage`): rank 0's session (and any other
    session on that member) fails over, resumes its watches with
    SET_WATCHES and the server replays the missed changes, which the owners
    forward like any other event.  Each event is identified by (path,
    version); :meth:`verify` checks that every rank saw every one (initial
    arm, live and replayed) exactly once.  ``max_versions`` bounds the
    writes per path the check can count.

    ``ctl`` is the :class:`EnsembleControl` on rank 0 (None elsewhere); the
    member ports are broadcast from rank 0."""

    def __init__(self, ctl=None, n_members=3, n_paths=256, writes=64,
                 failover_every=4, session_timeout=8000, codec_device=None,
                 group=None, seed=0, coll_device=None, max_versions=64,
                 trace=False):
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
        # (a member that went down is retried after 5 ms, not the 50-100
        # ms of an interactive client: the failover is the measured step.
        # A ping may wait up to 3/4 of the session timeout: a busy host
        # that stalls the client's loop for a second or two must not fail
        # a healthy connection over — that extra move would resume the
        # session's watches at a lastZxid older than events it had already
        # forwarded, and the member would replay them a second time.)
        cfg = ClientConfig(
            ping_floor_ms=500,
            ping_timeout_floor_ms=max(2000, session_timeout * 3 // 4),
            connect_policy=RecoveryPolicy(1000, 3, 5, 100),
            default_policy=RecoveryPolicy(1000, 3, 5, 100),
            codec_device=str(codec_device) if codec_device else None)
        self.dev = torch.device(codec_device) if codec_device else None
        if self.dev is not None and self.dev.type != 'cuda':
            self.dev = None
        self.connects = 0
        self._lk = threading.Lock()
        self._connected = threading.Event()

        def on_connect():
            with self._lk:
                self.connects += 1
            self._connected.set()
        self.client = Client({'servers': servers,
                              'sessionTimeout': session_timeout,
                              'config': cfg,
                              'device': self.dev if self.dev else False,
                              'listeners': [('connect', on_connect)]})
        self.client.wait_connected(20)
        self.paths = ['/ens/p%05d' % k for k in range(n_paths)]
        self.writes = min(writes, n_paths)
        self.failover_every = failover_every
        self.seed = seed
        self.fan = FrameFanout(group, device=self.dev)
        # (path, version) events: expected and seen, per rank
        self.vmax = max_versions
        self.version = np.zeros(n_paths, np.int64)      # last write's
        self.expected = np.zeros(n_paths * self.vmax, np.int32)
        dev = self.dev if self.dev is not None else torch.device('cpu')
        self.seen = torch.zeros(n_paths * self.vmax, dtype=torch.int32,
                                device=dev)
        self.bad_frames = torch.zeros(1, dtype=torch.int64, device=dev)
        # the newest version this rank forwarded per path it owns (-1: none)
        # and the repeats it dropped (module docstring)
        self.fwd_ver = np.full(n_paths, -1, np.int64)
        self.fwd_ver_dev = torch.from_numpy(self.fwd_ver.copy()).to(
            self.dev) if self.dev is not None else None
        self.redelivered = 0
        self.replayed = 0                 # writes made during outages
        self.step_ms = []
        self.phase_ms = collections.Counter()     # where a step's time goes
        self.step_no = 0
        # trace: (step, tick, paths this rank forwarded) per host-path tick
        self.trace = [] if trace else None
        self.failovers = 0
        self.down = None
        if self.rank == 0:
            self._create_tree()
        self._barrier()
        self.owner = np.array([owner_of(p, self.world) for p in self.paths],
                              np.int32)
        self.mine = [p for p, o in zip(self.paths, self.owner)
                     if o == self.rank]
        self.client.watch_bulk(self.mine)
        self.expected[np.arange(n_paths) * self.vmax] = 1
        # the initial values go out like every later event: a notification
        # (type -1: none) + the reply of the read that armed the watch
        notes = notification_frames(self.mine)
        self._deliver_until(len(self.paths), initial=(notes, self.mine))

    # -- plumbing -------------------------------------------------------------

    def _barrier(self):
        if self.world > 1:
            dist.barrier(group=self.group)

    def _bulk(self, call, *args, timeout=60.0, retry=False, **kw):
        """One bulk batch, blocking.  ``retry``: an idempotent batch (the
        re-arming reads) that failed because the session was between
        connections is sent again once it is connected (ZooKeeper fails a
        request with CONNECTION_LOSS during a move; the caller retries)."""
        for attempt in range(4 if retry else 1):
            done = threading.Event()
            box = {}

            def cb(err, res=None):
                box['err'], box['res'] = err, res
                done.set()
            try:
                call(*args, cb, **kw)
            except ZKProtocolError as e:
                box['err'] = e
                done.set()
            if not done.wait(timeout):
                raise RuntimeError('bulk batch timed out')
            err = box['err']
            if err is None:
                return box['res']
            if not retry or attempt == 3 or \
                    getattr(err, 'code', None) != 'CONNECTION_LOSS':
                raise err
            self.client.wait_connected(timeout)
        raise AssertionError('unreachable')

    def _create_tree(self):
        c = self.client
        c.call_sync('create', '/ens', b'', {})
        acl = [{'perms': ['READ', 'WRITE', 'CREATE', 'DELETE', 'ADMIN'],
                'id': {'scheme': 'world', 'id': 'anyone'}}]
        res = self._bulk(c.bulk, [{'opcode': 'CREATE', 'path': p,
                                   'data': b'init', 'acl': acl}
                                  for p in self.paths])
        bad = [e for e in res.errors() if e != 'OK']
        if bad:
            raise RuntimeError('ensemble tree create failed: %r' % bad[:3])

    def _rearm(self, notes, k):
        """The owner side of one tick: the ``k`` notification frames in
        ``notes`` re-armed with one bulk GET_DATA(watch); returns the
        forwardable stream [notifications][replies] and its frame count."""
        if k == 0:
            return b'', 0
        if self.dev is None:
            frames, _, _ = codec.scan_frames(notes, 0, len(notes),
                                             consts.MAX_PACKET)
            paths = [codec.decode_response(notes[o:o + ln], {})['path']
                     for o, ln in frames]
            res = self._bulk(self.client.bulk_get, paths, watch=True,
                             retry=True)
            raw = _patch_xids(res.raw)
            rf, _, _ = codec.scan_frames(raw, 0, len(raw), consts.MAX_PACKET)
            keep = []
            for i, pk in enumerate(res.packets()):
                st = pk.get('stat') if pk.get('err') == 'OK' else None
                if st is not None:
                    pid = int(paths[i][-_DIGITS:])
                    if st.version <= self.fwd_ver[pid]:
                        self.redelivered += 1         # forwarded already
                        continue
                    self.fwd_ver[pid] = st.version
                keep.append(i)
            if self.trace is not None:
                self.trace.append(('fwd', self.step_no,
                                   self.phase_ms['ticks'],
                                   [paths[i] for i in keep]))
            if len(keep) == k:
                return notes + raw, 2 * k
            return (b''.join(notes[frames[i][0] - 4:sum(frames[i])]
                             for i in keep) +
                    b''.join(raw[rf[i][0] - 4:sum(rf[i])] for i in keep),
                    2 * len(keep))
        from ..ops import batch as B
        nd = torch.frombuffer(bytearray(notes), dtype=torch.uint8) \
            .to(self.dev, non_blocking=True)
        ft = B.frame_scan(nd, len(notes), cap=k, window=B.frame_window(512))
        rep = B.decode_replies(nd, ft, self.fan.xt)
        triple = (nd, rep.pay_off[:k], rep.pay_len[:k])
        t0 = time.perf_counter()
        res = self._bulk(self.client.bulk_get, triple, watch=True, retry=True)
        ph = self.phase_ms
        ph['rearm_bulk_get'] += (time.perf_counter() - t0) * 1e3
        t = getattr(res, 'phases', None) or {}
        if _phased(t):
            ph['rb_encode'] += (t['encoded'] - t['submit']) * 1e3
            ph['rb_wire'] += (t['captured'] - t['encoded']) * 1e3
            ph['rb_finish'] += (t['finished'] - t['captured']) * 1e3
        fwd = self.fan.forward_replies(res)
        # the owner's dedup by version (module docstring), on the device
        rr = res.replies
        pid = path_ids(nd, rep.pay_off[:k], rep.pay_len[:k], _DIGITS) \
            .clamp(0, len(self.paths) - 1)
        ver = rr.stat32[0][:k].to(torch.int64)
        ok = (rr.status[:k] == 0) & (rr.err[:k] == 0)
        # a path twice in one batch (a replayed catch-up in the tick of the
        # original): the later copy is a repeat of the earlier one, as the
        # host path's entry-by-entry update sees it
        seen = _batch_prior_max(pid, torch.where(ok, ver, -1))
        dup = ok & (ver <= torch.maximum(self.fwd_ver_dev[pid], seen))
        self.fwd_ver_dev.scatter_reduce_(0, pid[ok], ver[ok], 'amax')
        ndup = int(dup.sum().item())
        if ndup == 0:
            return torch.cat([nd, fwd]), 2 * k
        self.redelivered += ndup
        keep = (~dup).nonzero().squeeze(1)

        def frames_of(buf, off, ln):
            # the kept frames' bytes, length prefixes included
            s0 = off[keep] - 4
            n = ln[keep].to(torch.int64) + 4
            base = torch.repeat_interleave(s0 - (torch.cumsum(n, 0) - n), n)
            return buf[base + torch.arange(int(n.sum().item()),
                                           device=buf.device)]
        return (torch.cat([frames_of(nd, ft.off[:k], ft.length[:k]),
                           frames_of(fwd, res.frames.off[:k],
                                     res.frames.length[:k])]),
                2 * (k - ndup))

    def _initial(self, notes, paths):
        res = self._bulk(self.client.bulk_get, list(paths), watch=True,
                         retry=True)
        for p in paths:                       # version 0 forwarded
            self.fwd_ver[int(p[-_DIGITS:])] = 0
        if self.fwd_ver_dev is not None:
            self.fwd_ver_dev.copy_(torch.from_numpy(self.fwd_ver))
        if self.dev is None:
            return notes + _patch_xids(res.raw), 2 * len(paths)
        nd = torch.frombuffer(bytearray(notes or b'\0'),
                              dtype=torch.uint8)[:len(notes)].to(self.dev)
        return torch.cat([nd, self.fan.forward_replies(res)]), 2 * len(paths)

    def _count(self, g):
        """Count the gathered events into ``seen``; returns how many."""
        nev = sum(g.frames) // 2
        if nev == 0:
            return 0
        if self.dev is None:
            pk = self.fan.decode(g)
            base = 0
            for src, f in enumerate(g.frames):
                m = f // 2
                for i in range(m):
                    nt, rp = pk[base + i], pk[base + m + i]
                    pid = int(nt['path'][-_DIGITS:])
                    if self.trace is not None:
                        self.trace.append((
                            'got', self.step_no, self.phase_ms['ticks'], src,
                            pid, rp['stat'].version if rp.get('stat')
                            else None))
                    ok = (nt['opcode'] == 'NOTIFICATION' and
                          rp['opcode'] == 'GET_DATA' and rp['err'] == 'OK')
                    if not ok:
                        self.bad_frames += 1
                        continue
                    v = min(rp['stat'].version, self.vmax - 1)
                    self.seen[pid * self.vmax + v] += 1
                base += f
            return nev
        ft, rep = self.fan.decode(g)
        nidx, ridx = FrameFanout.pair_index(g.frames, self.dev)
        pid = path_ids(g.buf, rep.pay_off[nidx], rep.pay_len[nidx], _DIGITS)
        ver = rep.stat32[0][ridx].to(torch.int64).clamp(0, self.vmax - 1)
        ok = (rep.opcode[nidx] == consts.OP_CODES['NOTIFICATION']) & \
             (rep.opcode[ridx] == consts.OP_CODES['GET_DATA']) & \
             (rep.status[ridx] == 0) & (rep.err[ridx] == 0) & \
             (rep.status[nidx] == 0)
        key = (pid.clamp(0, len(self.paths) - 1) * self.vmax + ver)[ok]
        self.seen.index_put_((key,), torch.ones_like(key, dtype=torch.int32),
                             accumulate=True)
        self.bad_frames += (~ok).sum()
        return nev

    def _deliver_until(self, want, timeout=60.0, mine=None, initial=None):
        """Tick the fan-out until every rank has received ``want`` events
        (collective; the stop decision is all-reduced).  ``mine``: the
        events this rank's notifications will bring — each tick first polls
        the transports' kept notifications until they are all in or a tick
        (5 ms) passes, so a step is usually ONE exchange."""
        got = 0
        t_end = time.monotonic() + timeout
        # [not done, timed out], all-reduced with MAX: every rank stops
        # together, and a rank's timeout makes every rank raise
        flag = torch.zeros(2, dtype=torch.int64, device=self.coll)
        have = 0
        ph = self.phase_ms
        while True:
            t0 = time.perf_counter()
            if initial is not None:
                stream, nf = self._initial(*initial)
                initial = None
            else:
                notes, k = self.client.take_notes()
                if mine is not None:
                    t_tick = time.monotonic() + 0.005
                    while have + k < mine and time.monotonic() < t_tick:
                        time.sleep(0.0002)
                        more, k2 = self.client.take_notes()
                        notes += more
                        k += k2
                have += k
                t1 = time.perf_counter()
                ph['notes_wait'] += (t1 - t0) * 1e3
                t0 = t1
                stream, nf = self._rearm(notes, k)
            t1 = time.perf_counter()
            ph['rearm'] += (t1 - t0) * 1e3
            g = self.fan.gather(stream, nf)
            t2 = time.perf_counter()
            ph['gather'] += (t2 - t1) * 1e3
            got += self._count(g)
            ph['count'] += (time.perf_counter() - t2) * 1e3
            ph['ticks'] += 1
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
        return rng.choice(len(self.paths), self.writes, replace=False)

    def _member(self):
        def go():
            conn = self.client.getSession().getConnection()
            return -1 if conn is None else conn.server['port']
        port = self.client.loop.run(go)
        return self.ports.index(port) if port in self.ports else -1

    # -- one step -------------------------------------------------------------

    def step(self):
        """One step (collective); returns the events this rank received."""
        t0 = time.perf_counter()
        try:
            return self._step()
        finally:
            self.step_ms.append((time.perf_counter() - t0) * 1e3)

    def _step(self):
        s = self.step_no
        self.step_no += 1
        data = b's%d' % s
        chosen = self._choose(s)
        self.version[chosen] += 1
        v = np.minimum(self.version[chosen], self.vmax - 1)
        np.add.at(self.expected, chosen * self.vmax + v, 1)
        cp = [self.paths[k] for k in chosen]
        t0 = time.perf_counter()
        fail = self.failover_every and (s % self.failover_every ==
                                        self.failover_every - 1)
        if fail:
            before = self.connects
            mine_m = self._member()
            self._barrier()
            m = None
            if self.rank == 0:
                m = mine_m
                t1 = time.perf_counter()
                if self.down is not None:
                    self.ctl.start(self.down)       # the last victim is back
                self.ctl.outage(m, [(p, data) for p in cp])
                self.down = m
                self.phase_ms['fo_outage'] += (time.perf_counter() - t1) * 1e3
            m = _bcast_ints([m] if m is not None else None, 1, 0,
                            self.coll)[0]
            self.replayed += len(cp)
            self.failovers += 1
            # every session on the killed member reconnects and replays
            if mine_m == m:
                t1 = time.perf_counter()
                t_end = time.monotonic() + 30
                while self.connects <= before:
                    if time.monotonic() > t_end:
                        raise RuntimeError('rank %d: no failover' % self.rank)
                    time.sleep(0.0002)
                self.phase_ms['fo_reconnect'] += \
                    (time.perf_counter() - t1) * 1e3
        else:
            mine = cp[self.rank::self.world]
            if mine:
                res = self._bulk(self.client.bulk_set, mine, data)
                t = getattr(res, 'phases', None) or {}
                if _phased(t):
                    ph = self.phase_ms
                    ph['wb_encode'] = ph.get('wb_encode', 0.0) + \
                        (t['encoded'] - t['submit']) * 1e3
                    ph['wb_wire'] = ph.get('wb_wire', 0.0) + \
                        (t['captured'] - t['encoded']) * 1e3
                    ph['wb_finish'] = ph.get('wb_finish', 0.0) + \
                        (t['finished'] - t['captured']) * 1e3
                bad = [e for e in res.errors() if e != 'OK']
                if bad:
                    raise RuntimeError('set failed: %r' % bad[:3])
        self.phase_ms['failover' if fail else 'write'] += \
            (time.perf_counter() - t0) * 1e3
        self._barrier()
        mine = int((self.owner[chosen] == self.rank).sum())
        return self._deliver_until(len(cp), mine=mine)

    def rearmed(self):
        """Watches this rank's session re-armed through SET_WATCHES."""
        return self.client.loop.run(lambda: self.client.getSession().rearmed)

    def verify(self):
        """Every expected (path, version) event seen exactly once on this
        rank, and nothing else.  Returns a problem description or None."""
        seen = self.seen.cpu().numpy()
        bad = int(self.bad_frames.item())
        miss = np.nonzero((self.expected > 0) & (seen == 0))[0]
        dup = np.nonzero(seen > 1)[0]
        extra = np.nonzero((self.expected == 0) & (seen > 0))[0]
        if len(miss) or len(dup) or len(extra) or bad:
            def name(i):
                return (self.paths[i // self.vmax], int(i % self.vmax))
            return {'missing': [name(i) for i in miss[:5]],
                    'dup': [name(i) for i in dup[:5]],
                    'extra': [name(i) for i in extra[:5]],
                    'n_missing': len(miss), 'n_dup': len(dup),
                    'bad_frames': bad}
        return None

    def close(self):
        try:
            self.client.close_sync(10)
        except Exception:                           # noqa: BLE001
            pass
