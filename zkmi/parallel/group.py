"""Node-level layer: one ZooKeeper session per rank (one process per GPU),
coordinated with collectives over ``torch.distributed`` — RCCL over xGMI
on MI355X (backend ``"nccl"``), gloo on CPU.

The reference has no collectives; its "parallelism" is request pipelining on
one connection, a connection set over an ensemble and session migration
(SURVEY §2.5).  Scaled to a node of 8 GPUs, each rank owns a session and the
group adds:

  R1 :class:`DistributedWatcher` — watch fan-out.  One rank (the path's
     owner, ``crc32(path) % world``) holds the real server watch; every
     other rank receives the owner's events (with the re-fetched data and
     Stat, so nobody re-reads).  8 sessions watching one hot path cost the
     ensemble 1 watch instead of 8.  The events travel as ZooKeeper wire
     frames — a NOTIFICATION and the reply of the owner's re-fetch — through
     :class:`~zkmi.parallel.fanout.FrameFanout`, the one R1 path (the bulk
     watches of config 4 and the GPU server's watch pipeline use it too),
     and every rank decodes the gathered stream (K1 + K2-K8 on its GPU).
  R2 :meth:`SessionGroup.batched_get` — request batching: ranks pool their
     reads, duplicates are dropped, each unique path is fetched once by one
     rank over its own session, results are exchanged.
  R3 :meth:`SessionGroup.broadcast_session` — session credentials (and the
     watch set) shared for failover / migration between ranks: a surviving
     rank can resume a dead rank's session, keeping its ephemerals.
  R4 :meth:`SessionGroup.allreduce_metrics` — node-level sums of the
     ``zookeeper_events`` / ``zookeeper_notifications`` counters.

Message sizes are tiny and latency-bound (tens of bytes per event), so
events are batched per :meth:`SessionGroup.tick` and moved with one
variable-size all-gather (sizes first, then a padded payload) rather than
per-event collectives.  Payloads are Jute-encoded records.
"""

import collections
import threading

import torch
import torch.distributed as dist

from .. import jute
from .fanout import FWD_XIDS, FrameFanout, owner_of
from ..utils.metrics import METRIC_ZK_EVENT_COUNTER, \
    METRIC_ZK_NOTIFICATION_COUNTER

METRIC_SCHEMA = (
    [(METRIC_ZK_EVENT_COUNTER, {'evtype': e})
     for e in ('session', 'connect', 'failed')] +
    [(METRIC_ZK_NOTIFICATION_COUNTER, {'event': e})
     for e in ('created', 'deleted', 'dataChanged', 'childrenChanged')])

_KINDS = ('created', 'deleted', 'dataChanged', 'childrenChanged')
# event kind <-> (notification type, the forwarded reply's opcode)
_NOTE_TYPE = {'created': 'CREATED', 'deleted': 'DELETED',
              'dataChanged': 'DATA_CHANGED',
              'childrenChanged': 'CHILDREN_CHANGED'}
_KIND_OF = {v: k for k, v in _NOTE_TYPE.items()}
_FWD_OF = {op: x for x, op in FWD_XIDS.items()}


class SessionGroup(object):
    """Wraps a per-rank :class:`~zkmi.Client` and a process group."""

    def __init__(self, client, group=None, device=None):
        if not dist.is_initialized():
            raise RuntimeError('torch.distributed must be initialised')
        self.client = client
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        backend = dist.get_backend(group)
        if device is None:
            device = torch.device('cuda', torch.cuda.current_device()) \
                if backend == 'nccl' else torch.device('cpu')
        self.device = torch.device(device)
        self._pending = collections.deque()
        self._lock = threading.Lock()
        self._watchers = {}
        self.stats = collections.Counter()
        # R1: frames decoded on this rank's GPU when the collectives run
        # there, by the host codec otherwise
        self.fan = FrameFanout(group, device=self.device
                               if self.device.type == 'cuda' else None,
                               coll_device=self.device)

    # -- low level: variable-size all-gather of byte strings --------------

    def _allgather_bytes(self, payload):
        """Variable-size all-gather: one size exchange (a single host read
        of the world's sizes), one padded payload all-gather, one copy of
        the gathered block to the host."""
        dev = self.device
        W = self.world
        n = torch.tensor([len(payload)], dtype=torch.int64, device=dev)
        sizes_t = torch.empty(W, dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(sizes_t, n, group=self.group)
        sizes = sizes_t.cpu().tolist()
        mx = max(max(sizes), 1)
        buf = torch.zeros(mx, dtype=torch.uint8, device=dev)
        if payload:
            buf[:len(payload)] = torch.frombuffer(bytearray(payload),
                                                  dtype=torch.uint8).to(dev)
        outs = torch.empty(W * mx, dtype=torch.uint8, device=dev)
        dist.all_gather_into_tensor(outs, buf, group=self.group)
        self.stats['allgather_bytes'] += sum(sizes)
        host = outs.cpu().numpy().tobytes()
        return [host[r * mx:r * mx + s] for r, s in enumerate(sizes)]

    def _broadcast_bytes(self, payload, src):
        dev = self.device
        n = torch.tensor([len(payload) if self.rank == src else 0],
                         dtype=torch.int64, device=dev)
        dist.broadcast(n, src, group=self.group)
        m = int(n.item())
        buf = torch.zeros(max(m, 1), dtype=torch.uint8, device=dev)
        if self.rank == src and m:
            buf[:m] = torch.frombuffer(bytearray(payload),
                                       dtype=torch.uint8).to(dev)
        dist.broadcast(buf, src, group=self.group)
        return bytes(buf[:m].cpu().numpy().tobytes())

    # -- R4 -----------------------------------------------------------------

    def allreduce_metrics(self, extra=None):
        """Sum the standard counters (plus ``extra`` = {name: int}) over the
        node.  Returns {'metric{labels}': total}."""
        vec = self.client.collector.as_vector(METRIC_SCHEMA)
        names = ['%s{%s}' % (n, ','.join('%s="%s"' % kv
                                         for kv in sorted(l.items())))
                 for n, l in METRIC_SCHEMA]
        for k in sorted(extra or {}):
            names.append(k)
            vec.append(int(extra[k]))
        t = torch.tensor(vec, dtype=torch.int64, device=self.device)
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return dict(zip(names, t.cpu().tolist()))

    # -- R3 -----------------------------------------------------------------

    def broadcast_session(self, src):
        """Every rank receives rank ``src``'s session credentials and its
        armed watch paths: {'sessionId', 'passwd', 'lastZxid', 'timeout',
        'watches': {kind: [paths]}}."""
        payload = b''
        if self.rank == src:
            cred = self.client.credentials()
            w = jute.JuteWriter()
            w.write_long(cred['sessionId'])
            w.write_buffer(cred['passwd'])
            w.write_long(cred['lastZxid'])
            w.write_int(cred['timeout'])
            watches = self.client.loop.run(self._watch_paths)
            for k in ('dataChanged', 'createdOrDeleted', 'childrenChanged'):
                w.write_string_vector(watches.get(k, []))
            payload = w.getvalue()
        raw = self._broadcast_bytes(payload, src)
        r = jute.JuteReader(raw)
        out = {'sessionId': r.read_long(), 'passwd': r.read_buffer(),
               'lastZxid': r.read_long(), 'timeout': r.read_int()}
        out['watches'] = {k: r.read_string_vector() for k in (
            'dataChanged', 'createdOrDeleted', 'childrenChanged')}
        return out

    def _watch_paths(self):
        res = {}
        for path, w in self.client.getSession().watchers.items():
            for ev in w.events():
                if not ev.isInState('disarmed'):
                    res.setdefault(ev.getEvent(), []).append(path)
        return res

    # -- R2 -----------------------------------------------------------------

    def batched_get(self, paths, timeout=30.0):
        """Collective: every rank passes its own list; returns
        [(data, stat) | ZKError] in that order.  Each unique path is read
        once on the node, by its owner rank."""
        w = jute.JuteWriter()
        w.write_string_vector(list(paths))
        lists = [jute.JuteReader(b).read_string_vector()
                 for b in self._allgather_bytes(w.getvalue())]
        uniq = sorted(set(p for lst in lists for p in lst))
        mine = [p for p in uniq if owner_of(p, self.world) == self.rank]
        self.stats['batched_get_unique'] += len(uniq)
        self.stats['batched_get_requested'] += sum(len(x) for x in lists)
        # never raise between the two collectives: a rank that left here
        # would leave every other rank blocked in the second all-gather
        try:
            results = self._fetch_all(mine, timeout)
        except Exception as e:                  # noqa: BLE001
            results = {p: e for p in mine}
        out = jute.JuteWriter()
        out.write_int(len(mine))
        for p in mine:
            out.write_ustring(p)
            res = results[p]
            if isinstance(res, Exception):
                out.write_ustring(getattr(res, 'code', 'SYSTEM_ERROR'))
            else:
                out.write_ustring('OK')
                out.write_buffer(res[0])
                out.write_stat(res[1])
        table = {}
        for blob in self._allgather_bytes(out.getvalue()):
            r = jute.JuteReader(blob)
            for _ in range(r.read_int()):
                p = r.read_ustring()
                code = r.read_ustring()
                if code == 'OK':
                    table[p] = (r.read_buffer(), r.read_stat())
                else:
                    from ..errors import ZKError
                    from .. import consts
                    table[p] = ZKError(code, consts.ERR_TEXT.get(code, ''))
        return [table[p] for p in paths]

    def _fetch_all(self, paths, timeout):
        """Pipeline all reads on this rank's session at once."""
        done = threading.Event()
        res = {}
        if not paths:
            return res
        left = [len(paths)]

        def mk(p):
            def cb(err, data=None, stat=None):
                res[p] = err if err is not None else (data, stat)
                left[0] -= 1
                if left[0] == 0:
                    done.set()
            return cb

        def go():
            for p in paths:
                self.client.get(p, mk(p))
        self.client.loop.run(go)
        if not done.wait(timeout):
            # the paths still outstanding fail with OPERATION_TIMEOUT; the
            # collective goes on (late callbacks only overwrite res entries)
            from ..errors import ZKError
            from .. import consts
            err = ZKError('OPERATION_TIMEOUT',
                          consts.ERR_TEXT.get('OPERATION_TIMEOUT', ''))
            return {p: res.get(p, err) for p in paths}
        return res

    # -- R1 -----------------------------------------------------------------

    def watcher(self, path):
        """A node-wide watcher for ``path`` (see :class:`DistributedWatcher`).
        Must be created on every rank (collective registration)."""
        w = self._watchers.get(path)
        if w is None:
            w = DistributedWatcher(self, path)
            self._watchers[path] = w
        return w

    def _publish(self, kind, path, args):
        """An owner's watcher event as two wire frames: the NOTIFICATION
        and the reply the watcher's re-fetch got (GET_DATA for dataChanged,
        GET_CHILDREN2 for childrenChanged, EXISTS for created; an EXISTS
        NO_NODE for deleted), its xid the forwarding xid of that opcode."""
        note = jute.encode_response({
            'xid': -1, 'zxid': -1, 'err': 'OK', 'opcode': 'NOTIFICATION',
            'type': _NOTE_TYPE[kind], 'state': 'SYNC_CONNECTED',
            'path': path})
        if kind == 'dataChanged':
            rep = {'opcode': 'GET_DATA', 'data': args[0], 'stat': args[1]}
        elif kind == 'childrenChanged':
            rep = {'opcode': 'GET_CHILDREN2', 'children': args[0],
                   'stat': args[1]}
        elif kind == 'created':
            rep = {'opcode': 'EXISTS', 'stat': args[0]}
        else:
            rep = {'opcode': 'EXISTS', 'err': 'NO_NODE'}
        rep['xid'] = _FWD_OF[rep['opcode']]
        rep['zxid'] = -1
        with self._lock:
            self._pending.append(jute.frame(note) +
                                 jute.frame(jute.encode_response(rep)))

    def tick(self):
        """Collective: exchange every rank's pending watch events and deliver
        them to local listeners, in owner order then arrival order.
        Returns the number of events delivered on this rank."""
        with self._lock:
            batch = list(self._pending)
            self._pending.clear()
        g = self.fan.gather(b''.join(batch), 2 * len(batch))
        pk = self.fan.decode_packets(g)
        n = 0
        for i in range(0, len(pk), 2):
            note, rep = pk[i], pk[i + 1]
            kind = _KIND_OF[note['type']]
            if kind == 'dataChanged':
                args = (rep['data'], rep['stat'])
            elif kind == 'childrenChanged':
                args = (rep['children'], rep['stat'])
            elif kind == 'created':
                args = (rep['stat'],)
            else:
                args = ()
            dw = self._watchers.get(note['path'])
            if dw is not None:
                dw._deliver(kind, args)
                n += 1
        self.stats['events_delivered'] += n
        return n


class DistributedWatcher(object):
    """Node-wide watcher: the owner rank arms the real ZooKeeper watch with
    its session; listeners on every rank get the events after the next
    :meth:`SessionGroup.tick`."""

    def __init__(self, group, path):
        self.group = group
        self.path = path
        self.owner = owner_of(path, group.world)
        self._listeners = collections.defaultdict(list)
        self._armed = set()

    @property
    def is_owner(self):
        return self.owner == self.group.rank

    def on(self, evt, cb):
        if evt not in _KINDS:
            raise ValueError('unknown watch event %r' % (evt,))
        self._listeners[evt].append(cb)
        if self.is_owner and evt not in self._armed:
            self._armed.add(evt)
            zw = self.group.client.watcher(self.path)
            zw.on(evt, lambda *a, e=evt: self.group._publish(e, self.path,
                                                             a))
        return self

    def _deliver(self, kind, args):
        for cb in list(self._listeners.get(kind, ())):
            cb(*args)
