#!/usr/bin/env python3
"""zkmi headline benchmark (BASELINE.json): "ZK ops/sec (whole node) + p50
get() RTT, 1M-znode synthetic tree".

Default config (BASELINE.json configs[1]): batched get() over a 1M-znode
synthetic tree with the Jute-decode HIP kernels on each MI355X.
``--workload mix`` is configs[2] (create/set/delete with version CAS and ACL
encode on the same 1M-znode tree), ``--workload storm`` configs[4]
(EPHEMERAL|SEQUENTIAL create storm with per-step session expiry) and
``--workload watch`` the watch fan-out of configs[3] driven by real writes
(each rank's GPU server arms GET_DATA watches and fires them on SET_DATA;
the notifications of every rank are all-gathered over RCCL and decoded by
every rank; the value counts node-wide deliveries).  ``--workload chain``
pipelines create -> set -> get -> delete of each path inside ONE batch
(in-batch ordering of the GPU server, 4 ordered passes); ``--workload nest``
does createWithEmptyParents-style depth-3 creates, the parent's EXISTS and
the bottom-up deletes in one batch (parent / child order).
One step = one batch
of ``--batch`` GET_DATA requests per GPU pushed through the full ZooKeeper
wire path on the GPU (see zkmi/bench/synthetic.py): client request encode
(K10) -> server frame scan + request decode (K1, K12) -> tree lookup in HBM
-> server reply encode (K13) -> client frame scan + reply decode (K1,
K2-K4) -> on-device check of every reply.  Synthetic data: random 100-byte
node payloads, uniformly random node per request.

Each GPU serves its batch over ``--streams`` (default 2) pipelined
connections, each on its own HIP stream with its own buffers and xid table;
a step makes no device-to-host read (K1 reads every stream's length from
the device byte count its encoder produced), so the connections' kernels
overlap.

GET scale-out (the headline at N > 1): every rank holds the whole tree in
its HBM and serves its own sessions' reads from it, as every ZooKeeper
server answers reads from its own replica (1M znodes take ~0.4 GB of the
288 GB).  The same run then times ONE tree sharded by path hash over the
ranks, every read routed to the rank that owns its path (R2,
zkmi/parallel/sharded.py: per connection and step, two equal-split
``all_to_all_single`` over RCCL/xGMI, the request slots out and the reply
slots back) and reports it as ``sharded_value`` — the layout for trees past
one GPU's memory; ``--sharded`` makes that the headline instead.  With one
GPU there is one replica and the step is the local pipeline, HIP-graph
captured (``--force-route`` runs the multi-rank step over a one-rank RCCL
group and compares it with the local one).

One process per GPU: ``--gpus N`` without a torchrun environment starts the
N rank processes itself (before anything touches the GPU); under torchrun
the ranks come from the environment.  Per-GPU work is fixed (weak
scaling).  The whole-node aggregate (sum over ranks of ops / max-rank time)
is reported.
``p50_get_rtt_us`` is the interactive path: one blocking ``Client.get``
round trip over loopback TCP to the fake server running as its own process
(``python -m zkmi.server``, started before the GPU is touched), with the
client on the native epoll loop; reported for honesty about where the GPU
helps.  ``p50_get_rtt_us_evloop`` is the same round trip
through the callback API on the client's event loop (one get issued from
the previous one's callback), the way the single-threaded reference runs
``get(path, cb)``.
"""

import argparse
import gc
import json
import os
import statistics
import subprocess
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Reference point (locally measured, not published): the
# reference's own ZKDecodeStream frame+decode on one Xeon core, best case
# 0.51 M packets/s.  The reference publishes no headline number.
REF_PKTS_PER_S = 0.51e6


def start_rtt_server():
    """The fake ZooKeeper in a child process (a real ZooKeeper does not share
    the client's interpreter).  Started before any GPU call."""
    p = subprocess.Popen([sys.executable, '-m', 'zkmi.server'], cwd=ROOT,
                         stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                         text=True)
    line = p.stdout.readline().split()
    if len(line) != 2 or line[0] != 'PORT':
        p.kill()
        raise SystemExit('fake server did not start: %r' % line)
    return p, int(line[1])


def start_fast_server(nodes, data_bytes):
    """The native wire server (csrc/host/zk_fastserver.cpp) preloaded with
    the synthetic tree; None when it is not built."""
    from zkmi.server import fast
    if not fast.available():
        return None
    return fast.FastZKServer(preload=nodes, data_bytes=data_bytes)


def measure_bulk_tcp(port, nodes, batch, iters, dev, conns=1, srv=None):
    """``Client.bulk_get`` over loopback TCP to the native server: every
    batch is ``batch`` GET_DATA of random existing nodes split over
    ``conns`` sessions (one connection and one event loop each, all
    submitted at once), device-resident paths -> K10 -> pinned TX ->
    socket -> server -> native-loop capture into pinned RX -> K1 + K2-K8 on
    the GPU; every reply checked OK.  Returns (ops/s, ms per batch, phase
    ms): the mean over sessions of encode (K10 + D2H, on the loop thread),
    wire + server (sent -> last reply captured), finish (H2D + decode
    enqueued) and decode (the device finishing it).

    With ``srv`` (the FastZKServer) the wire + server phase is split by the
    server's own clock (CLOCK_MONOTONIC, the clock of perf_counter) over
    3 more batches after the timed ones: client send (socket write begun ->
    the server's first read), server span (first read -> last reply write)
    made of serve (frames decoded + replies built), socket (recv + send
    calls) and blocked (replies waiting for the client to drain the
    socket), and client capture (last reply write -> the native loop's
    capture of the batch delivered)."""
    import threading
    import numpy as np
    from zkmi import Client
    from zkmi.runtime.loop import new_loop
    loops = [new_loop() for _ in range(conns)]
    cs = [Client({'address': '127.0.0.1', 'port': port, 'device': dev,
                  'loop': lp}) for lp in loops]
    for c in cs:
        c.wait_connected(10)
    i = np.arange(nodes)
    paths = np.char.add(np.char.add('/bench/d', np.char.zfill(
        (i // 1000).astype(str), 6)), np.char.add('/n', np.char.zfill(
            i.astype(str), 9)))
    blob = ''.join(paths.tolist()).encode()
    plen = len(paths[0])
    arena = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev)
    per = batch // conns
    ln = torch.full((per,), plen, dtype=torch.int32, device=dev)
    phases = []

    def one(seed):
        g = torch.Generator(device=dev)
        g.manual_seed(seed)
        idx = torch.randint(0, nodes, (per * conns,), device=dev, generator=g)
        boxes = [[] for _ in cs]
        evs = [threading.Event() for _ in cs]
        for k, c in enumerate(cs):
            c.bulk_get((arena, idx[k * per:(k + 1) * per] * plen, ln),
                       lambda err, res=None, k=k: (boxes[k].append((err, res)),
                                                   evs[k].set()))
        for k, ev in enumerate(evs):
            if not ev.wait(120):
                raise SystemExit('bulk_get timed out')
            err, res = boxes[k][0]
            if err is not None:
                raise SystemExit('bulk_get failed: %r' % (err,))
            if res.ok_count() != per:
                raise SystemExit('bulk_get: %d of %d replies OK'
                                 % (res.ok_count(), per))
            t_done = time.perf_counter()
            p = res.phases
            if p:
                phases.append((p['encoded'] - p['submit'],
                               p['captured'] - p['sent'],
                               p['finished'] - p['captured'],
                               t_done - p['finished']))
                stamps.append(p)
    stamps = []
    one(0)                                   # warm-up (allocations)
    phases.clear()
    t0 = time.perf_counter()
    for k in range(iters):
        one(k + 1)
    el = time.perf_counter() - t0
    ph = None
    if phases:
        m = np.mean(np.array(phases), axis=0) * 1e3
        ph = {'encode_ms': m[0], 'wire_server_ms': m[1], 'finish_ms': m[2],
              'decode_wait_ms': m[3]}
    if srv is not None and ph is not None:
        split = []
        for k in range(3):
            stamps.clear()
            srv.timing(reset=True)
            one(iters + 1 + k)
            w = srv.timing()
            s0 = min(p['send0'] for p in stamps)
            cap = max(p['captured'] for p in stamps)
            ns = 1e-6
            split.append((
                (w['first_rx'] * 1e-9 - s0) * 1e3,
                (w['last_tx'] - w['first_rx']) * ns,
                w['serve_ns'] * ns, (w['recv_ns'] + w['send_ns']) * ns,
                w['blocked_ns'] * ns,
                (cap - w['last_tx'] * 1e-9) * 1e3,
                (cap - s0) * 1e3))
        m = np.median(np.array(split), axis=0)
        ph['wire_split_ms'] = {
            'client_send': m[0], 'server_span': m[1], 'server_serve': m[2],
            'server_socket': m[3], 'server_blocked': m[4],
            'client_capture': m[5], 'send_to_capture': m[6]}
    for c in cs:
        c.close_sync(10)
    return per * conns * iters / el, el / iters * 1e3, ph


def _create_quiet(c, path):
    """The RTT node (an earlier measurement may have made it)."""
    from zkmi import ZKError
    try:
        c.call_sync('create', path, b'x' * 100, {})
    except ZKError as e:
        if e.code != 'NODE_EXISTS':
            raise


def measure_rtt(port, n=2000):
    from zkmi import Client
    c = Client(address='127.0.0.1', port=port)
    c.wait_connected(10)
    _create_quiet(c, '/rtt')
    for _ in range(200):
        c.call_sync('get', '/rtt')
    lat = []
    for _ in range(n):
        t = time.perf_counter()
        c.call_sync('get', '/rtt')
        lat.append((time.perf_counter() - t) * 1e6)
    c.close_sync(10)
    lat.sort()
    return statistics.median(lat), lat[int(0.99 * len(lat))]


def measure_rtt_async(port, n=2000, warm=200):
    """get() round trips the way the reference measures them: the callback
    API on the client's event loop, each reply's callback issuing the next
    get (node-zkstream is single-threaded; there is no cross-thread wake in
    its get(path, cb)).  ``measure_rtt`` adds a caller-thread hop per call
    (``call_sync``) and is reported next to it."""
    import threading
    from zkmi import Client
    c = Client(address='127.0.0.1', port=port)
    c.wait_connected(10)
    _create_quiet(c, '/rtt_a')
    lat = []
    done = threading.Event()
    st = {'k': 0, 't': 0.0, 'err': None}

    def issue():
        st['t'] = time.perf_counter()
        c.get('/rtt_a', on_reply)

    def on_reply(err, data=None, stat=None):
        now = time.perf_counter()
        if err is not None:
            st['err'] = err
            done.set()
            return
        st['k'] += 1
        if st['k'] > warm:
            lat.append((now - st['t']) * 1e6)
        if st['k'] >= n + warm:
            done.set()
            return
        issue()
    c.loop.call_soon(issue)
    ok = done.wait(120)
    c.close_sync(10)
    if not ok or st['err'] is not None or not lat:
        raise RuntimeError('async RTT run failed: %r' % (st['err'],))
    lat.sort()
    return statistics.median(lat), lat[int(0.99 * len(lat))]


def measure_pipelined(port, n=200000, window=256):
    """Interactive get(path, cb) throughput: ``window`` requests in flight
    on the client's event loop, each reply's callback issuing the next —
    the per-request API (no bulk batch), so every reply goes through the
    connection's completion path one at a time."""
    import threading
    from zkmi import Client
    c = Client(address='127.0.0.1', port=port)
    c.wait_connected(10)
    _create_quiet(c, '/rtt_p')
    done = threading.Event()
    st = {'sent': 0, 'got': 0, 'err': None}

    def on_reply(err, data=None, stat=None):
        if err is not None:
            st['err'] = err
            done.set()
            return
        st['got'] += 1
        if st['got'] >= n:
            done.set()
            return
        if st['sent'] < n:
            st['sent'] += 1
            c.get('/rtt_p', on_reply)

    def start():
        for _ in range(min(window, n)):
            st['sent'] += 1
            c.get('/rtt_p', on_reply)
    t0 = time.perf_counter()
    c.loop.call_soon(start)
    ok = done.wait(300)
    el = time.perf_counter() - t0
    c.close_sync(10)
    if not ok or st['err'] is not None:
        raise RuntimeError('pipelined run failed: %r' % (st['err'],))
    return n / el


def run_ensemble(a):
    """BASELINE config 4 (zkmi/parallel/ensemble.py): 3-server ensemble,
    one session per rank, member failover with watch replay, every event
    fanned out to every rank (R1: wire frames all-gathered on the collective
    device, K1 + K2-K8 decoded on each GPU).  Value: watch-event deliveries
    per second over the node (events x ranks).  Runs without a GPU too
    (gloo rehearsal: host decode)."""
    from zkmi.parallel import ensemble as E
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    # the ensemble process starts before anything touches the GPU
    ctl = E.EnsembleControl(3) if rank == 0 else None
    backend = os.environ.get('ZKMI_BENCH_BACKEND', 'nccl')
    ndev = torch.cuda.device_count()
    if ndev == 0:
        backend, dev = 'gloo', None
    else:
        dev = torch.device('cuda', local % ndev if backend == 'gloo'
                           else local)
        torch.cuda.set_device(dev)
    if world > 1:
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=dev)
        else:
            dist.init_process_group('gloo')
    try:
        wl = E.EnsembleWorkload(ctl, n_paths=a.paths, writes=a.writes,
                                failover_every=a.failover_every,
                                max_versions=a.warmup + a.steps + 2,
                                codec_device=dev)
        for _ in range(a.warmup):
            wl.step()
        wl.phase_ms.clear()
        if world > 1:
            dist.barrier()
        if dev is not None:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        got = 0
        for _ in range(a.steps):
            got += wl.step()
        if world > 1:
            dist.barrier()
        if dev is not None:
            torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        bad = wl.verify()
        stats = torch.tensor([elapsed * 1e6, got, 1 if bad else 0,
                              wl.failovers, wl.rearmed(),
                              wl.fan.stats['decoded_gpu'],
                              wl.fan.stats['decoded_host']],
                             dtype=torch.float64, device=wl.coll)
        if world > 1:
            mx = stats[:1].clone()
            dist.all_reduce(mx, op=dist.ReduceOp.MAX)
            dist.all_reduce(stats, op=dist.ReduceOp.SUM)
            stats[0] = mx[0]
        el_us, total, nbad, fo, rep, dg, dh = stats.cpu().tolist()
        if nbad:
            raise SystemExit('ensemble: rank %d saw %r' % (rank, bad)
                             if bad else 'ensemble: a rank failed')
        codec_calls = wl.client.loop.run(
            lambda: dict(getattr(wl.client.getSession().getConnection(),
                                 'gpu', None).calls)
            if dev is not None else {})
        wl.close()
    finally:
        if ctl is not None:
            ctl.close()
    value = total / (el_us / 1e6)
    if rank == 0:
        print(json.dumps({
            'metric': 'ZK ops/sec (whole node) + p50 get() RTT, 1M-znode '
                      'synthetic tree',
            'value': value, 'unit': 'ops/s', 'n_gpus': world,
            'steps': a.steps, 'warmup': a.warmup,
            'ms_per_step': el_us / 1e3 / a.steps,
            'higher_is_better': True, 'scaling': 'weak',
            'vs_baseline': None, 'dtype': 'uint8', 'data': 'synthetic',
            'config': {'model': 'zk-ensemble 3-server failover + watch '
                                'replay, %d znodes' % a.paths,
                       'global_batch': a.writes, 'seq_len': 1,
                       'parallelism': 'dp%d' % world},
            'ops_note': 'watch-event deliveries over the node (every event '
                        'reaches every rank exactly once, checked)',
            'failovers': int(fo // world),
            'step_ms_rank0': [round(x, 2) for x in wl.step_ms],
            'phase_ms_rank0': {k: round(v, 2)
                               for k, v in wl.phase_ms.items()},
            'watches_rearmed_by_set_watches': int(rep),
            'events_decoded_on_gpu': int(dg),
            'events_decoded_on_host': int(dh),
            'rank0_gpu_codec_calls': codec_calls,
            'backend': backend if world > 1 else None}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--batch', type=int, default=1 << 20,
                    help='GET_DATA requests per GPU per step')
    ap.add_argument('--nodes', type=int, default=1_000_000)
    ap.add_argument('--data-bytes', type=int, default=100)
    ap.add_argument('--data-dist', default=None,
                    help='uniform:LO-HI: leaf data lengths uniform in LO..HI '
                         'bytes instead of --data-bytes (variable frames)')
    ap.add_argument('--name-pad', default=None,
                    help='LO-HI: leaf names padded by a uniform LO..HI '
                         'characters (variable path lengths)')
    ap.add_argument('--no-rtt', action='store_true',
                    help='skip the interactive RTT and bulk-TCP runs')
    ap.add_argument('--bulk-batch', type=int, default=1 << 20,
                    help='requests per Client.bulk_get batch of the '
                         'bulk-TCP measurement')
    ap.add_argument('--bulk-conns', type=int, default=8,
                    help='sessions (connections, one event loop each) the '
                         'k-connection bulk-TCP measurement splits a batch '
                         'over (the native server serves each on its own '
                         'worker thread)')
    ap.add_argument('--streams', type=int, default=2,
                    help='get: pipelined connections per GPU, one HIP '
                         'stream each (the batch is split between them; 2 '
                         'overlaps one connection\'s latency-bound kernels '
                         'with the other\'s bandwidth-bound ones, more '
                         'streams than GPU_MAX_HW_QUEUES allows were '
                         'unstable)')
    ap.add_argument('--no-graph', action='store_true',
                    help='get: time eager steps instead of replays of one '
                         'step captured as a HIP graph after the warmup '
                         '(every replay draws a new batch from a '
                         'device-resident seed; ~2%% faster than eager)')
    ap.add_argument('--stream-priority', action='store_true',
                    help='get: connection 0 on a high-priority stream')
    ap.add_argument('--stagger', action='store_true',
                    help='get: offset the pipelined connections by half a '
                         'step (measured no faster than lockstep, 0.80 vs '
                         '0.79 ms)')
    ap.add_argument('--workload', choices=('get', 'mix', 'storm', 'watch',
                                           'ensemble', 'chain', 'nest'),
                    default='get')
    ap.add_argument('--replica', action='store_true',
                    help='get: every rank serves its own full replica of the '
                         'tree (the default; kept for old command lines)')
    ap.add_argument('--sharded', action='store_true',
                    help='get, N > 1: make the path-hash-sharded tree with '
                         'R2 routing over RCCL/xGMI the headline (default: '
                         'timed after the replica step, as sharded_*)')
    ap.add_argument('--ndirs', type=int, default=1024,
                    help='mix / storm: parent directories the writes spread '
                         'over (a workload shape knob; parents take the '
                         'cversion / child-count atomics)')
    ap.add_argument('--hash-factor', type=int, default=0,
                    help='hash entries per node slot, rounded up to a power '
                    'of two (0: 32 for storm / mix, 16 for chain / nest, '
                    '2 otherwise; profiles/r5_storm_hash_factor_ab.log)')
    ap.add_argument('--force-route', action='store_true',
                    help='get, N = 1: run the multi-rank sharded step over a '
                         'one-rank RCCL group (router, slots, '
                         'all_to_all_single on HBM tensors, captured in the '
                         'HIP graph) and compare it with the local pipeline')
    ap.add_argument('--no-sustain', action='store_true',
                    help='skip the second, ~1 s timed window')
    ap.add_argument('--no-compare', action='store_true',
                    help='get, N > 1: skip the replica comparison run')
    ap.add_argument('--paths', type=int, default=65536,
                    help='ensemble: watched znodes (one owner rank each)')
    ap.add_argument('--writes', type=int, default=4096,
                    help='ensemble: znodes set per step')
    ap.add_argument('--failover-every', type=int, default=4,
                    help='ensemble: every k-th step kills the member rank 0 '
                         'is on and makes that step\'s writes during the '
                         'outage (replayed through SET_WATCHES)')
    a = ap.parse_args()
    if a.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        return launch(a)
    # a rank that fails (tests inject one with ZKMI_BENCH_FAIL_RANK) ends
    # the whole launch; the other ranks are stopped by the launcher
    fail = os.environ.get('ZKMI_BENCH_FAIL_RANK')
    if fail is not None and fail == os.environ.get('RANK', '0'):
        raise SystemExit('rank %s: injected failure' % fail)
    if a.workload == 'ensemble':
        return run_ensemble(a)
    return run_rank(a)


def _free_port():
    import socket
    so = socket.socket()
    so.bind(('127.0.0.1', 0))
    port = so.getsockname()[1]
    so.close()
    return port


def launch(a):
    """``--gpus N`` outside torchrun: start the N rank processes (one per
    GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their environment,
    rendezvous on 127.0.0.1) and exit with the first failure's code.  This
    process never touches the GPU or asks how many there are: it trusts
    --gpus, and a rank without a GPU fails loudly (and ends the launch)."""
    n = a.gpus
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r),
                   WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK='0', MASTER_ADDR='127.0.0.1',
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen(
            [sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
            env=env, cwd=ROOT))
    rc = 0
    live = list(procs)
    while live:
        time.sleep(0.2)
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c
                for q in live:             # the others would wait forever
                    q.terminate()
    for p in procs:
        try:
            p.wait(30)
        except subprocess.TimeoutExpired:
            p.kill()
    if rc:
        raise SystemExit(rc if rc > 0 else 128 - rc)
    return 0


def _time_steps(pipe, a, world, dev):
    """Warm up, optionally capture one step as a HIP graph, then time
    ``a.steps`` steps between barriers + device syncs.  Returns (seconds
    on this rank, correct replies counted on the device, graph used)."""
    ok_total = torch.zeros(64, dtype=torch.int64, device=dev)
    for _ in range(a.warmup):
        pipe.step(acc=ok_total)
    run = lambda: pipe.step(acc=ok_total)            # noqa: E731
    graph = not a.no_graph and hasattr(pipe, 'capture') and \
        getattr(pipe, 'capturable', True)
    if graph:
        try:
            g = pipe.capture(ok_total)
            run = g.replay
            for _ in range(2):
                run()
        except RuntimeError as e:              # keep the run: eager steps
            print('graph capture failed, timing eager steps: %s' % e,
                  file=sys.stderr)
            graph = False
            run = lambda: pipe.step(acc=ok_total)    # noqa: E731
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ok_total.zero_()
    # (per-connection graphs do not wait on this stream: the zeroing must
    # land before the first replay)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    pipe._bench_run = run
    return time.perf_counter() - t0, ok_total, graph


def _sustained(pipe, ok_total, steps, world):
    """A second timed window of ``steps`` steps (sized from the first one
    to last about SUSTAIN_S seconds; the same on every rank), its replies
    counted like the first's: the rate over a window long enough that
    launch and clock granularity do not colour it."""
    run = pipe._bench_run
    torch.cuda.synchronize()
    ok_total.zero_()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    return time.perf_counter() - t0


SUSTAIN_S = 1.0


def _reduce(elapsed, ok_total, world, cdev):
    """(max seconds over ranks, correct replies summed over ranks) — R4."""
    el = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
    ok = ok_total.sum().view(1).to(cdev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        dist.all_reduce(ok, op=dist.ReduceOp.SUM)
    return el.item(), int(ok.item())


def run_rank(a):

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    rtt_srv = start_rtt_server() if rank == 0 and not a.no_rtt else None
    fast_srv = start_fast_server(a.nodes, a.data_bytes) \
        if rank == 0 and not a.no_rtt and a.workload == 'get' else None
    ev_idle = (None, None)
    if fast_srv is not None:
        # the same event-loop round trip before this process touches the
        # GPU, next to the one measured after the timed steps
        ev_idle = measure_rtt_async(fast_srv.port)
    # One rank per GPU over RCCL ("nccl").  ZKMI_BENCH_BACKEND=gloo (host
    # collectives, ranks may share a GPU) exists only to rehearse the
    # multi-rank path on a one-GPU box.
    backend = os.environ.get('ZKMI_BENCH_BACKEND', 'nccl')
    ndev = torch.cuda.device_count()
    gpu = local % ndev if backend == 'gloo' else local
    dev = torch.device('cuda', gpu)
    torch.cuda.set_device(dev)
    if world > 1:
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=dev)
        else:
            dist.init_process_group(backend)
    elif a.force_route and a.workload == 'get':
        # a one-rank RCCL group: the multi-rank step's collectives run
        # through RCCL on this GPU's HBM
        dist.init_process_group(
            'nccl', device_id=dev, rank=0, world_size=1,
            init_method='tcp://127.0.0.1:%d' % _free_port())
    cdev = dev if backend == 'nccl' else torch.device('cpu')

    from zkmi.bench import synthetic as S
    dd = npad = None
    if a.data_dist:
        kind, _, rng = a.data_dist.partition(':')
        if kind != 'uniform':
            raise SystemExit('--data-dist: only uniform:LO-HI')
        dd = tuple(int(x) for x in rng.split('-'))
    if a.name_pad:
        npad = tuple(int(x) for x in a.name_pad.split('-'))
    # GET at N > 1: every member holds the whole tree in its HBM and serves
    # its sessions' reads from it — ZooKeeper's read path (any server
    # answers a read from its replica); 1M znodes are ~0.4 GB of 288.  The
    # path-hash-sharded tree with reads routed over xGMI (R2) is for trees
    # past one GPU's memory: --sharded makes it the headline, otherwise it
    # is timed after the replica step (sharded_*).
    sharded = a.workload == 'get' and (a.sharded or a.force_route) and \
        not a.replica

    def make_get(replica):
        if replica:
            tree = S.GpuTree(a.nodes, a.data_bytes, device=dev, seed=rank,
                             data_dist=dd, name_pad=npad)
            return S.GetPipeline(tree, a.batch, seed=rank, streams=a.streams,
                                 stagger=a.stagger,
                                 priority=a.stream_priority)
        from zkmi.parallel.sharded import ShardedGetPipeline
        # every rank holds the same layout and data (seed 0); its index
        # covers only the leaves whose path hashes to it
        tree = S.GpuTree(a.nodes, a.data_bytes, device=dev, seed=0,
                         data_dist=dd, name_pad=npad, shard=(rank, world))
        return ShardedGetPipeline(tree, a.batch, seed=rank, coll_device=cdev,
                                  streams=a.streams,
                                  force_route=a.force_route)

    if a.workload == 'get':
        pipe = make_get(not sharded)
        per_step = a.batch
    elif a.workload == 'watch':
        tree = S.GpuTree(a.nodes, a.data_bytes, device=dev, seed=rank,
                         watch_cap=2 * a.batch)
        pipe = S.WatchPipeline(tree, a.batch, seed=rank,
                               coll_device=cdev if world > 1 else None)
        # write-triggered notifications decoded per rank (every rank's
        # writes reach every rank); a batch watches distinct nodes
        per_step = pipe.n * world
    else:
        # room for the write working set next to the 1M static nodes: the
        # mix keeps 3 generations of batch/3 nodes, the storm up to 3
        # batches (the expiring session's two, the new session's first)
        spare = (a.batch * (1 if a.workload in ('mix', 'chain', 'nest')
                            else 3 * world) + 8192) / a.nodes
        # chain: the set and get of every chain reply from a snapshot; nest:
        # the parents' EXISTS
        scratch = (a.batch // 2 + 64) * (80 + ((a.data_bytes + 15) & ~15)) \
            if a.workload in ('chain', 'nest') else 0
        # the storm's members hold one replicated tree: the same tree on
        # every rank (seed 0), every member applies every member's writes
        tree = S.GpuTree(a.nodes, a.data_bytes, device=dev,
                         seed=0 if a.workload == 'storm' else rank,
                         spare=spare + 0.05, scratch=scratch,
                         hash_factor=a.hash_factor or (
                             32 if a.workload in ('storm', 'mix') else
                             16 if a.workload in ('chain', 'nest')
                             else 2),
                         compact_free=a.workload in ('mix', 'nest'))
        if a.workload == 'chain':
            pipe = S.ChainPipeline(tree, a.batch, a.data_bytes, seed=rank)
            per_step = pipe.n
        elif a.workload == 'nest':
            pipe = S.NestPipeline(tree, a.batch, seed=rank)
            per_step = pipe.n
        elif a.workload == 'mix':
            pipe = S.MixPipeline(tree, a.batch, a.data_bytes,
                                 ndirs=a.ndirs, seed=rank)
            per_step = pipe.n
        else:
            # across GPUs the sessions move between members (R3)
            pipe = S.StormPipeline(tree, a.batch, ndirs=a.ndirs, seed=rank,
                                   coll_device=cdev if world > 1 else None)
            per_step = pipe.n

    ops = per_step * a.steps * world

    def checked(pipe, elapsed, ok_total):
        elapsed, ok = _reduce(elapsed, ok_total, world, cdev)
        if ok != ops:
            if hasattr(pipe, 'diagnose'):
                print('diagnose:', pipe.diagnose(), file=sys.stderr)
            raise SystemExit('validation failed: %d of %d replies wrong'
                             % (ops - ok, ops))
        return elapsed

    # 64 counter slots (the fused GET check spreads its per-block atomics
    # over them); the other checks add into slot 0
    elapsed, ok_total, a.graph = _time_steps(pipe, a, world, dev)
    elapsed = checked(pipe, elapsed, ok_total)
    value = ops / elapsed
    sustained = None
    if not a.no_sustain:
        # (elapsed is the max over ranks: every rank runs the same count)
        k = int(min(max(SUSTAIN_S / max(elapsed / a.steps, 1e-6), a.steps),
                    50000))
        sel = _sustained(pipe, ok_total, k, world)
        sel, sok = _reduce(sel, ok_total, world, cdev)
        if sok != per_step * k * world:
            raise SystemExit('validation failed in the sustained window: '
                             '%d of %d' % (per_step * k * world - sok,
                                           per_step * k * world))
        sustained = {'steps': k, 'seconds': sel,
                     'ops_s': per_step * k * world / sel,
                     'ms_per_step': sel / k * 1e3}
    def r2_stats(pipe):
        st = pipe.stats
        return {'bytes_sent_per_rank_step': st['bytes_sent'] / max(st['steps'],
                                                                   1),
              'wire_bytes_sent_per_rank_step':
                  st['wire_bytes_sent'] / max(st['steps'], 1),
              'remote_requests': st['remote_reqs'],
              'overflow_segments': st['overflow_segments'],
              'xgmi_lower_bound_ms': st['xgmi_lower_bound_ms'],
              'copy_bytes_per_step_max': st['copy_bytes_per_step_max'],
              'local_bytes_through_collective':
                  st['local_bytes_through_collective'],
              'slot_bytes': {'request': st['req_slot_bytes'],
                             'reply': st['rep_slot_bytes']}}
    r2 = r2_stats(pipe) if sharded else None
    replica = shard_cmp = None
    if a.workload == 'get' and (world > 1 or a.force_route) and \
            not a.no_compare:
        # the other GET mode on the same batch size: the replicas (no
        # collective in the step) after a sharded headline, or the sharded
        # tree (R2 over RCCL/xGMI) after the replicas — what routing the
        # reads across the GPUs costs
        del pipe
        torch.cuda.empty_cache()
        rp = make_get(sharded)
        rel, rok, rgraph = _time_steps(rp, a, world, dev)
        rel = checked(rp, rel, rok)
        res = {'value': ops / rel, 'ms_per_step': rel / a.steps * 1e3,
               'hip_graph': bool(rgraph)}
        if sharded:
            replica = res
        else:
            shard_cmp = res
            r2 = r2_stats(rp)
        del rp

    rtt50 = rtt99 = py50 = py99 = bulk_ops = bulk_ms = bulk_ph = None
    bulk_k = (None, None, None)
    ev50 = ev99 = pipe_ops = None
    if rtt_srv is not None:
        try:
            py50, py99 = measure_rtt(rtt_srv[1])
        finally:
            rtt_srv[0].stdin.close()
            rtt_srv[0].wait(10)
    if fast_srv is not None:
        try:
            rtt50, rtt99 = measure_rtt(fast_srv.port)
            ev50, ev99 = measure_rtt_async(fast_srv.port)
            pipe_ops = measure_pipelined(fast_srv.port)
            bulk_ops, bulk_ms, bulk_ph = measure_bulk_tcp(
                fast_srv.port, a.nodes, a.bulk_batch, 3, dev, 1, fast_srv)
            bulk_k = measure_bulk_tcp(fast_srv.port, a.nodes, a.bulk_batch,
                                      3, dev, a.bulk_conns)
        finally:
            fast_srv.shutdown()
    elif rtt_srv is not None:
        rtt50, rtt99 = py50, py99

    if rank == 0:
        line = {
            'metric': 'ZK ops/sec (whole node) + p50 get() RTT, 1M-znode '
                      'synthetic tree',
            'value': value,
            'unit': 'ops/s',
            'n_gpus': world,
            'steps': a.steps,
            'warmup': a.warmup,
            'ms_per_step': elapsed / a.steps * 1e3,
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': value / REF_PKTS_PER_S,
            'dtype': 'uint8',
            'hip_graph': bool(a.graph),
            'data': 'synthetic',
            'config': {
                'model': 'zk-%s %dk-znode tree, %s data%s' % (
                    a.workload,
                    a.nodes // 1000,
                    ('%d-%dB' % dd) if dd else '%dB' % a.data_bytes,
                    (', names +%d-%d chars' % npad) if npad else ''),
                'global_batch': per_step * world,
                'seq_len': 1,
                'parallelism': ('r2shard%d' % world) if sharded and
                               world > 1 else 'dp%d' % world,
            },
            'get_mode': ('sharded: one tree, path-hash shards over %d '
                         'ranks, reads routed with all_to_all over %s' % (
                             world, 'RCCL/xGMI' if backend == 'nccl' else
                             '%s (rehearsal, ranks may share a GPU)'
                             % backend) if world > 1 else
                         'sharded step forced over a one-rank RCCL group: '
                         'route -> seg_pack -> all_to_all_single (RCCL, HBM '
                         'tensors) -> seg_unpack; replica_* = the local '
                         'pipeline' if a.force_route else
                         'one shard (nothing to route), local pipeline')
                        if sharded else
                        ('replica per rank: every member holds the whole '
                         'tree and serves its reads locally (ZooKeeper\'s '
                         'read path); sharded_* = one tree sharded by path '
                         'hash, reads routed with all_to_all over %s' % (
                             'RCCL/xGMI' if backend == 'nccl' else backend)
                         if a.workload == 'get' and world > 1 else
                         'replica per rank' if a.workload == 'get' else None),
            'value_note': 'value: the on-device pipeline rate (K10 '
                          'request encode -> GPU-resident server -> K1 + '
                          'K2-K8 reply decode and check, all in HBM, no TCP '
                          'and no per-request client API); the end-to-end '
                          'figure through the client API over TCP is '
                          'end_to_end_ops_s (bulk_get over loopback to the '
                          'native server); sustained: the same steps timed '
                          'over a window of about %.0f s' % SUSTAIN_S,
            'sustained': sustained,
            'end_to_end_ops_s': bulk_k[0],
            # the client-API figure against the same reference decode rate
            # (value above is the on-device pipeline; value_note)
            'vs_baseline_end_to_end': (bulk_k[0] / REF_PKTS_PER_S
                                       if bulk_k[0] else None),
            'r2': r2,
            'workload_stats': dict(pipe.stats) if a.workload == 'storm'
                              else None,
            'replica_value': replica['value'] if replica else None,
            'replica_ms_per_step': replica['ms_per_step'] if replica else None,
            'sharded_value': shard_cmp['value'] if shard_cmp else None,
            'sharded_ms_per_step': shard_cmp['ms_per_step'] if shard_cmp
            else None,
            'p50_get_rtt_us': rtt50,
            'p99_get_rtt_us': rtt99,
            'rtt_note': 'one blocking Client.call_sync(get) over loopback '
                        'TCP to the native server (zk_fastserver), sent '
                        'from the calling thread and settled by the native '
                        'reply router; *_fakezk: to the Python fake server',
            'p50_get_rtt_us_evloop': ev50,
            'p99_get_rtt_us_evloop': ev99,
            'rtt_evloop_note': 'get(path, cb) chained on the client event '
                               'loop (each callback issues the next get), '
                               'as node-zkstream runs it: no caller-thread '
                               'hop; same native server',
            'pipelined_get_ops_s': pipe_ops,
            'pipelined_note': 'get(path, cb) with 256 in flight on one '
                              'connection (each callback issues the next): '
                              'the per-request API through the native '
                              'completion path (reply router + coalesced '
                              'writes in the native loop)',
            'p50_get_rtt_us_evloop_pre_gpu': ev_idle[0],
            'p99_get_rtt_us_evloop_pre_gpu': ev_idle[1],
            'p50_get_rtt_us_fakezk': py50,
            'p99_get_rtt_us_fakezk': py99,
            'bulk_tcp_ops_s': bulk_ops,
            'bulk_tcp_ms_per_batch': bulk_ms,
            'bulk_tcp_phases_ms': bulk_ph,
            'bulk_tcp_conns': a.bulk_conns,
            'bulk_tcp_ops_s_kconn': bulk_k[0],
            'bulk_tcp_ms_per_batch_kconn': bulk_k[1],
            'bulk_tcp_phases_ms_kconn': bulk_k[2],
            'bulk_tcp_note': 'Client.bulk_get of %d random nodes per batch '
                             'over loopback TCP to the native server: GPU '
                             'encode/decode, pinned TX/RX, replies captured '
                             'by the native loop; *_kconn: the batch split '
                             'over bulk_tcp_conns sessions at once' %
                             a.bulk_batch,
            'batch_latency_ms': elapsed / a.steps * 1e3,
            'baseline_note': 'vs_baseline = value / 0.51M pkts/s, the '
                             'reference ZKDecodeStream frame+decode on one '
                             'Xeon core (BASELINE.md, local, unpublished)',
            'dtype_note': 'byte codec over uint8 wire streams and int32/int64 '
                          'tables; no floating-point compute',
        }
        print(json.dumps(line), flush=True)
    # captured graphs hold the communicator's work: release them (and the
    # pipelines holding them) before the group goes — destroying an RCCL
    # group under a live graph waits forever in its shutdown
    pipe = None
    gc.collect()
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
