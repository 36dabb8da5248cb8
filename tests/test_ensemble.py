"""BASELINE config 4 as a multi-rank workload (zkmi/parallel/ensemble.py):
a 3-member ensemble, one session per rank, member failover with watch
replay through SET_WATCHES, every event fanned out to every rank.

CPU: gloo, world 2, 4 and 8, host decode of the fanned-out wire frames,
against the native 3-member ensemble server.  GPU: one rank with the live
connection's K9 / K11 records, the bulk re-arm on the GPU and the fan-out's
K1 + K2-K8 decode and (path, version) count on the device."""

import os
import socket
import sys
import traceback

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, mport, steps, errq, outq):
    try:
        sys.path.insert(0, ROOT)
        import torch.distributed as dist
        dist.init_process_group('gloo', init_method='tcp://127.0.0.1:%d'
                                % mport, rank=rank, world_size=world)
        from zkmi.parallel import ensemble as E
        ctl = E.EnsembleControl(3) if rank == 0 else None
        try:
            wl = E.EnsembleWorkload(ctl, n_paths=48, writes=12,
                                    failover_every=2, codec_device=None,
                                    trace=True)
            got = [wl.step() for _ in range(steps)]
            bad = wl.verify()
            extra = None
            if bad is not None:
                # what to look at when an event arrives twice: this rank's
                # resumes (relZxid, watches), forwards and receipts
                extra = {'resumes': wl.client.loop.run(
                    lambda: list(wl.client.getSession().resumes)),
                    'trace': wl.trace}
            outq.put((rank, bad, got, wl.failovers, wl.rearmed(),
                      wl.replayed, dict(wl.fan.stats), extra))
            dist.barrier()
            wl.close()
        finally:
            if ctl is not None:
                ctl.close()
        dist.destroy_process_group()
    except BaseException:
        errq.put((rank, traceback.format_exc()))
        raise


def _run(world, steps):
    ctx = mp.get_context('spawn')
    errq, outq = ctx.SimpleQueue(), ctx.SimpleQueue()
    try:
        mp.start_processes(_worker, args=(world, _free_port(), steps, errq,
                                          outq),
                           nprocs=world, join=True, start_method='spawn')
    except Exception:
        msgs = []
        while not errq.empty():
            msgs.append('rank %d:\n%s' % errq.get())
        while not outq.empty():
            msgs.append('rank %d finished: %r' % (outq.get()[0],))
        raise AssertionError('\n'.join(msgs) or 'worker failed')
    res = {}
    while not outq.empty():
        r = outq.get()
        res[r[0]] = r[1:]
    return res


@pytest.mark.parametrize('world', [2, 4, 8])
def test_ensemble_failover_replay_fanout(world):
    steps = 4                               # failovers at steps 1 and 3
    res = _run(world, steps)
    assert sorted(res) == list(range(world)), res
    # on any failure, every rank's (bad, got, failovers, rearmed, replayed,
    # fan-out stats) goes into the message
    report = {r: dict(zip(('bad', 'got', 'fo', 'rearmed', 'replayed',
                           'stats', 'trace'), v)) for r, v in res.items()}
    rearmed = 0
    for rank, (bad, got, fo, rea, replayed, st, _) in res.items():
        if bad is not None:
            d = os.path.join(ROOT, 'gpurun_out')
            os.makedirs(d, exist_ok=True)
            with open(os.path.join(d, 'ensemble_dup_w%d_%d.txt'
                                   % (world, os.getpid())), 'w') as f:
                f.write(repr(report))
        # every event (initial arm, live, replayed) exactly once per rank
        assert bad is None, (rank, report)
        assert got == [12] * steps, (rank, report)
        assert fo == 2 and replayed == 24, (rank, report)
        # a notification + its re-arm reply per event
        assert st['decoded_host'] == 2 * (48 + 12 * steps), (rank, report)
        rearmed += rea
    # the killed members' sessions resumed their watches (SET_WATCHES)
    assert rearmed > 0


@pytest.mark.gpu
def test_ensemble_gpu_codec_and_fanout_decode():
    """One rank on the GPU: its reconnects run K9 (ConnectRequest encode,
    ConnectResponse decode) and its watch resume K11 (SET_WATCHES); the
    fan-out frames are decoded by K1 + K2-K8."""
    import torch
    from zkmi.parallel import ensemble as E
    dev = torch.device('cuda', 0)
    ctl = E.EnsembleControl(3)
    try:
        wl = E.EnsembleWorkload(ctl, n_paths=40, writes=10,
                                failover_every=2, codec_device=dev)
        for _ in range(4):
            assert wl.step() == 10
        assert wl.verify() is None
        assert wl.fan.stats['decoded_gpu'] == 2 * (40 + 40)
        assert wl.rearmed() == 40 * 2        # one resume per failover
        from zkmi.models import gpucodec
        calls = gpucodec.for_device(dev).calls
        assert calls['connect_request'] >= 3          # initial + 2 failovers
        assert calls['connect_response'] >= 3
        # the resumes carry only bulk watches, whose path vector is kept
        # encoded (jute.PackedStrings): a byte copy, no K11 launch
        assert calls['set_watches'] == 0
        wl.close()
    finally:
        ctl.close()


def _replayed_catch_up(wl, gpu):
    """One watched path written once, then its catch-up notification
    forwarded twice (what a second SET_WATCHES at the same relZxid brings
    when the session moves again before the first one is answered): the
    owner forwards the change once and drops the repeat — also when both
    copies arrive in one re-arm batch."""
    from zkmi.parallel.fanout import notification_frames
    p = wl.mine[0]
    wl.client.call_sync('set', p, b'changed', -1)
    notes = notification_frames([p], evtype=3)         # NODE_DATA_CHANGED
    first, nf1 = wl._rearm(notes, 1)
    again, nf2 = wl._rearm(notes, 1)
    assert nf1 == 2 and len(first) > 0
    assert nf2 == 0 and len(again) == 0
    assert wl.redelivered == 1

    def fwd():
        k = int(p[-5:])
        return int(wl.fwd_ver_dev[k].item()) if gpu else int(wl.fwd_ver[k])
    assert fwd() == 1
    # a later change of the same path goes through again
    wl.client.call_sync('set', p, b'changed2', -1)
    _, nf3 = wl._rearm(notes, 1)
    assert nf3 == 2 and fwd() == 2
    # the replay in the same tick as the original: one batch holds the
    # path twice; only the first copy is forwarded
    wl.client.call_sync('set', p, b'changed3', -1)
    both = notification_frames([p, p], evtype=3)
    _, nf4 = wl._rearm(both, 2)
    assert nf4 == 2 and fwd() == 3
    assert wl.redelivered == 2


def test_ensemble_owner_drops_replayed_catch_up():
    from zkmi.parallel import ensemble as E
    ctl = E.EnsembleControl(3)
    try:
        wl = E.EnsembleWorkload(ctl, n_paths=8, writes=2, failover_every=0,
                                codec_device=None)
        try:
            _replayed_catch_up(wl, None)
        finally:
            wl.close()
    finally:
        ctl.close()


@pytest.mark.gpu
def test_ensemble_owner_drops_replayed_catch_up_gpu():
    """The same on the device path (K1 + K2-K8 decode of the notes, the
    dedup's compaction of the forwarded frames on the GPU)."""
    import torch
    from zkmi.parallel import ensemble as E
    ctl = E.EnsembleControl(3)
    try:
        wl = E.EnsembleWorkload(ctl, n_paths=8, writes=2, failover_every=0,
                                codec_device=torch.device('cuda', 0))
        try:
            _replayed_catch_up(wl, True)
        finally:
            wl.close()
    finally:
        ctl.close()
