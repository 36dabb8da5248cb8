"""K1's link repair (csrc/kernels/frame_scan.hip fs_link) on the streams
that defeat the speculative tile entry: exact against the host framer, and
bounded in time.

* every tile without a speculated entry (``nospec``): the grid repair
  settles all links in parallel rounds — the round-2 serial repair walked
  them one tile after the other (50 ms on one storm reply stream);
* frames longer than the entry window whose payloads are made of
  plausible length words (garbage chains that never die): the serial tail
  skips the tiles a frame covers whole;
* variable reply-sized frames (the 0-1024 B GET workload's reply stream);
* garbage entries forced into every P-th tile (``misspec``) of a stream
  whose garbage chains jump megabytes ahead (create replies: an xid or a
  zxid read as a length): the repair must not carry a garbage exit from
  tile to tile (the first storm reply stream: 1413 tiles over 71 rounds).

Reference framer: lib/zk-streams.js:47-64 (one frame at a time)."""

import numpy as np
import pytest
import torch

from zkmi.ops import batch as B

pytestmark = pytest.mark.gpu


def _stream(rng, lens, payload='random'):
    """Frames with the given body lengths; payload 'random' bytes or
    'plausible' big-endian words in [8, 200] (each reads as a valid
    length)."""
    lens = np.asarray(lens, np.int64)
    starts = np.zeros(len(lens), np.int64)
    np.cumsum(lens[:-1] + 4, out=starts[1:])
    total = int(starts[-1] + lens[-1] + 4)
    if payload == 'random':
        buf = rng.integers(0, 256, total, dtype=np.uint8)
    else:
        words = rng.integers(8, 201, (total + 3) // 4).astype('>u4')
        buf = np.frombuffer(words.tobytes(), np.uint8)[:total].copy()
    for k in range(4):
        buf[starts + k] = ((lens >> (8 * (3 - k))) & 0xff).astype(np.uint8)
    return buf, starts


def _scan_timed(buf, nframes, window, nospec=False, reps=3, misspec=0,
                group=None):
    dev = torch.device('cuda', 0)
    d = torch.from_numpy(buf).to(dev)
    sc = B.FrameScanner(nframes + 16, dev, window=window, group=group)
    sc.scan(d, len(buf), nospec=nospec, misspec=misspec)      # warm
    torch.cuda.synchronize()
    best = None
    for _ in range(reps):
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record()
        ft = sc.scan(d, len(buf), nospec=nospec, misspec=misspec)
        t1.record()
        torch.cuda.synchronize()
        ms = t0.elapsed_time(t1)
        best = ms if best is None else min(best, ms)
    r = ft.host_result()
    off = ft.off[:min(r['frames'], nframes)].cpu().numpy()
    return r, off, best, sc.chain_stats()


def _check(r, off, buf, starts):
    assert r['frames'] == len(starts) and not r['bad'] and not r['overflow']
    assert r['consumed'] == len(buf)
    assert np.array_equal(off, starts + 4)


def test_no_speculated_entries_repairs_in_parallel(gpu):
    rng = np.random.default_rng(11)
    lens = rng.integers(88, 1113, 60000)
    buf, starts = _stream(rng, lens)
    r, off, spec_ms, _ = _scan_timed(buf, len(lens), 2048)
    _check(r, off, buf, starts)
    r, off, ms, st = _scan_timed(buf, len(lens), 2048, nospec=True)
    _check(r, off, buf, starts)
    tiles = (len(buf) + 4095) // 4096
    # every tile but the first was repaired, by the grid rounds (a round
    # count of a few, not one per tile)
    assert st['no_spec'] >= 3 * (tiles - 1)           # 3 timed + warm scans
    assert st['rounds'] <= 4 * 8
    # bounded: a few times the speculative scan, not tiles x walk latency
    # (the serial repair: ~3-5 us per tile, ~40 ms here)
    assert ms < max(8 * spec_ms, 2.0), (ms, spec_ms)


def test_long_frames_with_plausible_payload(gpu):
    """Every frame longer than the window (256 B) and every payload word a
    plausible length: speculation is wrong everywhere, the chain is exact."""
    rng = np.random.default_rng(5)
    lens = rng.integers(2000, 9001, 6000)
    buf, starts = _stream(rng, lens, payload='plausible')
    r, off, ms, st = _scan_timed(buf, len(lens), 256)
    _check(r, off, buf, starts)
    # the serial tail costs one step per frame (covered tiles are filled in
    # one step), not per tile; a ~30 MB stream stays in milliseconds
    assert ms < 40.0, ms


def test_variable_reply_frames_exact(gpu):
    rng = np.random.default_rng(3)
    for lo, hi, win in ((88, 1112, 2048), (88, 1112, 512), (20, 300, 256)):
        lens = rng.integers(lo, hi + 1, 40000)
        buf, starts = _stream(rng, lens)
        r, off, ms, st = _scan_timed(buf, len(lens), win, reps=1)
        _check(r, off, buf, starts)


def _create_replies(n, xid0=0x300401, zxid0=0x3f4a2c):
    """The storm workload's CREATE replies: 50-byte frames {len 46, xid,
    zxid, err 0, path length 26, '/storm/dNNNNN/e-NNNNNNNNNN'}."""
    i = np.arange(n, dtype=np.int64)
    rec = np.zeros((n, 50), np.uint8)

    def be(col, v, w):
        for b in range(w):
            rec[:, col + b] = (v >> (8 * (w - 1 - b))) & 0xff
    be(0, np.full(n, 46), 4)
    be(4, xid0 + i, 4)
    be(8, zxid0 + i, 8)
    be(20, np.full(n, 26), 4)
    paths = np.frombuffer(b''.join(b'/storm/d%05d/e-%010d' % (k % 100, k)
                                   for k in range(n)), np.uint8)
    rec[:, 24:] = paths.reshape(n, 26)
    return rec.reshape(-1), np.arange(n, dtype=np.int64) * 50


@pytest.mark.parametrize('period', [97, 1])
def test_garbage_entries_do_not_propagate(gpu, period):
    """Every period-th tile (period 1: every tile) enters on a garbage chain.
    Few broken links are block 0's worklist, every tile the grid's rounds;
    either way each broken link settles in a round or two (a garbage exit
    walked on would cost one round per tile it crosses)."""
    n = 1 << 20
    buf, starts = _create_replies(n)
    _, _, base_ms, _ = _scan_timed(buf, n, 256)
    r, off, ms, st = _scan_timed(buf, n, 256, misspec=period)
    _check(r, off, buf, starts)
    tiles = (len(buf) + 4095) // 4096
    broken = (tiles - 1) // period
    scans = 4                                  # warm + 3 timed
    assert st['rounds'] <= scans * 6, st
    assert st['rewalked'] <= scans * (3 * broken + 8), st
    assert ms < max(6 * base_ms, 1.5), (ms, base_ms)


def test_garbage_entries_variable_and_long_frames(gpu):
    rng = np.random.default_rng(8)
    lens = rng.integers(88, 1113, 40000)
    buf, starts = _stream(rng, lens)
    for period in (3, 50):
        r, off, ms, st = _scan_timed(buf, len(lens), 2048, reps=1,
                                     misspec=period)
        _check(r, off, buf, starts)
    lens = rng.integers(2000, 9001, 3000)
    buf, starts = _stream(rng, lens, payload='plausible')
    for period in (2, 7):
        r, off, ms, st = _scan_timed(buf, len(lens), 256, reps=1,
                                     misspec=period)
        _check(r, off, buf, starts)


def test_side_branches_on_the_chain_keep_the_map(gpu):
    """Every create reply's path-length word (26, 20 past its frame's start)
    is a node whose frame ends at the next frame's start: a side branch
    with the chain node's root and count (fs_tile's ft_chain keeps each
    slot's smallest position, then checks the links).  Every 7th frame also
    holds a word 30 past its start reading 66 — a side branch BEFORE the
    next frame's node (it ends two frames on) that wins its slot, so the
    link check must send the tile to the exact walk.  Both exact; the
    clean stream no slower than a few times a plain one."""
    n = 1 << 19
    buf, starts = _create_replies(n, zxid0=0x500000)
    _, _, base_ms, _ = _scan_timed(buf, n, 256)
    r, off, ms, st = _scan_timed(buf, n, 256)
    _check(r, off, buf, starts)
    early = buf.copy()
    for p in starts[::7]:
        early[p + 30:p + 34] = (0, 0, 0, 66)
    r, off, ms2, st = _scan_timed(early, n, 256)
    _check(r, off, early, starts)
    assert ms2 < max(8 * base_ms, 2.0), (ms2, base_ms)


def test_phantom_chain_region_is_chased_not_walked(gpu):
    """Create replies whose zxids run through 0x2Exxxx: the bytes 10 past
    every frame start then read as the frame length 46, a phantom chain
    parallel to the true one over ~800 tiles.  No tile can tell the two
    apart; fs_link's chase follows the exact one through fs_tile's candidate
    exit map and the grid re-walks the tiles in parallel.  (The storm's
    first reply stream: 18 ms of tile-after-tile repair before.)"""
    n = 1 << 20
    clean, starts = _create_replies(n, zxid0=0x500000)
    _, _, base_ms, _ = _scan_timed(clean, n, 256)
    buf, starts = _create_replies(n, zxid0=0x2E0000 - 500000)
    r, off, ms, st = _scan_timed(buf, n, 256)
    _check(r, off, buf, starts)
    assert st['looked_up'] >= 4 * 700, st      # the region, looked up
    assert st['rounds'] <= 4 * 4, st           # in a round or two per scan
    assert ms < max(3 * base_ms, 0.6), (ms, base_ms)


def _set_replies(n, version=84, xid0=0x5000, zxid0=0xA12C929):
    """SET_DATA replies of nodes whose version is 84: 88-byte frames {len
    84, xid, zxid, err 0, Stat} — the Stat's version word reads as the
    frame length, so a phantom chain of the frame's own period runs through
    the whole stream beside the true one (the watch workload's write
    replies at its 84th write of every node: an 84 ms fs_link repair at
    step 83 of every run, rounds 4-5)."""
    i = np.arange(n, dtype=np.int64)
    rec = np.zeros((n, 88), np.uint8)

    def be(col, v, w):
        for b in range(w):
            rec[:, col + b] = (v >> (8 * (w - 1 - b))) & 0xff
    be(0, np.full(n, 84), 4)
    be(4, xid0 + i, 4)
    be(8, zxid0 + i, 8)
    st = 20                                            # the Stat
    be(st + 0, 1000 + i, 8)                            # czxid
    be(st + 8, zxid0 + i, 8)                           # mzxid
    be(st + 16, np.full(n, 0x19A3F2C1D00), 8)          # ctime
    be(st + 24, np.full(n, 0x19A3F2C2E11), 8)          # mtime
    be(st + 32, np.full(n, version), 4)                # version
    be(st + 52, np.full(n, 100), 4)                    # dataLength
    be(st + 60, 1000 + i, 8)                           # pzxid
    return rec.reshape(-1), np.arange(n, dtype=np.int64) * 88


def test_phantom_chain_through_the_whole_stream(gpu):
    """Every frame carries a phantom chain of its own period: both chains
    survive every tile, about half the tiles speculate the phantom one.
    One exact chase through fs_tile's candidate exits settles the stream
    (looked up, not walked tile by tile)."""
    n = 1 << 20
    clean, _ = _set_replies(n, version=3)
    _, _, base_ms, _ = _scan_timed(clean, n, 256)
    buf, starts = _set_replies(n)
    r, off, ms, st = _scan_timed(buf, n, 256)
    _check(r, off, buf, starts)
    assert ms < max(10 * base_ms, 5.0), (ms, base_ms, st)


def test_get_replies_exact_below_the_largest_frame(gpu, monkeypatch):
    """0-1024 B GET replies scanned at a 512 B window (half the largest
    frame, long-frame mode: frontier passes past the window, survivor exits
    past it as entries; the tiles still broken go through the grid rounds
    and the serial tail).  Every frame table must still equal the host
    framing — a refused repair walk once left a tile's frame starts
    overwritten under its old record (3 frames in 20M)."""
    from zkmi.ops import batch as B
    monkeypatch.setattr(B, 'FS_WINDOW_AUTO_MAX', 512)
    from zkmi.bench import synthetic as S
    tree = S.GpuTree(200_000, 100, device=gpu, seed=0, data_dist=(0, 1024))
    pipe = S.GetPipeline(tree, 1 << 16, seed=1)
    from zkmi.ops import batch as B
    assert pipe.rwindow == 512 | B.FS_WIN_LONG
    for _ in range(4):
        acc = pipe.step()
        idx, rep, rx, ft = pipe.last
        r = ft.host_result()
        b = rx[:r['consumed']].cpu().numpy().tobytes()
        want = []
        p = 0
        while p + 4 <= len(b):
            want.append(p + 4)
            p += 4 + int.from_bytes(b[p:p + 4], 'big')
        got = ft.off[:r['frames']].cpu().numpy()
        assert np.array_equal(got, np.asarray(want, np.int64))
        assert int(acc.item()) == 1 << 16


def test_length_like_words_keep_the_map(gpu):
    """Delete-reply-sized frames (16-byte bodies) whose zxid field reads as
    a 2-4 KiB length (zxid in [2^27, 2^28): bytes 00 00 08..0f xx): past
    the entry window such words are not nodes (the window covers the
    stream's frames), so every tile keeps its map and its speculated entry.
    Counting them took a tile past the map's 512 nodes — no speculation, a
    serial repair of ~200 ms per 50 MB reply stream."""
    rng = np.random.default_rng(5)
    n = 200000
    lens = np.full(n, 16, np.int64)
    buf, starts = _stream(rng, lens)
    zx = (1 << 27) + np.arange(n, dtype=np.int64) * 7
    for k in range(8):                     # xid 4 bytes, then the zxid
        buf[starts + 8 + k] = ((zx >> (8 * (7 - k))) & 0xff).astype(np.uint8)
    for k in range(4):                     # err = 0
        buf[starts + 16 + k] = 0
    r, off, ms, st = _scan_timed(buf, n, 512)
    _check(r, off, buf, starts)
    assert st['no_spec'] == 0 and st['rewalked'] == 0, st
    assert ms < 5.0, ms


@pytest.mark.parametrize('group', [1, 4, 8])
def test_dense_length_words_walk_the_candidates(gpu, group):
    """Frames within the window whose payloads are all plausible length
    words (a tile holds far more than the map's 512 nodes): the tile walks
    its window entries lane by lane instead of mapping and still publishes
    candidate exits; a group walks its survivor on through its other tiles.
    Exact, and bounded: every chain survives such payloads, so the
    speculated entry is often a phantom chain and the link repair runs
    (26 MB: 0.69 ms single tiles, 2.6 ms groups of 4, against 0.04 ms for
    random payloads; a run of tiles without candidates was a serial
    repair)."""
    rng = np.random.default_rng(9)
    lens = rng.integers(96, 249, 150000)
    buf_r, starts = _stream(rng, lens)
    r, off, ms_r, _ = _scan_timed(buf_r, len(lens), 256, group=group)
    _check(r, off, buf_r, starts)
    buf_p, starts = _stream(rng, lens, payload='plausible')
    r, off, ms_p, st = _scan_timed(buf_p, len(lens), 256, group=group)
    _check(r, off, buf_p, starts)
    print('group %d: random payloads %.3f ms, length words %.3f ms %r'
          % (group, ms_r, ms_p, st))
    assert ms_p < 8.0, (ms_p, ms_r, st)


def test_big_repair_beside_another_connection(gpu):
    """The grid-barrier repair (every tile without a speculated entry)
    while another connection's GET steps fill the GPU on a second stream:
    fs_link's 16 workgroups wait in their barrier for the ones still
    queued behind the other stream's kernels, which drain in microseconds;
    the scan stays exact and far below the barrier's 0.5 s abandon (no
    fallback to the serial repair)."""
    from zkmi.bench.synthetic import GpuTree, GetPipeline
    rng = np.random.default_rng(29)
    lens = rng.integers(88, 1113, 60000)
    buf, starts = _stream(rng, lens)
    dev = torch.device('cuda', 0)
    d = torch.from_numpy(buf).to(dev)
    sc = B.FrameScanner(len(lens) + 16, dev, window=2048)
    sc.scan(d, len(buf), nospec=True)                   # warm
    tree = GpuTree(100_000, 100, fanout=100, device=dev)
    pipe = GetPipeline(tree, 1 << 18)
    pipe.step()
    torch.cuda.synchronize()
    other = torch.cuda.Stream(dev)
    worst = 0.0
    for _ in range(3):
        with torch.cuda.stream(other):
            for _ in range(12):
                pipe.step()
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record()
        ft = sc.scan(d, len(buf), nospec=True)
        t1.record()
        torch.cuda.synchronize()
        worst = max(worst, t0.elapsed_time(t1))
        r = ft.host_result()
        off = ft.off[:min(r['frames'], len(lens))].cpu().numpy()
        _check(r, off, buf, starts)
    assert worst < 20.0, worst
