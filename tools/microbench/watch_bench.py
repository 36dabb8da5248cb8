"""Watchers the reference way at scale: N paths, watcher(p).on('dataChanged')
each, one bulk write firing every watch, the re-arms; timed with the native
watch engine and with the Python ZKWatchEvent state machines
(``ClientConfig(native_watch=False)``), against the native server.

    python tools/microbench/watch_bench.py [--n 20000] [--rounds 3]
"""
import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..',
                                'tests'))
from zkmi.server import fast  # noqa: E402
from zkhelpers import client, fast_config  # noqa: E402


def run(n, rounds, native):
    srv = fast.FastZKServer(preload=n, data_bytes=8, fanout=1000)
    try:
        c = client([srv.address], config=fast_config(native_watch=native))
        w = client([srv.address])
        c.wait_connected(10)
        w.wait_connected(10)
        paths = ['/bench/d%06d/n%09d' % (i // 1000, i) for i in range(n)]
        lock = threading.Lock()
        cnt = [0]
        done = threading.Event()
        want = [n]

        def on(data, stat):
            with lock:
                cnt[0] += 1
                if cnt[0] == want[0]:
                    done.set()
        t0 = time.perf_counter()
        for p in paths:
            c.watcher(p).on('dataChanged', on)
        assert done.wait(120)
        arm = time.perf_counter() - t0
        fire = []
        for r in range(rounds):
            done.clear()
            want[0] += n
            t0 = time.perf_counter()
            res = w.call_sync('bulk_set', paths, b'r%d' % r)
            assert res.ok_count() == n
            assert done.wait(120)
            fire.append(time.perf_counter() - t0)
        c.close_sync(10)
        w.close_sync(10)
        return {'native_watch': native, 'n': n, 'arm_s': round(arm, 4),
                'fire_rearm_s': [round(x, 4) for x in fire],
                'events_per_s': round(n / min(fire))}
    finally:
        srv.shutdown()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=20000)
    ap.add_argument('--rounds', type=int, default=3)
    a = ap.parse_args()
    for native in (True, False):
        print(json.dumps(run(a.n, a.rounds, native)), flush=True)


if __name__ == '__main__':
    main()
