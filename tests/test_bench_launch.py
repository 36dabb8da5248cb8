"""bench.py's own multi-rank launch: ``--gpus N`` outside torchrun starts
N rank processes (RANK / WORLD_SIZE / MASTER_* on 127.0.0.1) and rank 0
prints one JSON line with ``n_gpus == N``.  Runs the ensemble workload,
which works without a GPU (gloo, host decode)."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize('n', [2, 8])
def test_bench_gpus_flag_launches_ranks(n):
    env = {k: v for k, v in os.environ.items()
           if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR',
                        'MASTER_PORT')}
    out = subprocess.run(
        [sys.executable, 'bench.py', '--gpus', str(n), '--workload',
         'ensemble', '--steps', '2', '--warmup', '1', '--paths', '32',
         '--writes', '8', '--failover-every', '2'],
        cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
        text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec['n_gpus'] == n and rec['steps'] == 2 and rec['warmup'] == 1
    assert rec['value'] > 0 and rec['backend'] == 'gloo'
    assert rec['failovers'] >= 1


def test_bench_gpus_flag_fails_as_a_whole():
    """One rank failing ends the launch with a non-zero code (the others
    are stopped, not left waiting in a collective)."""
    env = dict(os.environ, ZKMI_BENCH_FAIL_RANK='1')
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK'):
        env.pop(k, None)
    out = subprocess.run(
        [sys.executable, 'bench.py', '--gpus', '2', '--workload',
         'ensemble', '--steps', '1', '--warmup', '0', '--paths', '8',
         '--writes', '4'],
        cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
        text=True, timeout=300)
    assert out.returncode != 0
