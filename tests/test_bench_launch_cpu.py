"""bench.py --gpus N: the launcher never ignores N.

Decision table (bench.launch_decision) and the spawn path end to end on CPU:
`python bench.py --gpus 2 --dry-run` starts two ranks under
torch.distributed.run as a child process, they join a gloo group and rank 0
reports world_size 2.  A WORLD_SIZE that disagrees with --gpus, or N > 1 with
fewer visible GPUs (no rehearsal requested), exits non-zero."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_decision_table():
    d = bench.launch_decision
    assert d(1, {}, 0) == ('run', None)
    assert d(1, {'WORLD_SIZE': '1'}, 1) == ('run', None)
    assert d(8, {'WORLD_SIZE': '8'}, 8) == ('run', None)
    assert d(8, {}, 8) == ('spawn', 'nccl')
    assert d(2, {}, 1)[0] == 'error'
    assert d(2, {'JDS_BENCH_REHEARSE': '1'}, 1) == ('spawn', 'gloo')
    assert d(2, {}, 0, dry_run=True) == ('spawn', 'gloo')
    act, msg = d(8, {'WORLD_SIZE': '2'}, 8)
    assert act == 'error' and 'WORLD_SIZE=2' in msg
    assert d(0, {}, 1)[0] == 'error'


def _env():
    env = dict(os.environ)
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT', 'JDS_BENCH_REHEARSE'):
        env.pop(k, None)
    env['CUDA_VISIBLE_DEVICES'] = ''
    env['HIP_VISIBLE_DEVICES'] = ''
    return env


def test_spawn_two_ranks_dry_run():
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '2', '--dry-run'],
                       capture_output=True, text=True, env=_env(), timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1
    rec = lines[0]
    assert rec['dry_run'] and rec['gpus_flag'] == 2 and rec['world_size'] == 2 and rec['rank_sum'] == 3.0


def test_mismatched_world_size_fails_loudly():
    env = _env()
    env['WORLD_SIZE'] = '2'
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '4'],
                       capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 2
    assert 'WORLD_SIZE=2' in r.stderr and not r.stdout.strip()


@pytest.mark.parametrize('gpus', [2, 8])
def test_more_gpus_than_visible_fails_loudly(gpus):
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', str(gpus)],
                       capture_output=True, text=True, env=_env(), timeout=180)
    assert r.returncode == 2
    assert 'GPU(s) visible' in r.stderr and not r.stdout.strip()
