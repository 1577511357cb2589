"""bench.py --gpus N with no launcher around it starts N rank processes itself (RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_* as torchrun sets them), before any GPU call in the parent.  --plan-only
makes every rank print its environment and shard plan and exit before touching the GPU, so the
launcher and the plan are checked here on the CPU.  (The reference's counterpart: the N
validator processes of general_method_paper_reproduction.py:802-823.)"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, 'bench.py')


def _run(args, env_extra=None, drop=('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT')):
    env = {k: v for k, v in os.environ.items() if k not in drop}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True, timeout=300)


@pytest.mark.parametrize('n_gpus', [1, 4])
def test_launcher_plan_only(n_gpus):
    n = 1 << 16
    p = _run(['--gpus', str(n_gpus), '--plan-only', '--n', str(n)])
    assert p.returncode == 0, p.stderr
    recs = sorted((json.loads(l) for l in p.stdout.splitlines() if l.startswith('{')), key=lambda r: r['rank'])
    assert [r['rank'] for r in recs] == list(range(n_gpus))
    assert all(r['world'] == n_gpus and r['local_rank'] == r['rank'] for r in recs)
    if n_gpus > 1:
        assert len({r['master_port'] for r in recs}) == 1
        assert all(r['master_addr'] == '127.0.0.1' for r in recs)
    # contiguous shards covering the global batch, FLOP-balanced
    total = n * n_gpus
    assert all(r['total'] == total for r in recs)
    assert recs[0]['range'][0] == 0 and recs[-1]['range'][1] == total
    assert all(a['range'][1] == b['range'][0] for a, b in zip(recs, recs[1:]))
    assert sum(r['n'] for r in recs) == total
    ft = recs[0]['flops_total']
    assert abs(sum(r['flops'] for r in recs) - ft) <= 1e-9 * ft
    assert max(r['flops'] for r in recs) / (ft / n_gpus) < 1.001


def test_launcher_rejects_world_mismatch():
    p = _run(['--gpus', '2', '--plan-only', '--n', '1024'], env_extra={'WORLD_SIZE': '4', 'RANK': '0'})
    assert p.returncode != 0
    assert 'WORLD_SIZE' in p.stderr


def test_launcher_propagates_rank_failure():
    # an invalid size makes every rank fail; the launcher returns non-zero instead of hanging
    p = _run(['--gpus', '2', '--plan-only', '--n', '-5'])
    assert p.returncode != 0
