"""bench.py's multi-rank launch contract (driver: ``python bench.py --gpus N``).

Without a launcher around it, ``--gpus N`` (N > 1) must start N local ranks
as child processes and every rank must see WORLD_SIZE == N; a mismatch is an
error, never a silent one-GPU run labelled with the wrong n_gpus.  The GPU
test runs the real thing: two ranks on one device (gloo), no launcher.
"""
import json
import os
import subprocess
import sys

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _args(argv):
    old = sys.argv
    try:
        sys.argv = ['bench.py', *argv]
        return bench.parse()
    finally:
        sys.argv = old


def test_single_gpu_runs_in_process(monkeypatch):
    monkeypatch.delenv('WORLD_SIZE', raising=False)
    assert bench.maybe_launch(_args([]), []) is None
    assert bench.maybe_launch(_args(['--gpus', '1']), ['--gpus', '1']) is None


def test_rank_under_a_launcher_does_not_relaunch(monkeypatch):
    monkeypatch.setenv('WORLD_SIZE', '4')
    assert bench.maybe_launch(_args(['--gpus', '4']), ['--gpus', '4']) is None


def test_gpus_n_starts_n_ranks(monkeypatch):
    monkeypatch.delenv('WORLD_SIZE', raising=False)
    calls = []
    monkeypatch.setattr(subprocess, 'call', lambda cmd: calls.append(cmd) or 0)
    argv = ['--gpus', '8', '--steps', '3']
    assert bench.maybe_launch(_args(argv), argv) == 0
    (cmd,) = calls
    assert cmd[:3] == [sys.executable, '-m', 'torch.distributed.run']
    assert '--nproc-per-node=8' in cmd and '--nnodes=1' in cmd
    assert '--master-addr=127.0.0.1' in cmd
    port = [c for c in cmd if c.startswith('--master-port=')]
    assert len(port) == 1 and int(port[0].split('=')[1]) > 0
    i = cmd.index(os.path.abspath(bench.__file__))
    assert cmd[i + 1:] == argv


def test_world_must_match_gpus():
    bench.check_world(_args(['--gpus', '2']), 2)
    with pytest.raises(RuntimeError, match='WORLD_SIZE=1'):
        bench.check_world(_args(['--gpus', '2']), 1)
    with pytest.raises(RuntimeError):
        bench.check_world(_args([]), 8)


def test_exit_code_of_the_ranks_is_returned(monkeypatch):
    monkeypatch.delenv('WORLD_SIZE', raising=False)
    monkeypatch.setattr(subprocess, 'call', lambda cmd: 3)
    assert bench.maybe_launch(_args(['--gpus', '2']), ['--gpus', '2']) == 3


@pytest.mark.gpu
def test_bench_gpus_2_without_launcher():
    """Two ranks sharing the one device (gloo, host-staged halos), started by
    bench.py itself: the JSON line says n_gpus 2, the process group saw 2
    ranks, the full-size property check through the halo exchanges passed."""
    env = {k: v for k, v in os.environ.items()
           if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT')}
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '2',
                        '--same-device', '--steps', '2', '--warmup', '1', '--cells', '6',
                        '--no-cpu-baseline'], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out['n_gpus'] == 2
    assert out['parity_check']['ok']
    d = out['distributed']
    assert d['backend'] == 'gloo' and d['world_size'] == 2
    assert [x['rank'] for x in d['ranks']] == [0, 1]
    assert sum(x['owned'] for x in d['ranks']) == 2 * 8 * 6 ** 3   # weak: 6^3 cells per rank
    assert all(x['ghosts'] > 0 and x['exchange_ms'] > 0 for x in d['ranks'])
    assert d['exchanges_per_step'] == 9   # 4 forward, 4 reverse, 1 ghost-force reverse


@pytest.mark.parametrize('argv,world,n_total,needle', [
    ([], 1, 97336, '97,336-atom box @1 GPU'),
    (['--gpus', '8'], 8, 778688, '97,336-atom box per GPU = 778,688-atom box @8 GPUs (weak scaling)'),
    (['--gpus', '8', '--strong'], 8, 778688, '778,688-atom box split over 8 GPUs (strong scaling)'),
    (['--strong'], 1, 778688, '778,688-atom box @1 GPU'),
])
def test_bench_line_names_the_evaluated_box(argv, world, n_total, needle):
    """The metric / workload of a bench line name the box actually evaluated:
    a weak --gpus 8 line is the 778,688-atom box (config 4), so is --strong."""
    import numpy as np
    args = _args(argv)
    cells, grid, total = bench.box_plan(args, world)
    assert 8 * int(np.prod(total)) == n_total
    assert (grid == (2, 2, 2)) == (world == 8)
    metric, work = bench.describe(n_total, world, cells, args.strong, grid)
    assert metric.startswith('atoms/sec energy+force, SevenNet-0 lmax=2, ')
    assert needle in metric, metric
    assert f'{n_total:,}-atom' in work
