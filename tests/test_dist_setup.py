"""The data-parallel fine-tune entry points (BASELINE config 5).

`train.setup_distributed()` must bind the rank's GPU before the RCCL process
group exists (reference: sevenn/main/sevenn.py:39-49 sets the device, then
init_process_group; trainer.py:19-24 puts the model on it), and
`bench_train.py --gpus N` must start its N ranks itself, like bench.py.
CPU only: torch.cuda and torch.distributed are monkeypatched.
"""
import os
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist

from sevennet_finetuning_amd import train

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _fake_cuda(monkeypatch, events, n_dev=8):
    monkeypatch.setattr(torch.cuda, 'is_available', lambda: True)
    monkeypatch.setattr(torch.cuda, 'device_count', lambda: n_dev)
    monkeypatch.setattr(torch.cuda, 'set_device', lambda d: events.append(('set_device', d)))
    monkeypatch.setattr(dist, 'is_initialized', lambda: any(e[0] == 'init' for e in events))
    monkeypatch.setattr(dist, 'init_process_group',
                        lambda backend, **kw: events.append(('init', backend, kw)))
    monkeypatch.setattr(dist, 'get_rank', lambda: 5)
    monkeypatch.setattr(dist, 'get_world_size', lambda: 8)


def test_setup_distributed_binds_the_local_gpu_before_rccl(monkeypatch):
    events = []
    _fake_cuda(monkeypatch, events)
    monkeypatch.setenv('LOCAL_RANK', '5')
    rank, world, local, device = train.setup_distributed()
    assert (rank, world, local) == (5, 8, 5)
    assert device == torch.device('cuda', 5)
    assert [e[0] for e in events] == ['set_device', 'init']
    assert events[0][1] == torch.device('cuda', 5)
    _, backend, kw = events[1]
    assert backend == 'nccl' and kw == {'device_id': torch.device('cuda', 5)}


def test_setup_distributed_refuses_a_rank_without_its_gpu(monkeypatch):
    events = []
    _fake_cuda(monkeypatch, events, n_dev=1)
    monkeypatch.setenv('LOCAL_RANK', '3')
    with pytest.raises(RuntimeError, match='LOCAL_RANK=3'):
        train.setup_distributed()
    assert events == []


def test_setup_distributed_on_cpu_is_gloo(monkeypatch):
    events = []
    _fake_cuda(monkeypatch, events)
    monkeypatch.setattr(torch.cuda, 'is_available', lambda: False)
    monkeypatch.setenv('LOCAL_RANK', '0')
    *_, device = train.setup_distributed()
    assert device == torch.device('cpu')
    assert events == [('init', 'gloo', {})]


def _run_bench_train(monkeypatch, argv):
    sys.path.insert(0, ROOT)
    import bench_train
    monkeypatch.setattr(sys, 'argv', ['bench_train.py', *argv])
    bench_train.main()


def test_bench_train_gpus_n_starts_n_ranks(monkeypatch):
    monkeypatch.delenv('WORLD_SIZE', raising=False)
    calls = []
    monkeypatch.setattr(subprocess, 'call', lambda cmd: calls.append(cmd) or 0)
    # the launcher process must not touch the GPU
    monkeypatch.setattr(torch.cuda, 'set_device', lambda d: pytest.fail('GPU touched'))
    argv = ['--gpus', '8', '--steps', '3']
    with pytest.raises(SystemExit) as ex:
        _run_bench_train(monkeypatch, argv)
    assert ex.value.code == 0
    (cmd,) = calls
    assert cmd[:3] == [sys.executable, '-m', 'torch.distributed.run']
    assert '--nproc-per-node=8' in cmd and '--master-addr=127.0.0.1' in cmd
    i = cmd.index(os.path.join(ROOT, 'bench_train.py'))
    assert cmd[i + 1:] == argv


def test_bench_train_rank_world_must_match(monkeypatch):
    monkeypatch.setenv('WORLD_SIZE', '2')
    monkeypatch.setattr(subprocess, 'call', lambda cmd: pytest.fail('relaunched'))
    with pytest.raises(RuntimeError, match=r'bench_train.py --gpus 4 but WORLD_SIZE=2'):
        _run_bench_train(monkeypatch, ['--gpus', '4'])


@pytest.mark.parametrize('device', ['cpu', torch.device('cpu')])
def test_calculator_refuses_cpu_device(device):
    """Config 1 asks for the calculator 'on CPU'; the reference runs its torch
    model there (sevennet_calculator.py:57-65).  This build has no CPU engine
    and must say so before loading anything -- never fall back silently."""
    from sevennet_finetuning_amd.sevennet_calculator import SevenNetCalculator
    with pytest.raises(ValueError, match=r"device='cpu'.*HIP library.*no CPU path"):
        SevenNetCalculator('7net-0', device=device)
    with pytest.raises(ValueError, match='torch.device or str'):
        SevenNetCalculator('7net-0', device=0)
