"""Benchmark of the fine-tune step (BASELINE config 5).

``python bench_train.py --gpus N --steps K --warmup W`` (N > 1: one process
per GPU over RCCL; started under torchrun, or it launches its N ranks itself).  A step = one iteration of the reference's
RehearsalTrainer.run_one_epoch_rehearsal (trainer.py:174-206) with the
FT_w_reEWC recipe (Huber delta 0.01, force weight 1, stress weight 0.01, EWC
lambda 1e5, Adam): forward + force/stress (create_graph) + loss backward
(double backward through the HIP convolution kernels) + gradient all-reduce +
Adam step on a batch of 8 structures, then the same on a memory batch of 8.
Structures: 54-atom primitive diamond cells (3x3x3), species drawn from
{Li, P, S, Cl}, N(0, 0.05 A) displacements, rc = 5 A; synthetic labels
(energy -4 eV/atom + noise, forces/stress noise; default_rng(2)); synthetic
Fisher (the reference's fisher_sevenn.pt does not travel to the GPU box).
Every rank draws its own batches (weak scaling: 16 structures per rank per
step).  value = structures processed by all ranks / max-over-ranks time.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def log(msg):
    if int(os.environ.get('RANK', '0')) == 0:
        print(f'[bench_train] {msg}', file=sys.stderr, flush=True)


def make_batches(rank, n_batches, batch_size, symbols):
    from sevennet_finetuning_amd import train
    from sevennet_finetuning_amd.structures import diamond_primitive, mixed_symbols
    rng = np.random.default_rng(2)
    graphs = []
    for k in range(n_batches * batch_size):
        seed = 10_000 * rank + k
        pos, cell = diamond_primitive((3, 3, 3), sigma=0.05, seed=seed)
        types = [symbols.index(s) for s in mixed_symbols(len(pos), seed=seed + 1)]
        graphs.append(train.labeled_graph(
            pos, cell, types, 5.0, energy=-4.0 * len(pos) + rng.normal(0, 0.5),
            force=rng.normal(0, 0.3, (len(pos), 3)), stress=rng.normal(0, 2e-3, 6)))
    return [graphs[i * batch_size:(i + 1) * batch_size] for i in range(n_batches)]


def cpu_baseline(batches, cfg, seconds):
    """The same rehearsal step on the host CPU: the trainable model with the
    oracle's uvu tensor product (tests/_conv_cpu.py, plain PyTorch, fp32) in
    place of the HIP kernels, all host threads of this process's share."""
    sys.path.insert(0, os.path.join(ROOT, 'tests'))
    from _conv_cpu import CpuConvBackend
    from sevennet_finetuning_amd import train
    from sevennet_finetuning_amd.nn import SevenNetTrainable
    threads = min(len(os.sched_getaffinity(0)), int(os.environ.get('OMP_NUM_THREADS', '16')))
    torch.set_num_threads(threads)
    model = SevenNetTrainable(device='cpu', conv_backend=CpuConvBackend())
    c = dict(cfg, device='cpu', is_ddp=False, hip_graph=False, explicit_grad=False)
    c['continue'] = dict(cfg['continue'],
                         fisher_information={k: v.cpu() for k, v in
                                             cfg['continue']['fisher_information'].items()},
                         opt_params={k: v.cpu() for k, v in
                                     cfg['continue']['opt_params'].items()})
    tr = train.Trainer(model, c)
    model.train(True)
    b = [train.collate(x, dtype=torch.float32) for x in batches[:2]]
    t0, n = time.perf_counter(), 0   # ~17 s per step on 8 cores: no separate warm step
    while time.perf_counter() - t0 < seconds:
        tr.rehearsal_step(b[0], b[1])
        n += 1
    dt = time.perf_counter() - t0
    structs = n * sum(len(x) for x in batches[:2])
    return {'value': round(structs / dt, 3), 'unit': 'structures/s', 'cores': threads,
            'kind': 'port',
            'sample': f'{n} rehearsal steps (2 x {len(batches[0])} structures) in {dt:.1f} s, '
                      'trainable model + oracle uvu TP (tests/_conv_cpu.py), torch CPU fp32'}


def step_bench(device, steps, warmup, batch=8, rank=0, world=1, eager=False, autograd=False,
               blas='rocblas'):
    """The timed rehearsal step (module docstring) on `device`: builds the
    model, the synthetic batches and the trainer, runs `warmup` untimed and
    `steps` timed steps (barrier + synchronize around the timed region, max
    over ranks).  Returns a dict of the measurement (bench.py's fine_tune
    leg uses it too)."""
    from sevennet_finetuning_amd import train
    from sevennet_finetuning_amd.nn import SevenNetTrainable
    model = SevenNetTrainable(device=device)
    fisher = {n: torch.full_like(p, 1e-3) for n, p in model.named_parameters()}
    opt = {n: p.detach().clone() for n, p in model.named_parameters()}
    cfg = {'loss': 'huber', 'loss_param': {'delta': 0.01}, 'force_loss_weight': 1.0,
           'stress_loss_weight': 0.01, 'is_train_stress': True, 'optimizer': 'adam',
           'optim_param': {'lr': 1e-5}, 'scheduler': 'exponentiallr',
           'scheduler_param': {'gamma': 0.99}, 'is_ddp': world > 1, 'device': device,
           'hip_graph': not eager, 'explicit_grad': not autograd, 'blas': blas,
           'continue': {'fisher_information': fisher, 'opt_params': opt, 'ewc_lambda': 1e5}}
    tr = train.Trainer(model, cfg)
    n_b = 4
    batches = make_batches(rank, 2 * n_b, batch, model.chemical_symbols)
    dev_batches = [train.collate(b, device=device, dtype=torch.float32) for b in batches]
    atoms_per_step = sum(int(b['num_atoms'].sum()) for b in dev_batches[:2])
    edges = int(dev_batches[0]['edge_index'].shape[1])
    log(f'{batch} x 54-atom structures per batch, {edges} edges; rank {rank}/{world}')
    model.train(True)

    def step(i):
        b, m = dev_batches[(2 * i) % (2 * n_b)], dev_batches[(2 * i + 1) % (2 * n_b)]
        return tr.rehearsal_step(b, m)

    def barrier():
        if world > 1:
            torch.distributed.barrier()

    for i in range(warmup):
        step(i)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        loss, mloss = step(i)
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=device)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t)
    structs = 2 * batch * world * steps
    return {'ms_per_step': dt / steps * 1e3, 'structures_per_s': structs / dt,
            'atoms_per_s': atoms_per_step * world * steps / dt, 'atoms_per_rank_step': atoms_per_step,
            'edges_per_batch': edges, 'loss': float(loss), 'mem_loss': float(mloss),
            'hip_graph': bool(tr.hip_graph), 'explicit_grad': tr.explicit is not None,
            'gemm': ('libe3gnn_hip e3gnn_gemm_grouped (no rocBLAS / hipBLASLt kernel)'
                     if tr.explicit is not None and tr.explicit.gm.lib is not None
                     else f'torch ({blas})'),
            'batches': batches, 'cfg': cfg}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--batch', type=int, default=8)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--eager', action='store_true',
                    help='no HIP-graph capture of the step (for N > 1 the graphed step '
                         'is three captured segments around the two gradient all-reduces)')
    ap.add_argument('--cpu-seconds', type=float, default=10.0)
    ap.add_argument('--blas', default='rocblas', choices=['rocblas', 'hipblaslt'],
                    help='torch GEMM backend for the linears and the radial MLP')
    ap.add_argument('--autograd', action='store_true',
                    help='the loss gradient by autograd double backward instead of the '
                         'hand-scheduled derivatives (train_explicit.py)')
    args = ap.parse_args()
    import bench
    # `--gpus N` without a launcher: start the N ranks as children before this
    # process touches the GPU, and exit with their code (bench.py's contract)
    rc = bench.maybe_launch(args, sys.argv[1:], script=__file__)
    if rc is not None:
        sys.exit(rc)
    world = int(os.environ.get('WORLD_SIZE', '1'))
    bench.check_world(args, world, 'bench_train.py')
    from sevennet_finetuning_amd import train
    if world > 1:
        rank, world, local, device = train.setup_distributed()
    else:
        rank, local, device = 0, 0, torch.device('cuda', 0)
        torch.cuda.set_device(device)

    r = step_bench(device, args.steps, args.warmup, args.batch, rank, world, args.eager,
                   args.autograd, args.blas)
    ms, batches, cfg = r['ms_per_step'], r['batches'], r['cfg']
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log('cpu baseline ...')
        cpu = cpu_baseline(batches, cfg, args.cpu_seconds)
    if rank == 0:
        print(json.dumps({
            'metric': 'structures/sec fine-tune step (rehearsal + EWC), SevenNet-0',
            'value': round(r['structures_per_s'], 2), 'unit': 'structures/s', 'n_gpus': world,
            'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(ms, 3),
            'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
            'dtype': 'f32 (radial-MLP W2 products on bf16x6 MFMA pieces: f32-grade)',
            'data': 'synthetic 54-atom mixed-species diamond cells, synthetic labels/Fisher',
            'config': {'workload': f'rehearsal step: 2 x {args.batch} structures per rank '
                                   f'({r["atoms_per_rank_step"]} atoms), force+stress+energy Huber + EWC, '
                                   'Adam, grad all-reduce',
                       'atoms_per_rank_step': r['atoms_per_rank_step'],
                       'edges_per_batch': r['edges_per_batch'],
                       'parallelism': f'dp{world}',
                       'hip_graph': r['hip_graph'], 'explicit_grad': r['explicit_grad'],
                       # which GEMMs ran: the library's grouped GEMM (no vendor
                       # BLAS kernel in the step) or torch's with the --blas choice
                       'gemm': r['gemm']},
            'atoms_per_s': round(r['atoms_per_s'], 1),
            'loss': r['loss'], 'mem_loss': r['mem_loss'], 'cpu_baseline': cpu}), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == '__main__':
    main()
