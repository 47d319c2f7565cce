"""Diagnostic: repeatability of the decomposed HIP evaluation (two gloo ranks
sharing cuda:0).  Evaluates the same rank graph several times, plain and with
the serial-exchange timing pass, and prints per-rank max differences of the
energy, forces, atomic energies and virial against the first evaluation.

    python tools/diag_parallel_repeat.py [system] [world]
"""
import os
import socket
import sys

import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))


def worker(rank, world, port, name):
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from _systems import load_manifest_symbols, system
    from sevennet_finetuning_amd.model import E3GNNModel
    from sevennet_finetuning_amd.parallel import (HipSegmentEngine, ParallelE3GNN, brick_grid,
                                                  build_rank_graph)
    pos, cell, types = system(name, load_manifest_symbols())
    rg = build_rank_graph(pos, cell, types, 5.0, brick_grid(world), rank)
    torch.cuda.set_device(0)
    drv = ParallelE3GNN(HipSegmentEngine(E3GNNModel(device='cuda:0')))
    drv.set_graph(rg)
    ref = None
    for it, mode in enumerate(['plain', 'plain', 'timed', 'plain', 'timed', 'plain']):
        res = drv.evaluate(timing={} if mode == 'timed' else None)
        cur = {k: res[k].detach().double().cpu().clone() for k in ('energy', 'forces',
                                                                   'atomic_energy', 'virial')}
        if ref is None:
            ref = cur
            print(f'[rank {rank}] n_local {rg.n_local} n_ghost {rg.n_ghost} '
                  f'n_interior {rg.n_interior} edges {len(rg.center)} E {float(cur["energy"]):.9f}',
                  flush=True)
            continue
        d = {k: float((cur[k] - ref[k]).abs().max()) if cur[k].numel() else 0.0 for k in cur}
        if d['forces'] > 0:
            i = int((cur['forces'] - ref['forces']).abs().max(1).values.argmax())
            d['worst_row'] = i
        print(f'[rank {rank}] eval {it} ({mode}): ' + ', '.join(f'{k} {v:.3g}' for k, v in d.items()),
              flush=True)
    dist.barrier()
    dist.destroy_process_group()


def free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


if __name__ == '__main__':
    name = sys.argv[1] if len(sys.argv) > 1 else 'mixed_3x3x3'
    world = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    print(f'E3GNN_CONV={os.environ.get("E3GNN_CONV")}', flush=True)
    mp.spawn(worker, args=(world, free_port(), name), nprocs=world, join=True)
