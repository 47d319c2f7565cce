"""Spawn targets of the multi-process decomposition tests (gloo, world_size > 1)."""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, HERE):
    if p not in sys.path:
        sys.path.insert(0, p)


def _init(rank, world, port):
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    return dist


def worker(rank, world, port, name, engine, out, model_dir=None, tile=None):
    """Evaluate system `name` decomposed over `world` ranks; rank 0 saves
    the gathered energy / virial / forces / atomic energies to `out`.
    ``model_dir``: another deployment (HIP engine; its species list), ``tile``:
    replicate the system's cell (nx, ny, nz) first."""
    import torch
    if engine == 'cpu':
        # one thread per rank: the repeated-evaluation check compares bits, and
        # a multi-threaded CPU BLAS may split its sums differently from call to
        # call when the ranks compete for the host's cores (seen once, 4 ranks)
        torch.set_num_threads(1)
    dist = _init(rank, world, port)
    from _systems import load_manifest_symbols, system
    from sevennet_finetuning_amd.parallel import (ParallelE3GNN, brick_grid, build_rank_graph,
                                                  gather_all)
    syms = load_manifest_symbols() if model_dir is None else \
        json.load(open(os.path.join(model_dir, 'manifest.json')))['chemical_symbols']
    pos, cell, types = system(name, syms)
    if tile is not None:
        from sevennet_finetuning_amd.structures import tile as tile_cells
        n0 = len(pos)
        pos, cell = tile_cells(pos, cell, tuple(tile))
        types = np.tile(types, len(pos) // n0)
    cutoff = 5.0 if model_dir is None else \
        float(json.load(open(os.path.join(model_dir, 'manifest.json')))['cutoff'])
    rg = build_rank_graph(pos, cell, types, cutoff, brick_grid(world), rank)
    if engine == 'cpu':
        from _segment_cpu import make_engine
        eng = make_engine(rg)
    else:
        from sevennet_finetuning_amd.model import E3GNNModel
        from sevennet_finetuning_amd.parallel import HipSegmentEngine
        torch.cuda.set_device(0)
        eng = HipSegmentEngine(E3GNNModel(device='cuda:0') if model_dir is None else
                               E3GNNModel(model_dir, device='cuda:0'))
    drv = ParallelE3GNN(eng)
    drv.set_graph(rg)
    # several evaluations of one neighbour list: the rank graph is uploaded
    # once (set_graph), every evaluation gives the same result
    res = drv.evaluate()
    first = (float(res['energy']), res['forces'].detach().cpu().clone())
    # the bench's serial-exchange timing pass gives the same result too
    tm = {}
    res = drv.evaluate(timing=tm)
    same = first[0] == float(res['energy']) and torch.equal(first[1], res['forces'].detach().cpu())
    timed_ok = tm.get("exchanges") == 2 * (eng.num_layers - 1) + 1 and 0 < tm["exchange_s"] < tm["total_s"]
    res = drv.evaluate()
    same = same and first[0] == float(res['energy']) and torch.equal(first[1],
                                                                     res['forces'].detach().cpu())
    uploads = getattr(eng, 'uploads', -1)
    f, ea = gather_all(res, len(pos))
    if rank == 0:
        np.savez(out, energy=float(res['energy']), virial=res['virial'].cpu().numpy(),
                 forces=f.numpy(), atomic=ea.numpy(), repeat_same=np.array([same]),
                 uploads=np.array([uploads]), timed_ok=np.array([timed_ok]),
                 n_ghost=np.array([rg.n_ghost]), n_local=np.array([rg.n_local]))
    dist.barrier()
    dist.destroy_process_group()
