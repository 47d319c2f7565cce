"""Benchmark: atoms/s of one SevenNet-0 energy+force(+virial) evaluation.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W`` prints ONE
JSON line on rank 0.  A step = one full evaluation through the C ABI
(graph indices + edge embedding + 5 interaction blocks + readout + the
complete force/virial backward) of a synthetic periodic Si diamond box
(a = 5.43 A, 23^3 conventional cells = 97,336 atoms,
default_rng(0) N(0, 0.05 A) displacements, rc = 5 A, 2,725,408 edges), with
the inputs already resident in HBM.  Neighbour list built once on the host
before timing ("graph prebuilt").

N > 1: one process per GPU (torchrun), spatial domain decomposition
(parallel.py, the reference's e3gnn/parallel path): the box grows with N
(23^3 cells per rank in a px x py x pz brick grid, e.g. 46^3 cells = 778,688
atoms on 8 GPUs) -- weak scaling -- and every step does the per-layer ghost
feature exchange, the reverse gradient and ghost-force exchanges (RCCL
all_to_all) and the energy/virial all_reduce.  ``--strong``: one 46^3-cell
box (778,688 atoms, north_star's 800k config) split over the N ranks, N = 1
included (one device holds it).  The timed region is bracketed by barrier +
synchronize; the max over ranks is reported and value = total atoms / that
time.  The rank graph is uploaded once (a step moves no host data, like the
single-device step).

Before timing, a full-size property check runs at the same size (a displaced
8-atom cell tiled to the box: E = k^3 E_cell, per-image forces equal; through
the halo exchanges when N > 1) and the run fails if it does not hold.

Also reported: ``roofline`` for the dominant kernel class (HIP-event timed
inside the library, on the stream the kernels run on) and ``cpu_baseline``
(the oracle CPU restatement timed on this host on a bounded sample).
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

PEAK_FP32_TFLOPS = 157.3   # MI355X FP32 matrix = vector peak (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0      # MI355X HBM3E peak
# what the step computes in: f32 data and accumulation everywhere; the radial
# MLP's matrix products (and the wide node linears) on bf16 MFMA with f32
# operands split into bf16 pieces -- six piece products (f32-grade) where the
# energy is formed, three (~2^-16 relative) for the backward's dH2 = dw W2^T
# and its w recompute
DTYPE = 'f32 (MLP / linear products on bf16 MFMA pieces: bf16x6 fwd, bf16x3 bwd)'


def log(msg):
    if int(os.environ.get('RANK', '0')) == 0:
        print(f'[bench] {msg}', file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--cells', type=int, default=None,
                    help='n for an n^3 conventional-cell box: per rank (weak scaling, default '
                         '23) or in total (--strong, default 46)')
    ap.add_argument('--strong', action='store_true',
                    help='strong scaling: one --cells^3 box (default 46^3 = 778,688 atoms, '
                         'north_star config 4) split over the N ranks')
    ap.add_argument('--no-parity-check', action='store_true')
    ap.add_argument('--cpu-cells', type=int, default=11,
                    help='cpu_baseline sample: n^3 cells (11 -> 10,648 atoms, SURVEY.md 8d)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-seconds', type=float, default=15.0)
    ap.add_argument('--same-device', action='store_true',
                    help='N > 1 rehearsal: every rank on cuda:0, gloo instead of RCCL')
    ap.add_argument('--profile-only', action='store_true',
                    help='warmup + steps only, no stats pass (for rocprofv3)')
    ap.add_argument('--system', default='si', choices=['si', 'hfo2'],
                    help='si: the displaced Si diamond box (BASELINE config 3); hfo2: the '
                         "reference's example HfO2 snapshot (res.dat, 96 atoms, non-uniform "
                         'degree) tiled --cells^3 times (default 10^3 = 96,000 atoms), N = 1')
    ap.add_argument('--rank-emulation', default=None, metavar='R[,R...]',
                    help='N = 1 only: build every rank graph of the --strong box (default 46^3 '
                         'cells = 778,688 atoms) split over --emulate-world ranks, time the listed '
                         'ranks one at a time on this GPU (ParallelE3GNN.evaluate with each '
                         'all_to_all replaced by a same-size local copy: compute + halo kernels, '
                         'no network) and the whole box on this GPU; prints one JSON line')
    ap.add_argument('--emulate-world', type=int, default=8)
    ap.add_argument('--no-fine-tune', action='store_true',
                    help='skip the fine_tune leg (N = 1: the fine-tune rehearsal step of '
                         'BASELINE config 5, bench_train.step_bench, timed after the main line)')
    ap.add_argument('--model-config', default=None, metavar='cCHlL',
                    help='instead of SevenNet-0: the SevenNet-0 preset with channel CH and L '
                         'blocks (e.g. c64l4), built by model_build (e3nn init, seed 0) and '
                         'deployed to a temporary directory')
    return ap.parse_args()


def make_box(cells, device, si=69):
    from sevennet_finetuning_amd.neighbor import neighbor_list
    from sevennet_finetuning_amd.structures import si_diamond
    pos, cell = si_diamond((cells,) * 3, sigma=0.05)
    order = os.environ.get('E3GNN_BENCH_ORDER')   # experiment: atom order of the box
    if order == 'morton':
        from sevennet_finetuning_amd.structures import morton_order
        pos = pos[morton_order(pos, cell, 2.7)]
    t0 = time.perf_counter()
    ei, sh = neighbor_list(pos, cell, 5.0)
    host_nl_s = time.perf_counter() - t0
    vec = pos[ei[1]] + sh @ cell - pos[ei[0]]
    return {
        'pos': pos, 'cell': cell, 'host_nl_ms': host_nl_s * 1e3,
        'n': len(pos), 'E': ei.shape[1],
        'types': torch.full((len(pos),), si, dtype=torch.int32, device=device),  # Si
        'center': torch.tensor(ei[0], dtype=torch.int32, device=device),
        'nbr': torch.tensor(ei[1], dtype=torch.int32, device=device),
        'vec': torch.tensor(vec, dtype=torch.float32, device=device),
    }


HFO2_RESDAT = os.path.join(ROOT, 'sevennet_finetuning_amd', 'assets', 'structures', 'hfo2_resdat.npz')


def make_box_hfo2(k, device, symbols):
    """The reference's HfO2 example snapshot (example_inputs/md_serial_example
    res.dat: 96 atoms of a triclinic cell, 44.5 edges per atom at 5 A with a
    spread) tiled k^3 times: a box whose per-atom degree is NOT uniform, so the
    fused kernels' 16-edge tile padding and the lock-step backward's
    max-of-four tile counts are exercised as on a real MD configuration."""
    from sevennet_finetuning_amd.neighbor import neighbor_list
    from sevennet_finetuning_amd.structures import tile
    d = np.load(HFO2_RESDAT)
    types1 = np.array([symbols.index(str(x)) for x in d['symbols']], dtype=np.int64)
    pos, cell = tile(d['pos'], d['cell'], (k, k, k))
    types = np.tile(types1, k ** 3)
    t0 = time.perf_counter()
    ei, sh = neighbor_list(pos, cell, 5.0)
    host_nl_s = time.perf_counter() - t0
    vec = pos[ei[1]] + sh @ cell - pos[ei[0]]
    e1, s1 = neighbor_list(d['pos'], d['cell'], 5.0)
    return {
        'pos': pos, 'cell': cell, 'host_nl_ms': host_nl_s * 1e3, 'n': len(pos), 'E': ei.shape[1],
        'types': torch.tensor(types, dtype=torch.int32, device=device),
        'center': torch.tensor(ei[0], dtype=torch.int32, device=device),
        'nbr': torch.tensor(ei[1], dtype=torch.int32, device=device),
        'vec': torch.tensor(vec, dtype=torch.float32, device=device),
        'k': k, 'cell1': (d['pos'], d['cell'], types1, e1, s1), 'center_np': ei[0],
    }


def degree_stats(center, n, wpg=4):
    """Per-atom degree spread and what it costs the fused kernels: every
    centre's edges run in 16-edge tiles (padding = tile slots / edges), and
    the lock-step backward runs each workgroup of `wpg` consecutive centres
    for the max of their tile counts (imbalance = workgroup tile slots /
    the centres' own tiles)."""
    deg = np.bincount(np.asarray(center), minlength=n)
    tiles = (deg + 15) // 16
    m = (n // wpg) * wpg
    wg = tiles[:m].reshape(-1, wpg).max(axis=1).sum() * wpg + (tiles[m:].max() * (n - m) if n > m else 0)
    return {'edges_per_atom_mean': round(float(deg.mean()), 3), 'min': int(deg.min()),
            'max': int(deg.max()), 'std': round(float(deg.std()), 3),
            'tile_padding': round(float(tiles.sum() * 16 / max(deg.sum(), 1)), 4),
            'lockstep_imbalance': round(float(wg / max(tiles.sum(), 1)), 4)}


def parity_check_tiled(model, box, device):
    """E(k^3-tiled box) = k^3 E(cell) and per-image forces equal, on the box
    the bench times (make_box_hfo2)."""
    pos1, cell1, types1, ei, sh = box['cell1']
    vec1 = pos1[ei[1]] + sh @ cell1 - pos1[ei[0]]
    t = lambda a, dt=torch.int32: torch.as_tensor(a, dtype=dt, device=device)
    one = model.energy_forces(t(types1), t(ei[0]), t(ei[1]), t(vec1, torch.float32))
    e1, f1 = float(one['energy']), one['forces'].cpu().numpy()
    big = model.energy_forces(box['types'], box['center'], box['nbr'], box['vec'])
    k3 = box['k'] ** 3
    de = abs(float(big['energy']) - k3 * e1) / abs(k3 * e1)
    df = float(np.abs(big['forces'].cpu().numpy().reshape(k3, len(pos1), 3) - f1[None]).max())
    return {'property': f'res.dat tiled {box["k"]}^3, {box["n"]} atoms: E = k^3 E_cell, '
                        'per-image forces equal', 'energy_rel_err': de, 'max_force_err': df,
            'ok': bool(de <= 2e-6 and df <= 1e-4)}


def device_nl_timing(box, device, reps=5):
    """Graph build on the GPU (e3gnn_nlist_*, the step in front of the hot
    path; outside the timed region): best of `reps`, positions already on the
    device; checks the edge count against the host list."""
    from sevennet_finetuning_amd.neighbor import DeviceNeighborList
    nl = DeviceNeighborList(device)
    pos = torch.tensor(box['pos'], dtype=torch.float64, device=device)
    best = None
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        c, _, _, _ = nl(pos, box['cell'], 5.0)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    if c.numel() != box['E']:
        raise RuntimeError(f'device neighbour list: {c.numel()} edges, host {box["E"]}')
    return {'device_ms': round(best * 1e3, 3), 'host_ms': round(box['host_nl_ms'], 1),
            'edges': int(c.numel())}


# template arguments of the fused kernels' layer structs per channel family
# (csrc/tp.h Family<f>): rocprofv3 prints e.g. k_conv_bwd_ls<e3gnn::LayerMidT<128, 64, 32> >
FAMILY_DIMS = {0: ('128', '128, 64, 32'), 1: ('64', '64, 64, 64'), 2: ('32', '32, 32, 32')}


def rocprof_name(cls, family=0):
    """Kernel symbol prefix (as rocprofv3 prints it) of a fused timing class
    of the given channel family (so PMC entries of another family's kernels
    never match)."""
    kinds = {'first': 'LayerFirst', 'mid': 'LayerMid', 'last': 'LayerLast'}
    if '.' in cls:  # template prefix
        k, kind = cls.split('.')
        if k == 'conv_bwd_x':
            # first / middle blocks: the lock-step kernel; the last block: one
            # wave per neighbour node
            k = 'conv_bwd_nbr' if kind == 'last' else 'conv_bwd_ls'
        first, rest = FAMILY_DIMS.get(family, FAMILY_DIMS[0])
        return f'k_{k}<e3gnn::{kinds[kind]}T<{first if kind == "first" else rest}>'
    return cls


PEAK_BF16_TFLOPS = 16 * 157.3   # dense bf16 MFMA (MI355X_MICROARCH.md: 1/16 ratio to f32)


def pmc_entry(kernel, cells):
    """The committed PMC summary entry (profiles/pmc_traffic.json) of `kernel`."""
    path = os.path.join(ROOT, 'profiles', 'pmc_traffic.json')
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None
    if d.get('cells') != cells:
        return None
    for k, v in d.get('kernels', {}).items():
        if kernel in k:
            return v
    return None


def mfma_fracs(kernel, cells, ms_per_launch):
    """Matrix-core rate of `kernel` by the precision its MFMA work runs in:
    executed FLOP per launch (SQ_INSTS_VALU_MFMA_MOPS_* x 512, committed PMC
    pass) / the launch time measured in this run, against that precision's
    dense peak.  The fused kernels run the radial MLP's products on bf16x6
    (six bf16 MFMAs per f32-grade product), so this counts the bf16 work the
    matrix cores did, not the algorithmic FLOP of `achieved`."""
    e = pmc_entry(kernel, cells)
    if not e or 'mfma_flop_bf16' not in e or not ms_per_launch:
        return None
    out = {}
    for prec, peak in (('bf16', PEAK_BF16_TFLOPS), ('f32', PEAK_FP32_TFLOPS)):
        f = e.get(f'mfma_flop_{prec}', 0)
        ach = f / (ms_per_launch * 1e9)
        out[prec] = {'flop_per_launch': f, 'achieved': round(ach, 2), 'peak': round(peak, 1),
                     'unit': 'TFLOP/s', 'frac': round(ach / peak, 4)}
    out['source'] = 'profiles/pmc_traffic.json (rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_*)'
    return out


def pmc_traffic(kernel, cells):
    """HBM bytes per launch of `kernel` from the committed PMC summary
    (tools/pmc_traffic.py: FETCH_SIZE x 2 (gfx950 correction) + WRITE_SIZE,
    separate rocprofv3 --pmc passes of this bench), or None."""
    path = os.path.join(ROOT, 'profiles', 'pmc_traffic.json')
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None
    if d.get('cells') != cells:
        return None
    for k, v in d.get('kernels', {}).items():
        if kernel in k:
            return v.get('bytes_per_launch')
    return None


def cpu_baseline(seconds, cells, model_dir=None):
    """Oracle (plain-PyTorch CPU restatement of the reference) on a bounded
    sample of the same workload: a cells^3 Si box (default 11^3 = 10,648
    atoms, SURVEY.md 8d's sample; the CPU path is NOT flat in box size --
    1,728 atoms ran at 65 and 10,648 at 115 atoms/s on 8 threads, so the
    smaller sample understated it), the same recipe as the bench box: one
    untimed warm-up call on a 64-atom box of the same lattice (allocator,
    thread pool, kernel selection), then >= 1 timed evaluation and >=
    `seconds` of CPU work on the host's thread share."""
    from oracle.neighbor import neighbor_list
    from oracle.nequip_ref import NequIPRef
    from oracle.sevennet_ref import SevenNet0Ref
    from sevennet_finetuning_amd.structures import si_diamond
    # the box's CPU share is OMP_NUM_THREADS (16); sched_getaffinity reports the
    # whole machine there, and oversubscribing it stalls the run
    threads = min(len(os.sched_getaffinity(0)), int(os.environ.get('OMP_NUM_THREADS', '16')))
    torch.set_num_threads(threads)
    log(f'cpu baseline: {threads} threads, {cells}^3 cells, ~{seconds:.0f} s')
    # --model-config: the same deployment on the family's restatement
    ref = SevenNet0Ref(dtype=torch.float32) if model_dir is None else \
        NequIPRef(model_dir, dtype=torch.float32)
    si = 69 if model_dir is None else ref.symbols.index('Si')
    pos, cell = si_diamond((cells,) * 3, sigma=0.05)
    ei, sh = neighbor_list(pos, cell, 5.0)
    args = (torch.tensor(pos, dtype=torch.float32), torch.full((len(pos),), si),
            torch.tensor(ei), torch.tensor(sh, dtype=torch.float32),
            torch.tensor(cell, dtype=torch.float32))
    pw, cw = si_diamond((2, 2, 2), sigma=0.05)
    ew, sw = neighbor_list(pw, cw, 5.0)
    ref(torch.tensor(pw, dtype=torch.float32), torch.full((len(pw),), si), torch.tensor(ew),
        torch.tensor(sw, dtype=torch.float32), torch.tensor(cw, dtype=torch.float32))   # warm-up: not timed
    t0, n = time.perf_counter(), 0
    while n < 1 or time.perf_counter() - t0 < seconds:
        ref(*args)
        n += 1
    dt = time.perf_counter() - t0
    return {'value': round(n * len(pos) / dt, 2), 'unit': 'atoms/s', 'cores': threads,
            'kind': 'port',
            'sample': f'{n} energy+force+stress evals of a {len(pos)}-atom Si box ({cells}^3 '
                      f'cells, {ei.shape[1]} edges) in {dt:.1f} s, oracle/sevennet_ref.py fp32, '
                      f'torch CPU, after an untimed warm-up call on a 64-atom box',
            'reference_context': 'the reference frozen TorchScript CPU path measured in the '
                                 'survey container: 272 atoms/s at 10,648 atoms, 8 threads '
                                 '(SURVEY.md 8d); not re-run here (a shipped program), not '
                                 'part of vs_baseline'}


def parity_check_serial(model, cells, device, si=69):
    """Full-size property check outside the timed region: a displaced 8-atom
    cell tiled cells^3 times (same size as the bench box) has E = cells^3
    E_cell and per-image forces equal to the cell's (tests/test_gpu_fullsize.py)."""
    from sevennet_finetuning_amd.neighbor import DeviceNeighborList, neighbor_list
    from sevennet_finetuning_amd.structures import si_diamond, tile
    pos1, cell1 = si_diamond((1, 1, 1), sigma=0.05)
    ei, sh = neighbor_list(pos1, cell1, 5.0)
    vec1 = pos1[ei[1]] + sh @ cell1 - pos1[ei[0]]
    t = lambda a, dt=torch.int32: torch.as_tensor(a, dtype=dt, device=device)
    one = model.energy_forces(t(np.full(8, si)), t(ei[0]), t(ei[1]), t(vec1, torch.float32))
    e1, f1 = float(one['energy']), one['forces'].cpu().numpy()
    posk, cellk = tile(pos1, cell1, (cells,) * 3)
    c, nb, _, vec = DeviceNeighborList(device)(posk, cellk, 5.0)
    big = model.energy_forces(t(np.full(len(posk), si)), c, nb, vec)
    k3 = cells ** 3
    de = abs(float(big['energy']) - k3 * e1) / abs(k3 * e1)
    df = float(np.abs(big['forces'].cpu().numpy().reshape(k3, 8, 3) - f1[None]).max())
    return {'property': f'tiled displaced 8-atom cell, {len(posk)} atoms: E = k^3 E_cell, '
                        'per-image forces equal', 'energy_rel_err': de, 'max_force_err': df,
            'ok': bool(de <= 2e-6 and df <= 1e-4)}


def parity_check_parallel(model, cells_total, grid, rank, device, si=69):
    """Same property through the decomposed path (halo exchanges over the
    process group): tiled 8-atom cell over the whole box."""
    from sevennet_finetuning_amd.neighbor import neighbor_list
    from sevennet_finetuning_amd.parallel import HipSegmentEngine, ParallelE3GNN, build_rank_graph
    from sevennet_finetuning_amd.structures import si_diamond, tile
    pos1, cell1 = si_diamond((1, 1, 1), sigma=0.05)
    ei, sh = neighbor_list(pos1, cell1, 5.0)
    vec1 = pos1[ei[1]] + sh @ cell1 - pos1[ei[0]]
    t = lambda a, dt=torch.int32: torch.as_tensor(a, dtype=dt, device=device)
    one = model.energy_forces(t(np.full(8, si)), t(ei[0]), t(ei[1]), t(vec1, torch.float32))
    e1, f1 = float(one['energy']), one['forces'].cpu().numpy()
    posk, cellk = tile(pos1, cell1, cells_total)
    rg = build_rank_graph(posk, cellk, np.full(len(posk), si), 5.0, grid, rank)
    drv = ParallelE3GNN(HipSegmentEngine(model))
    drv.set_graph(rg)
    out = drv.evaluate()
    k3 = int(np.prod(cells_total))
    de = abs(float(out['energy']) - k3 * e1) / abs(k3 * e1)
    f = out['forces'].cpu().numpy()
    df = float(np.abs(f - f1[np.asarray(out['owned']) % 8]).max()) if len(f) else 0.0
    t = torch.tensor([df], dtype=torch.float64, device=device)
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    df = float(t)
    return {'property': f'tiled displaced 8-atom cell, {len(posk)} atoms over the ranks: '
                        'E = k^3 E_cell, per-image forces equal', 'energy_rel_err': de,
            'max_force_err': df, 'ok': bool(de <= 2e-6 and df <= 1e-4)}


def distributed_report(drv, rg, world, step_ms, device):
    """Backend, the world the process group saw, per-rank owned / ghost / edge
    counts, and the halo exchange against the compute: one extra evaluation
    with every exchange run serially (ParallelE3GNN.evaluate(timing=...)), so
    exchange_ms is what the exchanges cost on their own, compute_ms the rest
    of that evaluation, and overlap = (compute + exchange - overlapped step) /
    exchange: the share of the exchange time the overlapped step hides."""
    import torch.distributed as dist
    tm = {}
    drv.evaluate(timing=tm)
    x_ms, tot_ms = tm.get('exchange_s', 0.0) * 1e3, tm['total_s'] * 1e3
    backend = dist.get_backend()
    comm_dev = device if backend == 'nccl' else torch.device('cpu')
    mine = torch.tensor([rg.n_local, rg.n_ghost, len(rg.center), rg.n_interior, x_ms,
                         tot_ms - x_ms], dtype=torch.float64, device=comm_dev)
    rows = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(rows, mine)
    ranks = []
    for r, v in enumerate(rows):
        owned, ghost, edges, interior, xr, cr = v.tolist()
        ranks.append({'rank': r, 'owned': int(owned), 'ghosts': int(ghost), 'edges': int(edges),
                      'interior': int(interior), 'exchange_ms': round(xr, 3),
                      'compute_ms': round(cr, 3),
                      'overlap': round(min(1.0, max(0.0, (cr + xr - step_ms) / xr)), 3)
                      if xr > 0 else None})
    info = {'backend': backend, 'world_size': dist.get_world_size(),
            'exchanges_per_step': tm.get('exchanges', 0),
            'exchange_ms_max': max(r['exchange_ms'] for r in ranks),
            'compute_ms_max': max(r['compute_ms'] for r in ranks),
            'overlap_min': min((r['overlap'] for r in ranks if r['overlap'] is not None),
                               default=None),
            'ranks': ranks}
    if backend == 'nccl':
        try:
            info['rccl_version'] = '.'.join(str(v) for v in torch.cuda.nccl.version())
        except Exception:  # version query unavailable: not part of the measurement
            pass
    return info


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def launcher_cmd(argv, n, port, script=None):
    """The torch.distributed.run command that starts `n` local ranks of
    `script` (default: this file) with the same arguments (one process per GPU)."""
    return [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
            f'--nproc-per-node={n}', '--master-addr=127.0.0.1', f'--master-port={port}',
            os.path.abspath(script or __file__), *argv]


def maybe_launch(args, argv, script=None):
    """`python bench.py --gpus N` with no launcher around it: start the N ranks
    as child processes (before anything touches the GPU in this process) and
    return their exit code; None when this process is a rank itself.
    bench_train.py shares it (`script`)."""
    if args.gpus <= 1 or 'WORLD_SIZE' in os.environ:
        return None
    import subprocess
    cmd = launcher_cmd(argv, args.gpus, free_port(), script)
    log(f'launching {args.gpus} ranks: {" ".join(cmd)}')
    return subprocess.call(cmd)


def check_world(args, world, script='bench.py'):
    """A rank must see exactly the --gpus N world it was asked for."""
    if world != args.gpus:
        raise RuntimeError(f'{script} --gpus {args.gpus} but WORLD_SIZE={world}: '
                           'run it directly or under torch.distributed.run with '
                           f'--nproc-per-node {args.gpus}')


def box_plan(args, world):
    """(cells, brick grid, total cells per axis) of the evaluated box: one
    cells^3 box at N = 1 and with --strong, N bricks of cells^3 (weak scaling)
    otherwise.  8 atoms per conventional Si cell."""
    from sevennet_finetuning_amd.parallel import brick_grid
    cells = args.cells or (46 if args.strong else 23)
    grid = tuple(brick_grid(world)) if world > 1 else (1, 1, 1)
    total = (cells,) * 3 if (args.strong or world == 1) else tuple(cells * g for g in grid)
    return cells, grid, total


def describe(n_total, world, cells, strong, grid=(1, 1, 1), model='SevenNet-0'):
    """(metric, workload) of a bench line, naming the box actually evaluated:
    BASELINE.json's metric is quoted on the 100k-atom box per GPU; a weak
    multi-rank run evaluates world x that box, a strong run one box split over
    the ranks (46^3 cells = 778,688 atoms: config 4, the 800k box)."""
    base = f'atoms/sec energy+force, {model} lmax=2'
    g = 'x'.join(str(v) for v in grid)
    if world == 1:
        metric = f'{base}, {n_total:,}-atom box @1 GPU'
        work = f'{model} energy+force+virial, {n_total:,}-atom periodic Si box ({cells}^3 cells), 1 GPU'
    elif strong:
        metric = f'{base}, {n_total:,}-atom box split over {world} GPUs (strong scaling)'
        work = (f'{model} energy+force+virial, one {n_total:,}-atom periodic Si box ({cells}^3 cells) '
                f'domain-decomposed {g} over {world} GPUs, halo exchange per layer')
    else:
        per = n_total // world
        metric = f'{base}, {per:,}-atom box per GPU = {n_total:,}-atom box @{world} GPUs (weak scaling)'
        work = (f'{model} energy+force+virial, {n_total:,}-atom periodic Si box ({world} bricks of '
                f'{cells}^3 cells, {g}) over {world} GPUs, halo exchange per layer')
    return metric, work


def model_config_deployment(spec):
    """'c64l4' -> (deployment dir, label): the SevenNet-0 preset with channel 64
    and 4 blocks (model_build.sevennet_shaped_config), written by
    model_build.deploy_config to a temporary directory."""
    import re
    import tempfile
    from sevennet_finetuning_amd import model_build as mb
    m = re.fullmatch(r'c(\d+)l(\d+)', spec)
    if not m:
        raise SystemExit(f'--model-config {spec!r}: expected cCHlL, e.g. c64l4')
    ch, nl = int(m.group(1)), int(m.group(2))
    d = mb.deploy_config(mb.sevennet_shaped_config(ch, nl, species=['Si']), tempfile.mkdtemp(), seed=0)
    return d, f'SevenNet-0 preset with channel {ch}, {nl} blocks'


def rank_emulation(args, model, device, si):
    """One-GPU rehearsal of a decomposed --strong step (north_star config 4):
    the per-rank compute a W-GPU run would do, measured rank by rank, next to
    the whole box on this GPU.  Compute-bound ceiling of the strong-scaling
    speedup = (whole box ms) / (slowest emulated rank ms); the real W-GPU step
    adds whatever part of the exchanges the interior work does not hide (the
    bytes per exchange are reported; no link rate is assumed here)."""
    from sevennet_finetuning_amd.parallel import (HipSegmentEngine, ParallelE3GNN, brick_grid,
                                                  build_rank_graph, local_handshake)
    from sevennet_finetuning_amd.structures import si_diamond
    world = args.emulate_world
    cells = args.cells or 46
    grid = tuple(brick_grid(world))
    pos, cell = si_diamond((cells,) * 3, sigma=0.05)
    n = len(pos)
    t0 = time.perf_counter()
    rgs = [build_rank_graph(pos, cell, np.full(n, si), 5.0, grid, r) for r in range(world)]
    local_handshake(rgs)
    log(f'rank graphs: {world} ranks {grid} of {n} atoms in {time.perf_counter() - t0:.1f} s')
    counts = [{'rank': rg.rank, 'owned': rg.n_local, 'ghosts': rg.n_ghost, 'interior': rg.n_interior,
               'edges': int(len(rg.center)), 'send_rows': int(rg.send_counts.sum()),
               'recv_rows': int(rg.recv_counts.sum())} for rg in rgs]

    def timed(fn, steps, warmup):
        for _ in range(warmup):
            fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / steps * 1e3

    # the whole box on this GPU (the 1-GPU point of the strong-scaling curve)
    box = make_box(cells, device, si)
    whole_ms = timed(lambda: model.energy_forces(box['types'], box['center'], box['nbr'], box['vec']),
                     max(1, min(args.steps, 3)), 1)
    del box
    log(f'whole box: {whole_ms:.2f} ms/step')
    ranks = [int(r) for r in args.rank_emulation.split(',')]
    per = []
    for r in ranks:
        rg = rgs[r]
        drv = ParallelE3GNN(HipSegmentEngine(model))
        drv.set_graph(rg, emulate=True)
        ms = timed(drv.evaluate, args.steps, args.warmup)
        tm = {}
        drv.evaluate(timing=tm)   # every exchange (pack + local copy + unpack) serialised
        sent, recv = drv.halo.bytes_per_step(model.num_layers)
        per.append({**counts[r], 'ms': round(ms, 3),
                    'exchange_kernels_ms': round(tm.get('exchange_s', 0.0) * 1e3, 3),
                    'exchanges_per_step': tm.get('exchanges', 0),
                    'halo_bytes_sent_per_step': sent, 'halo_bytes_received_per_step': recv,
                    'largest_exchange_bytes': max(sum(drv.halo.sc), sum(drv.halo.rc)) *
                    max(model.lib.e3gnn_feature_dim(model._ctx, t) for t in range(1, model.num_layers)) * 4})
        log(f'rank {r}: {per[-1]}')
    worst = max(p['ms'] for p in per)
    return {
        'metric': f'one-GPU rank emulation of the {n:,}-atom box split {"x".join(map(str, grid))} '
                  f'over {world} GPUs: per-rank ms and the compute-bound strong-scaling ceiling',
        'value': round(whole_ms / worst, 3), 'unit': 'x (whole-box ms / slowest emulated rank ms)',
        'n_gpus': 1, 'steps': args.steps, 'warmup': args.warmup, 'higher_is_better': True,
        'dtype': DTYPE, 'data': 'synthetic Si diamond box, default_rng(0) 0.05 A displacements',
        'config': {'workload': f'SevenNet-0 energy+force+virial, {n:,}-atom periodic Si box '
                               f'({cells}^3 cells), rank graphs of a {world}-rank brick decomposition',
                   'total_atoms': n, 'grid': list(grid)},
        'whole_box_ms': round(whole_ms, 3), 'emulated_ranks': per,
        'all_ranks': counts,
        'note': 'each all_to_all is a same-size device copy (no peer data, no link): ms = one rank\'s '
                'compute + halo pack/unpack kernels; a W-GPU step adds the exchange time the interior '
                'work does not hide'}


def main():
    args = parse()
    rc = maybe_launch(args, sys.argv[1:])
    if rc is not None:
        sys.exit(rc)
    world = int(os.environ.get('WORLD_SIZE', '1'))
    check_world(args, world)
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if args.same_device:  # rehearsal of the N > 1 path on a one-GPU box (gloo)
        local = 0
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if args.same_device:
            dist.init_process_group('gloo')
        else:
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    device = torch.device('cuda', local if world > 1 else 0)
    torch.cuda.set_device(device)

    from sevennet_finetuning_amd.model import E3GNNModel
    model_dir, label = None, 'SevenNet-0'
    if args.model_config:
        model_dir, label = model_config_deployment(args.model_config)
    model = E3GNNModel(device=device) if model_dir is None else E3GNNModel(model_dir, device=device)
    si = model.chemical_symbols.index('Si')
    cells, grid, total = box_plan(args, world)
    scaling = 'strong' if args.strong else 'weak'
    parity = None
    if args.rank_emulation is not None:
        if world != 1:
            raise SystemExit('--rank-emulation runs on one GPU (N = 1)')
        print(json.dumps(rank_emulation(args, model, device, si)), flush=True)
        return
    degrees = None
    if args.system == 'hfo2' and world != 1:
        raise SystemExit('--system hfo2 runs on one GPU (N = 1)')
    if world == 1:
        if args.system == 'hfo2':
            cells = args.cells or 10
            box = make_box_hfo2(cells, device, model.chemical_symbols)
            degrees = degree_stats(box['center_np'], box['n'])
            label = f'{label} on HfO2'
        else:
            box = make_box(cells, device, si)
        n, E = box['n'], box['E']
        n_rank, parallelism = n, 'single'
        log(f'box: {n} atoms, {E} edges; workspace after first step follows')
        if degrees:
            log(f'degrees: {degrees}')
        if not args.no_parity_check:
            parity = parity_check_tiled(model, box, device) if args.system == 'hfo2' else \
                parity_check_serial(model, cells, device, si)
            log(f'parity check: {parity}')

        def step():
            return model.energy_forces(box['types'], box['center'], box['nbr'], box['vec'])
    else:
        # spatial decomposition (parallel.py): weak -- an (cells * grid) box, one
        # brick of cells^3 per rank; strong -- one cells^3 box split over the
        # ranks; halo exchange per layer over RCCL
        from sevennet_finetuning_amd.parallel import (HipSegmentEngine, ParallelE3GNN,
                                                      build_rank_graph)
        from sevennet_finetuning_amd.structures import si_diamond
        pos, cell = si_diamond(total, sigma=0.05)
        n = len(pos)
        rg = build_rank_graph(pos, cell, np.full(n, si), 5.0, grid, rank)
        if not args.no_parity_check:
            parity = parity_check_parallel(model, total, grid, rank, device, si)
            log(f'parity check: {parity}')
        drv = ParallelE3GNN(HipSegmentEngine(model))
        drv.set_graph(rg)
        E, n_rank = len(rg.center), rg.n_local
        parallelism = f'spatial {grid[0]}x{grid[1]}x{grid[2]}, {rg.n_ghost} ghosts on rank 0'
        log(f'box: {n} atoms over {world} ranks ({grid}); rank 0: {rg.n_local} owned, '
            f'{rg.n_ghost} ghosts, {E} edges')

        def step():
            return drv.evaluate()

    if parity is not None and not parity['ok']:
        raise RuntimeError(f'full-size parity check failed: {parity}')

    def barrier():
        if world > 1:
            torch.distributed.barrier()

    for i in range(args.warmup):
        step()
        log(f'warmup {i} done, workspace {model.workspace_bytes() / 1e9:.1f} GB')
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=device)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t)
    ms = dt / args.steps * 1e3
    value = n * args.steps / dt  # whole system (world == 1: the one box)
    log(f'timed: {ms:.3f} ms/step')
    energy = float(out['energy'])

    roofline, kernels = None, None
    if not args.profile_only:
        model.set_timing(True)
        model.reset_stats()
        step()
        stats = model.kernel_stats()
        model.set_timing(False)
        log('stats pass done')
        total = sum(s['ms'] for s in stats.values())
        kernels = {k: {'ms': round(v['ms'], 3), 'launches': v['launches'],
                       'tflops': round(v['flops'] / (v['ms'] * 1e9), 2) if v['ms'] else 0.0,
                       'gbs': round(v['bytes'] / (v['ms'] * 1e6), 1) if v['ms'] else 0.0}
                   for k, v in stats.items() if v['launches']}
        dom = max(stats, key=lambda k: stats[k]['ms'])
        d = stats[dom]
        rp_name = rocprof_name(dom, max(getattr(model, 'family', 0), 0))
        if d['flops'] > 0:
            ach = d['flops'] / (d['ms'] * 1e9)
            roofline = {'bound': 'mfma', 'kernel': dom, 'achieved': round(ach, 3),
                        'peak': PEAK_FP32_TFLOPS, 'unit': 'TFLOP/s',
                        'frac': round(ach / PEAK_FP32_TFLOPS, 4), 'traffic': None,
                        'ms_per_launch': round(d['ms'] / d['launches'], 4),
                        'share_of_step': round(d['ms'] / total, 3)}
        else:
            ach = d['bytes'] / (d['ms'] * 1e6)
            roofline = {'bound': 'hbm', 'kernel': dom, 'achieved': round(ach, 1),
                        'peak': PEAK_HBM_GBS, 'unit': 'GB/s', 'frac': round(ach / PEAK_HBM_GBS, 4),
                        'traffic': None, 'ms_per_launch': round(d['ms'] / d['launches'], 4),
                        'share_of_step': round(d['ms'] / total, 3)}
        tot_flops = sum(v['flops'] for v in stats.values())
        roofline['step_tflops'] = round(tot_flops / (ms * 1e9), 3)
        roofline['rocprof_kernel'] = rp_name
        roofline['traffic'] = pmc_traffic(rp_name, cells)
        roofline['mfma_by_precision'] = mfma_fracs(rp_name, cells, roofline['ms_per_launch'])

    distributed = None
    if world > 1:
        distributed = distributed_report(drv, rg, world, ms, device)
        log(f'distributed: {distributed}')

    nl = None
    if world == 1 and not args.profile_only:
        nl = device_nl_timing(box, device)
        log(f'neighbour list: device {nl["device_ms"]} ms, host {nl["host_ms"]} ms')
    cpu = None
    if rank == 0 and not args.no_cpu_baseline and world == 1 and not args.profile_only:
        cpu = cpu_baseline(args.cpu_seconds, args.cpu_cells, model_dir)
    fine_tune = None
    if world == 1 and not args.profile_only and not args.no_fine_tune and model_dir is None:
        # BASELINE config 5 measured in the same run (bench_train.py's step,
        # same recipe and timing contract): the driver records it with the line
        import bench_train
        r = bench_train.step_bench(device, 10, 3)
        fine_tune = {'workload': 'rehearsal step (RehearsalTrainer.run_one_epoch_rehearsal, FT_w_reEWC '
                                 'recipe): 2 x 8 synthetic 54-atom structures, forward + forces/stress + '
                                 'loss gradient + EWC + Adam, twice; HIP graph per batch shape',
                     'ms_per_step': round(r['ms_per_step'], 3),
                     'structures_per_s': round(r['structures_per_s'], 2),
                     'atoms_per_s': round(r['atoms_per_s'], 1), 'steps': 10, 'warmup': 3,
                     'gemm': r['gemm'], 'loss': r['loss']}
        log(f'fine-tune step: {fine_tune}')

    if rank == 0:
        metric, workload = describe(n, world, cells, args.strong, grid, label)
        if args.system == 'hfo2':
            metric = f'atoms/sec energy+force, {label} lmax=2, {n:,}-atom box @1 GPU'
            workload = (f'SevenNet-0 energy+force+virial, {n:,}-atom periodic HfO2 box (the reference '
                        f"example's res.dat, 96 atoms, tiled {cells}^3), 1 GPU")
        line = {
            'metric': metric,
            'value': round(value, 2), 'unit': 'atoms/s', 'n_gpus': world,
            'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(ms, 3),
            'higher_is_better': True, 'scaling': scaling, 'vs_baseline': None, 'dtype': DTYPE,
            'data': ('synthetic Si diamond box, default_rng(0) 0.05 A displacements; '
                     if args.system == 'si' else "reference example HfO2 snapshot (res.dat) tiled; ")
                    + ('SevenNet-0 weights (reference opt_params_sevenn.pt)' if model_dir is None else
                       f'{label}: e3nn initialisation (model_build, seed 0), fused-kernel family '
                       f'{model.family}'),
            'config': {'workload': workload, 'total_atoms': n, 'scaling': scaling,
                       'atoms_per_rank': n_rank, 'edges_per_rank': E,
                       'parallelism': parallelism},
            'energy': energy,
            'parity_check': parity,
            'roofline': roofline,
            'cpu_baseline': cpu,
            'neighbor_list': nl,
            'fine_tune': fine_tune,
            'degrees': degrees,
            'distributed': distributed,
            'kernels': kernels,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == '__main__':
    main()
