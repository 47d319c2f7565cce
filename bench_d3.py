"""Benchmark of the DFT-D3 kernels (the reference's
pair_style d3, sevenn/pair_e3gnn/pair_d3.cu).

``python bench_d3.py [--cells 10] [--steps K] [--warmup W]``: one step = one
PairD3 compute (CN, C6(CN) + BJ damping, C6 chain, reductions; energy, forces,
virial) of an n^3-cell Si diamond box (default 10^3 cells = 8,000 atoms),
PBE-D3(BJ), the reference's default cutoffs (rthr 9000 bohr^2, cn_thr 1600
bohr^2).  Reports atoms/s, the pair-image evaluations per second of each
kernel class (HIP-event timed on the stream the kernels run on) and, for the
dominant kernel, achieved FP32 throughput against the VALU peak, plus the
oracle (numpy fp64 restatement) on a bounded sample as the CPU baseline.
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
PEAK_FP32_TFLOPS = 157.3
# algorithmic FP32 operations per evaluated pair-image (counted from d3.hip:
# BJ dispersion term incl. its force/virial/dE/dCN parts; CN term; chain term)
FLOP_DISP, FLOP_CN, FLOP_CHAIN = 60, 20, 40


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--cells', type=int, default=10)
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--cpu-seconds', type=float, default=10.0)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    args = ap.parse_args()
    from sevennet_finetuning_amd.d3 import PairD3
    from sevennet_finetuning_amd.structures import si_diamond
    pos, cell = si_diamond((args.cells,) * 3, sigma=0.05)
    n = len(pos)
    types = np.zeros(n, np.int32)
    pair = PairD3(9000.0, 1600.0, 'damp_bj', 'pbe').coeff(['Si'])
    torch.cuda.init()
    for _ in range(args.warmup):
        out = pair.compute(pos, cell, types)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = pair.compute(pos, cell, types)
    dt = (time.perf_counter() - t0) / args.steps
    # image counts as the library forms them
    lat = cell / 0.52917726
    def n_images(thr, lat=lat):
        rep = []
        for k in range(3):
            c = np.cross(lat[(k + 1) % 3], lat[(k + 2) % 3])
            rep.append(int(abs(np.sqrt(thr) / (abs(c @ lat[k]) / np.linalg.norm(c)))) + 1)
        return int(np.prod([2 * r + 1 for r in rep]))
    items_v = n * n * n_images(9000.0)
    items_c = n * n * n_images(1600.0)
    # algorithmic work: the within-cutoff pair-images of a homogeneous box
    # (n x density x sphere volume); items the kernels cull are overhead
    dens = n / abs(np.linalg.det(lat))
    in_v = n * dens * 4.0 / 3.0 * np.pi * 9000.0 ** 1.5
    in_c = n * dens * 4.0 / 3.0 * np.pi * 1600.0 ** 1.5
    flops = in_v * FLOP_DISP + in_c * (FLOP_CN + FLOP_CHAIN)
    tflops = flops / dt / 1e12
    cpu = None
    if not args.no_cpu_baseline:
        from oracle import d3_ref as D
        tables, funcs = D.load_tables()
        tt = D.type_tables([14], tables)
        fp = D.functional(funcs, 'damp_bj', 'pbe')
        sp, sc = si_diamond((1, 1, 1), sigma=0.05)
        t1, k = time.perf_counter(), 0
        while time.perf_counter() - t1 < args.cpu_seconds:
            D.d3(sp, sc, np.zeros(len(sp), int), tt, fp)
            k += 1
        cdt = (time.perf_counter() - t1) / k
        cpu = {'value': round(len(sp) / cdt, 2), 'unit': 'atoms/s', 'cores': 1, 'kind': 'port',
               'sample': f'{k} evaluations of the 8-atom Si cell (default cutoffs, '
                         f'{len(sp) ** 2 * n_images(9000.0, sc / 0.52917726) // 2} pair-images), '
                         'oracle/d3_ref.py numpy fp64'}
    print(json.dumps({
        'metric': 'atoms/sec DFT-D3(BJ) energy+force+virial', 'value': round(n / dt, 1),
        'unit': 'atoms/s', 'ms_per_step': round(dt * 1e3, 3), 'n_gpus': 1,
        'steps': args.steps, 'warmup': args.warmup, 'dtype': 'f32 (C6 interpolation f64)',
        'config': {'workload': f'PBE-D3(BJ), {n}-atom Si box ({args.cells}^3 cells), '
                               'rthr 9000 / cn_thr 1600 bohr^2',
                   'all_images_vdw': items_v, 'all_images_cn': items_c,
                   'within_cutoff_vdw': int(in_v), 'within_cutoff_cn': int(in_c)},
        'energy_eV': out['energy'],
        'roofline': {'bound': 'valu', 'achieved': round(tflops, 2), 'peak': PEAK_FP32_TFLOPS,
                     'unit': 'TFLOP/s', 'frac': round(tflops / PEAK_FP32_TFLOPS, 4),
                     'flop_model': f'{FLOP_DISP}/{FLOP_CN}/{FLOP_CHAIN} FP32 FLOP per within-cutoff '
                                   'disp/CN/chain pair-image (C6 interpolation, n(n+1)/2 '
                                   'fp64 pair evaluations, not counted); host-timed step'},
        'cpu_baseline': cpu}), flush=True)


if __name__ == '__main__':
    main()
