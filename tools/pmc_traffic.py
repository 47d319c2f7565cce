"""HBM traffic per kernel launch from the rocprofv3 PMC passes of bench.py.

Inputs: gpurun_out/pmc_fetch/run_counter_collection.csv (--pmc FETCH_SIZE) and
gpurun_out/pmc_write/run_counter_collection.csv (--pmc WRITE_SIZE), collected
in SEPARATE passes (tools/gpu_job.sh pmcf / pmcw), and, when present,
gpurun_out/pmc_mops/run_counter_collection.csv (tools/gpu_job.sh pmcmops:
SQ_INSTS_VALU_MFMA_MOPS_BF16 / _F32, the matrix-core work actually executed,
in units of 512 FLOP) for the roofline's per-precision MFMA fractions.  FETCH_SIZE and WRITE_SIZE
are in KiB; on gfx950 FETCH_SIZE counts half of the bytes of wide streaming
reads (MI355X_MICROARCH.md, HBM section), so bytes = 2 x FETCH + WRITE.  Both
count Infinity-Cache traffic too (memory-side L2 requests), so this is an
upper bound on HBM bytes.  Writes profiles/pmc_traffic.json, which bench.py
reads for roofline.traffic.

usage: python tools/pmc_traffic.py [--cells 23] [--out profiles/pmc_traffic.json]
"""
import argparse
import collections
import csv
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r['Counter_Name'] == counter:
            acc[r['Kernel_Name']].append(float(r['Counter_Value']))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--cells', type=int, default=23)
    ap.add_argument('--fetch', default=os.path.join(ROOT, 'gpurun_out/pmc_fetch/run_counter_collection.csv'))
    ap.add_argument('--write', default=os.path.join(ROOT, 'gpurun_out/pmc_write/run_counter_collection.csv'))
    ap.add_argument('--mops', default=os.path.join(ROOT, 'gpurun_out/pmc_mops/run_counter_collection.csv'))
    ap.add_argument('--out', default=os.path.join(ROOT, 'profiles/pmc_traffic.json'))
    a = ap.parse_args()
    fetch = per_kernel(a.fetch, 'FETCH_SIZE')
    write = per_kernel(a.write, 'WRITE_SIZE')
    mops = {}
    if os.path.exists(a.mops):
        mops = {c: per_kernel(a.mops, c) for c in ('SQ_INSTS_VALU_MFMA_MOPS_BF16',
                                                   'SQ_INSTS_VALU_MFMA_MOPS_F32')}
    out = {}
    for k in sorted(set(fetch) | set(write)):
        if not k.startswith(('void e3gnn', 'e3gnn')):
            continue
        f, w = fetch.get(k, 0.0), write.get(k, 0.0)
        out[k] = {'fetch_kib': round(f, 1), 'write_kib': round(w, 1),
                  'bytes_per_launch': round((2 * f + w) * 1024)}
        if mops:
            # matrix-core work executed per launch: MOPS x 512 FLOP
            out[k]['mfma_flop_bf16'] = round(mops['SQ_INSTS_VALU_MFMA_MOPS_BF16'].get(k, 0.0) * 512)
            out[k]['mfma_flop_f32'] = round(mops['SQ_INSTS_VALU_MFMA_MOPS_F32'].get(k, 0.0) * 512)
    json.dump({'cells': a.cells, 'note': 'bytes = 2*FETCH_SIZE + WRITE_SIZE (KiB -> B), '
               'averaged over launches; includes Infinity-Cache traffic; mfma_flop_* = '
               'SQ_INSTS_VALU_MFMA_MOPS_* x 512 (matrix-core FLOP executed per launch)',
               'kernels': out},
              open(a.out, 'w'), indent=1)
    for k, v in out.items():
        print(f"{v['bytes_per_launch'] / 1e9:9.3f} GB  {k[:100]}")


if __name__ == '__main__':
    main()
