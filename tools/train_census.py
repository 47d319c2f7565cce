"""Per-step kernel census of the fine-tune bench (bench_train.py under
rocprofv3 --kernel-trace --stats, tools/gpu_job.sh proftrain2): launches and
GPU time per step by kernel, grouped into the library's kernels and torch's.

usage: python tools/train_census.py [stats.csv] [--steps 16]
(16 = 3 warmup + 10 timed + the 3 capture / first-call steps of bench_train)
"""
import argparse
import collections
import csv
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    n = name
    for pre in ('void ', 'e3gnn::(anonymous namespace)::', 'at::native::', '(anonymous namespace)::',
                'e3gnn::'):
        n = n.replace(pre, '')
    return n.split('(')[0][:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('stats', nargs='?', default=os.path.join(ROOT, 'gpurun_out/prof_train2/run_kernel_stats.csv'))
    ap.add_argument('--steps', type=int, default=16)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.stats)))
    groups = collections.defaultdict(lambda: [0, 0.0])
    per = collections.defaultdict(lambda: [0, 0.0])
    for r in rows:
        calls, ns = int(r['Calls']), float(r['TotalDurationNs'])
        name = r['Name']
        g = ('library GEMM (tgemm)' if 'k_tgemm' in name else
             'library (other)' if 'e3gnn::' in name else
             'copies / fills (runtime)' if '__amd_rocclr' in name else
             'rocprim' if 'rocprim' in name else 'torch')
        groups[g][0] += calls
        groups[g][1] += ns
        per[short(name)][0] += calls
        per[short(name)][1] += ns
    S = a.steps
    tot_c = sum(v[0] for v in groups.values()) / S
    tot_t = sum(v[1] for v in groups.values()) / S / 1e6
    print(f'per step: {tot_c:.0f} kernels, {tot_t:.3f} ms of kernel time ({a.stats}, {S} steps)')
    for g, (c, t) in sorted(groups.items(), key=lambda x: -x[1][1]):
        print(f'  {g:28s} {c / S:7.1f} launches {t / S / 1e6:7.3f} ms')
    print('top kernels:')
    for n, (c, t) in sorted(per.items(), key=lambda x: -x[1][1])[:40]:
        print(f'  {c / S:7.1f} x {t / max(c, 1) / 1e3:7.1f} us = {t / S / 1e6:6.3f} ms  {n}')


if __name__ == '__main__':
    main()
