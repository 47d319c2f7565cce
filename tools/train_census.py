"""Per-step kernel census of the fine-tune bench from a rocprofv3 kernel trace
of bench_train.py (tools/gpu_job.sh proftraint): the kernels of one
steady-state rehearsal step (two batches) -- between the k_loss_efs launches
that open the last two reverse sweeps but one -- by count and GPU time,
grouped into the library's kernels and torch's / the runtime's.

usage: python tools/train_census.py [run_kernel_trace.csv]
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
    ap.add_argument('trace', nargs='?', default=os.path.join(ROOT, 'gpurun_out/prof_traint/run_kernel_trace.csv'))
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r['Start_Timestamp']))
    marks = [i for i, r in enumerate(rows) if 'k_loss_efs' in r['Kernel_Name']]
    if len(marks) < 4:
        raise SystemExit('need at least two steady-state steps in the trace')
    seg = rows[marks[-4]:marks[-2]]        # one rehearsal step: two batches' sweeps
    dur = lambda r: (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3   # noqa: E731 (us)
    busy = sum(dur(r) for r in seg)
    span = (int(seg[-1]['End_Timestamp']) - int(seg[0]['Start_Timestamp'])) / 1e3
    groups = collections.defaultdict(lambda: [0, 0.0])
    per = collections.defaultdict(lambda: [0, 0.0])
    for r in seg:
        name = r['Kernel_Name']
        g = ('library GEMM (tgemm)' if 'k_tgemm' in name else
             'library (other)' if 'e3gnn::' in name else
             'copies / fills (runtime)' if '__amd_rocclr' in name else 'torch')
        groups[g][0] += 1
        groups[g][1] += dur(r)
        per[short(name)][0] += 1
        per[short(name)][1] += dur(r)
    print(f'one rehearsal step: {len(seg)} kernels, {busy / 1e3:.3f} ms of kernel time, '
          f'{span / 1e3:.3f} ms span ({a.trace})')
    for g, (c, t) in sorted(groups.items(), key=lambda x: -x[1][1]):
        print(f'  {g:28s} {c:5d} launches {t / 1e3:7.3f} ms')
    print('kernels by time:')
    for n, (c, t) in sorted(per.items(), key=lambda x: -x[1][1])[:45]:
        print(f'  {c:4d} x {t / c:7.1f} us = {t / 1e3:6.3f} ms  {n}')


if __name__ == '__main__':
    main()
