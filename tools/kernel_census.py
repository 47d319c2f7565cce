"""Per-step kernel census of a rocprofv3 --kernel-trace CSV.

usage: python tools/kernel_census.py <run_kernel_trace.csv> [marker] [steps]

A step is the span between two occurrences of ``marker`` (a kernel-name
substring; default ``k_edge_embed``, one per evaluated batch) taken ``steps``
apart (default 2: the fine-tune rehearsal step evaluates two batches).  Prints
the kernel count, the summed kernel time, the wall span and the kernels grouped
by class, largest first.
"""
import collections
import csv
import re
import sys


def short(name):
    m = re.search(r'(k_[a-z0-9_]+)(<[^>]*>)?', name)
    if m:
        return m.group(1) + (m.group(2) or '').replace('e3gnn::', '')
    if 'Cijk' in name:
        t = re.search(r'Cijk_(\w{4}_\w{4})', name)
        mt = re.search(r'MT(\w+?)_', name)
        return f"GEMM {t.group(1) if t else ''} {mt.group(1) if mt else ''}"
    if 'multi_tensor' in name:
        return 'optimizer (multi_tensor_apply)'
    if 'copyBuffer' in name:
        return 'copyBuffer'
    m = re.findall(r'at::native::(?:\(anonymous namespace\)::)?([a-zA-Z_]+)', name)
    f = sorted({x.replace('Functor', '') for x in re.findall(r'(\w*Functor\w*)', name)})
    return f"torch {m[0] if m else name[:24]} {','.join(f)[:40]}"


def main(path, marker='k_edge_embed', steps=2):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r['Start_Timestamp']))
    names = [short(r['Kernel_Name']) for r in rows]
    st = [int(r['Start_Timestamp']) for r in rows]
    en = [int(r['End_Timestamp']) for r in rows]
    idx = [i for i, r in enumerate(rows) if marker in r['Kernel_Name']]
    if len(idx) < steps + 1:
        raise SystemExit(f'fewer than {steps + 1} "{marker}" kernels in {path}')
    a, b = idx[-1 - steps], idx[-1]
    acc = collections.defaultdict(lambda: [0, 0.0])
    for i in range(a, b):
        acc[names[i]][0] += 1
        acc[names[i]][1] += (en[i] - st[i]) / 1e3
    total = sum(v[1] for v in acc.values())
    print(f'kernels per step: {b - a}   kernel time: {total:.0f} us   wall: {(st[b] - st[a]) / 1e3:.0f} us')
    for k, (n, us) in sorted(acc.items(), key=lambda x: -x[1][1]):
        print(f'{n:5d} {us:9.1f} us  {k}')


if __name__ == '__main__':
    a = sys.argv[1:]
    main(a[0], *(a[1:2]), *([int(a[2])] if len(a) > 2 else []))
