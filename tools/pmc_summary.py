"""Per-kernel averages of every counter in rocprofv3 --pmc CSVs.

usage: python tools/pmc_summary.py gpurun_out/pmc_sq [gpurun_out/pmc_tcp ...]
"""
import collections
import csv
import os
import re
import sys


def short(name):
    m = re.search(r'(k_[a-z0-9_]+)(<[^(]*>)?', name)
    if not m:
        return name[:40]
    t = (m.group(2) or '').replace('e3gnn::', '').replace(' ', '')
    return m.group(1) + t


def main(dirs):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        for r in csv.DictReader(open(os.path.join(d, 'run_counter_collection.csv'))):
            acc[short(r['Kernel_Name'])][r['Counter_Name']].append(float(r['Counter_Value']))
    names = sorted({c for k in acc.values() for c in k})
    for k, cs in sorted(acc.items()):
        if not k.startswith('k_conv') and '--all' not in sys.argv:
            continue
        print(k)
        for c in names:
            if c in cs:
                v = cs[c]
                print(f'   {c:40s} {sum(v) / len(v):16.4g}')


if __name__ == '__main__':
    main([a for a in sys.argv[1:] if not a.startswith('--')])
