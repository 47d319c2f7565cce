"""Print the HIP path's errors against the fp64 oracle on the parity systems
(numbers quoted in DESIGN.md §2).  GPU box:  python tools/parity_report.py"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'tests')]

from _systems import load_manifest_symbols, oracle_eval, system  # noqa: E402
from test_gpu_parity import run  # noqa: E402


def main():
    from sevennet_finetuning_amd.model import E3GNNModel
    model = E3GNNModel(device='cuda:0')
    syms = load_manifest_symbols()
    rows = []
    for name in ['si_rng0_2x2x1', 'si_rng0_3x3x3', 'hfo2_resdat', 'mixed_2x2x2', 'si_perfect_1x1x1']:
        pos, cell, types = system(name, syms)
        ref = oracle_eval(pos, cell, types)
        got = run(model, pos, cell, types)
        rows.append({'system': name, 'atoms': len(pos),
                     'dE_rel': abs(got['energy'] - ref['energy']) / abs(ref['energy']),
                     'dF_max': float(np.abs(got['forces'] - ref['forces']).max()),
                     'dS_max': float(np.abs(got['stress'] - ref['stress']).max())})
        print(json.dumps(rows[-1]), flush=True)


if __name__ == '__main__':
    main()
