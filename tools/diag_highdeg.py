"""Energy/force error of the dense high-degree cluster (tests/test_gpu_parity.py
test_high_degree_centres) against the fp64 oracle, for the node-linear path
selected by E3GNN_NODELIN; also the energy of a float64-rounded re-run to see
the fp32 noise floor (run-to-run determinism check)."""
import os
import sys
import numpy as np
import torch
_ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path.insert(0, os.path.join(_ROOT, 'tests'))
sys.path.insert(0, _ROOT)
from _systems import load_manifest_symbols, oracle_eval  # noqa: E402
from sevennet_finetuning_amd.model import E3GNNModel  # noqa: E402
from sevennet_finetuning_amd.neighbor import neighbor_list  # noqa: E402

SYMS = load_manifest_symbols()
rng = np.random.default_rng(5)
pos = rng.uniform(0, 6.5, size=(400, 3))
keep = [0]
for i in range(1, len(pos)):
    if np.min(np.linalg.norm(pos[keep] - pos[i], axis=1)) > 1.1:
        keep.append(i)
pos = pos[keep]
cell = np.eye(3) * 30.0
types = np.full(len(pos), SYMS.index('Si'))
model = E3GNNModel(device='cuda:0')
ei, sh = neighbor_list(pos, cell, model.cutoff)
data = {'x': torch.tensor(types), 'pos': torch.tensor(pos, dtype=torch.float32),
        'edge_index': torch.tensor(ei), 'pbc_shift': torch.tensor(sh, dtype=torch.float32),
        'cell_lattice_vectors': torch.tensor(cell, dtype=torch.float32)}
out = model(data)
ref = oracle_eval(pos, cell, types)
e = float(out['inferred_total_energy'])
f = out['inferred_force'].cpu().numpy()
print('NODELIN', os.environ.get('E3GNN_NODELIN', '1'), 'atoms', len(pos), 'E', e, 'ref', ref['energy'],
      'rel', abs(e - ref['energy']) / abs(ref['energy']),
      'max|dF|', float(np.abs(f - ref['forces']).max()), 'max|F|', float(np.abs(ref['forces']).max()))
# the same input as float32-rounded positions in the oracle: separates input
# rounding from arithmetic
ref32 = oracle_eval(pos.astype(np.float32).astype(np.float64), cell, types)
print('oracle(f32-rounded pos) rel', abs(ref32['energy'] - ref['energy']) / abs(ref['energy']))
