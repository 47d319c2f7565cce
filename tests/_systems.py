"""Deterministic test systems (SURVEY.md 8d recipes) and oracle helpers."""
import json
import os

import numpy as np
import torch

from sevennet_finetuning_amd.structures import si_diamond, MIXED_SYMBOLS

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def symbols_index(symbols_all, syms):
    return np.array([symbols_all.index(s) for s in syms], dtype=np.int64)


def load_manifest_symbols():
    root = os.path.dirname(GOLD)
    man = os.path.join(root, '..', 'sevennet_finetuning_amd', 'assets', 'sevennet0', 'manifest.json')
    return json.load(open(man))['chemical_symbols']


def kat_list():
    return json.load(open(os.path.join(GOLD, 'kat_reference.json')))['kats']


def system(name, symbols_all):
    """Returns (pos float64 [N,3], cell [3,3], types int64 [N])."""
    if name.startswith('si_'):
        parts = name.split('_')
        cells = tuple(int(c) for c in parts[-1].split('x'))
        sigma = 0.0 if parts[1] == 'perfect' else 0.05
        pos, cell = si_diamond(cells, sigma=sigma)
        types = np.full(len(pos), symbols_all.index('Si'), dtype=np.int64)
        return pos, cell, types
    if name == 'hfo2_resdat':
        d = np.load(os.path.join(GOLD, 'hfo2_resdat.npz'))
        return d['pos'], d['cell'], symbols_index(symbols_all, [str(s) for s in d['symbols']])
    if name.startswith('mixed_'):
        cells = tuple(int(c) for c in name.split('_')[1].split('x'))
        pos, cell = si_diamond(cells, sigma=0.08, seed=3)
        rng = np.random.default_rng(1)
        syms = [MIXED_SYMBOLS[i] for i in rng.integers(0, 4, len(pos))]
        return pos, cell, symbols_index(symbols_all, syms)
    raise KeyError(name)


def oracle_eval(pos, cell, types, dtype=torch.float64, trace=None):
    from oracle.neighbor import neighbor_list
    from oracle.sevennet_ref import SevenNet0Ref
    ref = SevenNet0Ref(dtype=dtype)
    ei, sh = neighbor_list(pos, cell, ref.cutoff)
    posd = torch.tensor(pos, dtype=dtype).requires_grad_(True)
    out = ref.energy(posd, torch.tensor(types), torch.tensor(ei), torch.tensor(sh, dtype=dtype),
                     torch.tensor(cell, dtype=dtype), True, trace=trace)
    g = torch.autograd.grad(out['energy'], [posd, out['strain']])
    vol = abs(np.linalg.det(cell))
    s = -g[1] / vol
    return {'energy': float(out['energy']), 'atomic_energy': out['atomic_energy'].detach().numpy(),
            'forces': (-g[0]).numpy(),
            'stress': np.array([s[0, 0], s[1, 1], s[2, 2], s[0, 1], s[1, 2], s[0, 2]]),
            'edge_index': ei, 'shift': sh}
