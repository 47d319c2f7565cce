"""The oracle (CPU restatement) against the reference's known answers.

The KATs are energies the survey measured by running the reference's own
frozen SevenNet-0 deployment (tests/golden/kat_reference.json);
the CG tables are the deployment's frozen constants (tests/golden/cg_frozen.npz).
"""
import numpy as np
import pytest
import torch

from _systems import kat_list, load_manifest_symbols, system, GOLD

SYMS = load_manifest_symbols()


def _kat_system(k):
    if k['name'].startswith('si_'):
        cells = 'x'.join(str(c) for c in k['cells'])
        return system(('si_rng0_' if k.get('displace') else 'si_perfect_') + cells, SYMS)
    return system(k['name'], SYMS)


@pytest.mark.parametrize('kat', kat_list(), ids=lambda k: k['name'])
def test_oracle_energy_matches_reference_kat(kat):
    from oracle.neighbor import neighbor_list
    from oracle.sevennet_ref import SevenNet0Ref
    pos, cell, types = _kat_system(kat)
    ref = SevenNet0Ref(dtype=torch.float32)
    ei, sh = neighbor_list(pos, cell, ref.cutoff)
    assert ei.shape[1] == kat['n_edges']
    out = ref(torch.tensor(pos, dtype=torch.float32), torch.tensor(types), torch.tensor(ei),
              torch.tensor(sh, dtype=torch.float32), torch.tensor(cell, dtype=torch.float32))
    # fp32 with a different summation order than the frozen graph: 1e-6 relative
    assert abs(float(out['energy']) - kat['energy']) <= 1e-6 * abs(kat['energy']) + 1e-4
    if 'stress_diag' in kat:
        s = out['stress'].numpy()
        assert np.allclose(s[:3], kat['stress_diag'], atol=2e-6)
        assert np.abs(s[3:]).max() < 1e-6
    if 'max_abs_force' in kat:
        assert float(out['forces'].abs().max()) < 1e-4


def test_oracle_cg_matches_frozen_tables():
    from oracle.cg import tp_cg
    d = np.load(f'{GOLD}/cg_frozen.npz')
    for key in d.files:
        l1, l2, l3 = map(int, key[3:])
        assert np.abs(tp_cg(l1, l2, l3) - d[key]).max() < 1e-6, key


def test_oracle_forces_are_energy_gradient():
    """Finite differences of the fp64 oracle energy (no reference needed)."""
    from _systems import oracle_eval
    pos, cell, types = system('mixed_1x1x1', SYMS)
    res = oracle_eval(pos, cell, types)
    h = 1e-5
    for atom, comp in [(0, 0), (3, 1), (5, 2)]:
        p1, p2 = pos.copy(), pos.copy()
        p1[atom, comp] += h
        p2[atom, comp] -= h
        e1 = oracle_eval(p1, cell, types)['energy']
        e2 = oracle_eval(p2, cell, types)['energy']
        assert abs(-(e1 - e2) / (2 * h) - res['forces'][atom, comp]) < 1e-6


# ------------------------------------------------ the nequip-family restatement
def _nequip(model):
    import os
    from oracle.nequip_ref import NequIPRef
    root = os.path.join(os.path.dirname(GOLD), '..', 'sevennet_finetuning_amd', 'assets', model)
    return NequIPRef(root)


def test_nequip_oracle_matches_hfo2_example_kat():
    """The generic restatement on the HfO2 example deployment (sevenn 0.8.6:
    odd parity, nequip self-connection, polynomial cutoff, raw-vector SH)
    against the reference's own frozen-model energy and force on res.dat."""
    import json
    from oracle.neighbor import neighbor_list
    kat = json.load(open(f'{GOLD}/kat_reference.json'))['kats_hfo2_example']
    ref = _nequip(kat['model'])
    d = np.load(f'{GOLD}/hfo2_resdat.npz')
    types = np.array([ref.symbols.index(str(s)) for s in d['symbols']])
    ei, sh = neighbor_list(d['pos'], d['cell'], ref.cutoff)
    assert ei.shape[1] == kat['n_edges']
    out = ref(torch.tensor(d['pos']), torch.tensor(types), torch.tensor(ei),
              torch.tensor(sh), torch.tensor(d['cell']))
    # the reference value is fp32 (ulp at 2.8e3 eV: 2.4e-4): 1e-6 relative
    assert abs(float(out['energy']) - kat['energy']) <= 1e-6 * abs(kat['energy'])
    assert np.abs(out['forces'][0].numpy() - np.array(kat['force0'])).max() < 2e-5
    assert float(out['forces'].sum(0).abs().max()) < 1e-9


def test_nequip_oracle_reproduces_sevennet0_oracle():
    """SevenNet-0 is an instance of the generic restatement: both oracles agree
    to fp64 round-off (and hence both sit on the SevenNet-0 KATs)."""
    from oracle.neighbor import neighbor_list
    from oracle.sevennet_ref import SevenNet0Ref
    pos, cell, types = system('mixed_1x1x1', SYMS)
    ei, sh = neighbor_list(pos, cell, 5.0)
    args = (torch.tensor(pos), torch.tensor(types), torch.tensor(ei), torch.tensor(sh),
            torch.tensor(cell))
    a = _nequip('sevennet0')(*args)
    b = SevenNet0Ref(dtype=torch.float64)(*args)
    assert abs(float(a['energy'] - b['energy'])) < 1e-9 * abs(float(b['energy']))
    assert float((a['forces'] - b['forces']).abs().max()) < 1e-10
    assert float((a['stress'] - b['stress']).abs().max()) < 1e-12


def test_oracle_cg_matches_hfo2_frozen_w3j():
    """The HfO2 deployment froze wigner_3j(1,1,1) itself (a parity-odd path of
    the 1o x 1o product): the oracle's coupling / sqrt(3) equals it."""
    import math
    from oracle.cg import tp_cg
    w = np.load(f'{GOLD}/hfo2_frozen_w3j111.npz')['w3j_111']
    assert np.abs(tp_cg(1, 1, 1) / math.sqrt(3.0) - w).max() < 1e-7
