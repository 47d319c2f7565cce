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
