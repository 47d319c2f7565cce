"""DFT-D3 on the GPU (csrc/d3.hip via e3gnn_d3_*) against the float64 oracle
(oracle/d3_ref.py; parity with the reference's own numbers is unpinned, see
tests/test_d3.py).  Needs an MI355X: ``pytest -m gpu``.

Tolerances (fp32 pair terms as in the reference, fp64 row sums, vs fp64):
energy 1e-5 relative, forces 1e-4 of the largest force component + 1e-6 eV/A,
virial 1e-5 of the largest component.  Bitwise run-to-run determinism.
"""
import numpy as np
import pytest

from _systems import GOLD
from oracle import d3_ref as D
from sevennet_finetuning_amd.structures import si_diamond, mixed_symbols, CHEMICAL_SYMBOLS

pytestmark = pytest.mark.gpu
TABLES, FUNCS = D.load_tables()


def _hip(pos, cell, z, damping, functional, pbc=(True, True, True), **kw):
    from sevennet_finetuning_amd.d3 import PairD3
    elems = sorted(set(int(v) for v in z))
    pair = PairD3(damping=damping, functional_name=functional, **kw).coeff(elems)
    types = np.searchsorted(np.asarray(elems), z)
    return pair.compute(pos, cell, types, pbc), pair, types


def _oracle(pos, cell, z, damping, functional, pbc=(True, True, True), **kw):
    elems = sorted(set(int(v) for v in z))
    tt = D.type_tables(elems, TABLES)
    types = np.searchsorted(np.asarray(elems), z)
    return D.d3(pos, cell, types, tt, D.functional(FUNCS, damping, functional), damping,
                pbc=pbc, **kw)


def _compare(got, ref):
    de = abs(got['energy'] - ref['energy']) / abs(ref['energy'])
    df = np.abs(got['forces'] - ref['forces']).max()
    dv = np.abs(got['virial'] - ref['virial']).max()
    fs = np.abs(ref['forces']).max()
    vs = np.abs(ref['virial']).max()
    print(f'dE/E {de:.2e}  max|dF| {df:.2e} (max|F| {fs:.2e})  max|dW| {dv:.2e} (max {vs:.2e})')
    assert de < 1e-5
    assert df < 1e-4 * fs + 1e-6
    assert dv < 1e-5 * vs


def si8():
    pos, cell = si_diamond((1, 1, 1), sigma=0.05)
    return pos, cell, np.full(len(pos), 14)


@pytest.mark.parametrize('damping,functional', [('damp_bj', 'pbe'), ('damp_zero', 'pbe'),
                                                ('damp_bj', 'b3-lyp'), ('damp_bjm', 'pbe')])
def test_si8_default_cutoffs(damping, functional):
    pos, cell, z = si8()
    got, _, _ = _hip(pos, cell, z, damping, functional)
    _compare(got, _oracle(pos, cell, z, damping, functional))


def test_hfo2_triclinic_bj():
    d = np.load(f'{GOLD}/hfo2_resdat.npz')
    z = np.array([CHEMICAL_SYMBOLS.index(str(s)) for s in d['symbols']])
    kw = dict(rthr=3000.0)
    got, _, _ = _hip(d['pos'], d['cell'], z, 'damp_bj', 'pbe', **kw)
    _compare(got, _oracle(d['pos'], d['cell'], z, 'damp_bj', 'pbe', **kw))


def test_mixed_species_zero_damping():
    pos, cell = si_diamond((2, 2, 2), sigma=0.08, seed=3)
    z = np.array([CHEMICAL_SYMBOLS.index(s) for s in mixed_symbols(len(pos))])
    kw = dict(rthr=2000.0, cn_thr=900.0)
    got, _, _ = _hip(pos, cell, z, 'damp_zero', 'pbe0', **kw)
    _compare(got, _oracle(pos, cell, z, 'damp_zero', 'pbe0', **kw))


def test_isolated_cluster():
    rng = np.random.default_rng(7)
    pos = rng.uniform(0, 6.0, (12, 3))
    z = np.array([6, 1, 8, 1, 6, 7, 1, 1, 6, 8, 1, 16])
    cell = np.eye(3) * 30.0
    got, _, _ = _hip(pos, cell, z, 'damp_bj', 'pbe', pbc=(False, False, False))
    ref = _oracle(pos, cell, z, 'damp_bj', 'pbe', pbc=(False, False, False))
    _compare(got, ref)
    # no images: the LAMMPS virial is sum_i x_i (x) F_i
    w = np.einsum('ia,ib->ab', pos - pos.mean(0), got['forces'])
    assert np.allclose([w[0, 0], w[1, 1], w[2, 2], w[0, 1], w[0, 2], w[1, 2]],
                       got['virial'], atol=1e-5 * np.abs(got['virial']).max())


def test_deterministic_and_wrap_invariant():
    pos, cell, z = si8()
    a, pair, types = _hip(pos, cell, z, 'damp_bj', 'pbe')
    b = pair.compute(pos, cell, types)
    assert a['energy'] == b['energy'] and np.array_equal(a['forces'], b['forces'])
    c = pair.compute(pos + cell[0] * 2 - cell[2], cell, types)   # unwrapped copy
    assert abs(c['energy'] - a['energy']) < 1e-6 * abs(a['energy'])
    assert np.abs(c['forces'] - a['forces']).max() < 1e-5


def test_errors_and_empty():
    from sevennet_finetuning_amd._lib import E3GNNError
    from sevennet_finetuning_amd.d3 import PairD3
    with pytest.raises(NotImplementedError):
        PairD3(damping='damp_zerom')
    pair = PairD3().coeff(['Si'])
    with pytest.raises(E3GNNError, match='type out of range'):
        pair.compute(np.zeros((2, 3)), np.eye(3) * 5, [0, 3])
    out = pair.compute(np.zeros((0, 3)), np.eye(3) * 5, np.zeros(0, int))
    assert out['energy'] == 0.0 and out['forces'].shape == (0, 3)


def test_d3_calculator_stress_convention():
    from sevennet_finetuning_amd.d3 import D3Calculator
    from sevennet_finetuning_amd.structures import Atoms
    pos, cell, z = si8()
    at = Atoms(numbers=z, positions=pos, cell=cell, pbc=True)
    res = D3Calculator().calculate(at)
    ref = _oracle(pos, cell, z, 'damp_bj', 'pbe')
    v = ref['virial']
    want = -np.array([v[0], v[1], v[2], v[5], v[4], v[3]]) / abs(np.linalg.det(cell))
    assert np.allclose(res['stress'], want, atol=1e-5 * np.abs(want).max())


def test_per_item_c6_path_matches_table_path(monkeypatch):
    """Systems above 32,768 atoms evaluate C6 per pair-image instead of from
    the n x n table; both paths give the same result."""
    d = np.load(f'{GOLD}/hfo2_resdat.npz')
    z = np.array([CHEMICAL_SYMBOLS.index(str(s)) for s in d['symbols']])
    a, pair, types = _hip(d['pos'], d['cell'], z, 'damp_zero', 'pbe', rthr=3000.0)
    monkeypatch.setenv('E3GNN_D3_NO_C6TAB', '1')
    b = pair.compute(d['pos'], d['cell'], types)
    assert abs(a['energy'] - b['energy']) <= 1e-6 * abs(a['energy'])
    assert np.abs(a['forces'] - b['forces']).max() <= 1e-6 * np.abs(a['forces']).max() + 1e-9


@pytest.mark.parametrize('bin_bohr', ['5', '8', '13'])
def test_multi_bin_traversal_matches_oracle(monkeypatch, bin_bohr):
    """Small bins (E3GNN_D3_BIN) put several bins along every axis of these
    small cells, so the stencil walk, the image arithmetic of out-of-cell bins
    and the centre-distance culling are all exercised against the oracle
    (the default 30-bohr bins give one bin per axis below ~16 A)."""
    monkeypatch.setenv('E3GNN_D3_BIN', bin_bohr)
    d = np.load(f'{GOLD}/hfo2_resdat.npz')
    z = np.array([CHEMICAL_SYMBOLS.index(str(s)) for s in d['symbols']])
    kw = dict(rthr=3000.0)
    got, _, _ = _hip(d['pos'], d['cell'], z, 'damp_bj', 'pbe', **kw)
    _compare(got, _oracle(d['pos'], d['cell'], z, 'damp_bj', 'pbe', **kw))
    pos, cell = si_diamond((2, 2, 2), sigma=0.08, seed=3)
    zz = np.array([CHEMICAL_SYMBOLS.index(s) for s in mixed_symbols(len(pos))])
    kw = dict(rthr=2000.0, cn_thr=900.0)
    got, _, _ = _hip(pos, cell, zz, 'damp_zero', 'pbe0', **kw)
    _compare(got, _oracle(pos, cell, zz, 'damp_zero', 'pbe0', **kw))


def test_sevennet_d3_calculator_is_the_sum():
    """SevenNetD3Calculator (pair_style hybrid/overlay e3gnn d3) = SevenNet-0 +
    D3 term by term."""
    from sevennet_finetuning_amd.d3 import D3Calculator
    from sevennet_finetuning_amd.sevennet_calculator import (SevenNetCalculator,
                                                             SevenNetD3Calculator)
    from sevennet_finetuning_amd.structures import Atoms
    pos, cell, z = si8()
    at = Atoms(numbers=z, positions=pos, cell=cell, pbc=True)
    both = SevenNetD3Calculator(device='cuda:0')
    both.calculate(at)
    a = SevenNetCalculator(device='cuda:0')
    a.calculate(at)
    b = D3Calculator().calculate(at)
    assert abs(both.results['energy'] - (a.results['energy'] + b['energy'])) < 1e-6
    assert np.allclose(both.results['forces'], a.results['forces'] + b['forces'], atol=1e-6)
    assert np.allclose(both.results['stress'], a.results['stress'] + b['stress'], atol=1e-9)
    assert both.results['energy'] < a.results['energy']   # dispersion binds


def test_sevennet_d3_calculator_molecule():
    """A molecule without cell or pbc: energies and forces summed, no stress
    (neither term defines one), no division by the zero cell volume."""
    from sevennet_finetuning_amd.d3 import D3Calculator
    from sevennet_finetuning_amd.sevennet_calculator import (SevenNetCalculator,
                                                             SevenNetD3Calculator)
    from sevennet_finetuning_amd.structures import Atoms
    rng = np.random.default_rng(11)
    pos = rng.uniform(0, 5.0, (10, 3))
    keep = [0]
    for i in range(1, len(pos)):
        if np.min(np.linalg.norm(pos[keep] - pos[i], axis=1)) > 1.2:
            keep.append(i)
    pos = pos[keep]
    z = np.array([6, 8, 1, 7, 6, 1, 8, 6, 1, 1])[:len(pos)]
    at = Atoms(numbers=z, positions=pos, cell=None, pbc=False)
    both = SevenNetD3Calculator(device='cuda:0')
    both.calculate(at)
    assert 'stress' not in both.results
    a = SevenNetCalculator(device='cuda:0')
    a.calculate(at)
    b = D3Calculator().calculate(at)
    assert 'stress' not in b
    ref = _oracle(pos, np.eye(3) * 30.0, z, 'damp_bj', 'pbe', pbc=(False, False, False))
    assert abs(b['energy'] - ref['energy']) <= 1e-5 * abs(ref['energy'])
    assert abs(both.results['energy'] - (a.results['energy'] + b['energy'])) < 1e-6
    assert np.allclose(both.results['forces'], a.results['forces'] + b['forces'], atol=1e-6)
