"""DFT-D3 host logic and oracle (CPU).  The oracle (oracle/d3_ref.py) is a
numpy float64 restatement of the reference's pair_d3.cu; parity with the
reference's own numbers is UNPINNED (no D3 test, fixture or output ships with
the reference and pair_d3.cu builds only inside LAMMPS + CUDA), so the oracle
is checked for self-consistency here: forces = -dE/dx and virial = -dE/d(strain)
by central differences, translation invariance, and the parameter-table
mapping of PairD3::coeff / setfuncpar.  The HIP kernels are compared with this
oracle in tests/test_gpu_d3.py."""
import numpy as np
import pytest

from oracle import d3_ref as D
from sevennet_finetuning_amd import d3 as D3
from sevennet_finetuning_amd.structures import si_diamond

TABLES, FUNCS = D.load_tables()


def si8():
    pos, cell = si_diamond((1, 1, 1), sigma=0.05)
    return pos, cell, np.zeros(len(pos), int), D.type_tables([14], TABLES)


@pytest.mark.parametrize('damping', ['damp_bj', 'damp_zero'])
def test_oracle_forces_are_energy_gradients(damping):
    pos, cell, types, tt = si8()
    fp = D.functional(FUNCS, damping, 'pbe')
    r = D.d3(pos, cell, types, tt, fp, damping)
    h = 1e-5   # small: hard cutoffs make larger steps jump (pairs crossing rthr)
    for k, c in ((3, 1), (0, 0), (6, 2)):
        p1, p2 = pos.copy(), pos.copy()
        p1[k, c] += h
        p2[k, c] -= h
        fd = -(D.d3(p1, cell, types, tt, fp, damping)['energy']
               - D.d3(p2, cell, types, tt, fp, damping)['energy']) / (2 * h)
        assert abs(fd - r['forces'][k, c]) < 2e-7 + 1e-4 * abs(fd)
    assert np.abs(r['forces'].sum(0)).max() < 1e-12


@pytest.mark.parametrize('damping', ['damp_bj', 'damp_zero'])
def test_oracle_virial_is_strain_derivative(damping):
    """With rthr = 40000 bohr^2 (the pairs that cross the hard cutoff under a
    strain step carry ~rc^-4 less energy than at the default 9000, whose
    crossings alone shift a central difference by ~1e-3 relative)."""
    pos, cell, types, tt = si8()
    fp = D.functional(FUNCS, damping, 'pbe')
    kw = dict(rthr=40000.0)
    r = D.d3(pos, cell, types, tt, fp, damping, **kw)
    h = 1e-5
    scale = np.abs(r['virial']).max()
    for idx, (a, b) in enumerate([(0, 0), (1, 1), (2, 2), (0, 1), (0, 2), (1, 2)]):
        eps = np.zeros((3, 3))
        eps[a, b] = eps[b, a] = 1.0 if a == b else 0.5

        def e(s):
            m = np.eye(3) + s * eps
            return D.d3(pos @ m.T, cell @ m.T, types, tt, fp, damping, **kw)['energy']
        de = (e(h) - e(-h)) / (2 * h)
        assert abs(-de - r['virial'][idx]) < 1e-4 * scale, (a, b)


def test_oracle_translation_invariance():
    pos, cell, types, tt = si8()
    fp = D.functional(FUNCS, 'damp_bj', 'pbe')
    a = D.d3(pos, cell, types, tt, fp)
    b = D.d3(pos + np.array([1.3, -0.4, 7.9]), cell, types, tt, fp)
    assert abs(a['energy'] - b['energy']) < 1e-10
    assert np.abs(a['forces'] - b['forces']).max() < 1e-10


def test_element_tables_match_oracle_restatement():
    z = [72, 8, 14]
    got = D3.element_tables(z)
    want = D.type_tables(z, TABLES)
    assert np.array_equal(got['mxc'], want['mxc'])
    assert np.allclose(got['c6ab'], want['c6ab'], rtol=1e-6)
    assert np.allclose(got['r0ab'], want['r0ab'], rtol=1e-6)
    assert np.allclose(got['rcov'], want['rcov']) and np.allclose(got['r2r4'], want['r2r4'])
    # Hf has more C6 reference points than O
    assert got['mxc'][0] >= 1 and got['mxc'][1] >= 1


def test_functional_mapping_setfuncpar():
    # PBE-D3(BJ): a1 = 0.4289, s8 = 0.7875, a2 = 4.4407 (Grimme's table)
    s6, s8, a1, a2, alp6, alp8 = D3.functional_params('damp_bj', 'PBE')
    assert (s6, alp6, alp8) == (1.0, 14.0, 16.0)
    assert np.allclose([s8, a1, a2], [0.7875, 0.4289, 4.4407])
    s6, s8, a1, a2, _, _ = D3.functional_params('damp_zero', 'pbe')
    assert np.allclose([s6, s8, a1, a2], [1.0, 0.722, 1.217, 1.0])
    with pytest.raises(ValueError):
        D3.functional_params('damp_bj', 'not-a-functional')
    with pytest.raises(ValueError):
        D3.functional_params('damp_xyz', 'pbe')
