"""SevenNet-0-shaped models of other widths and depths on the fused kernels.

The reference builds any nequip configuration (model_build.py:196-372); the
SevenNet-0 preset with another ``channel`` or ``num_convolution_layer``
(lmax 2, even parity, XPLOR, 8 Bessel, 64-64 radial MLP, linear
self-connection) is served by the same fused radial-MLP + tensor-product
kernels as SevenNet-0 itself, instantiated per channel family (csrc/tp.h
Family<f>): uniform 64 and uniform 32 channels, any number of blocks >= 2.
Needs an MI355X: ``pytest -m gpu``.

Oracle: oracle/nequip_ref.py (the fp64 restatement of the whole family,
pinned by the reference KATs in tests/test_oracle.py) on the same deployment
(model_build.deploy_config, e3nn initialisation, seeded).  Tolerances
(north_star): energy 2e-6 relative, forces 1e-4 eV/A, stress 2e-6 eV/A^3.
Cross-check: the same deployment on the generic runtime-table engine
(E3GNN_GENERIC=1), an independent implementation of every kernel.
"""
import os

import numpy as np
import pytest
import torch

from _systems import system

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'


@pytest.fixture(scope='module', params=[(64, 4, 1), (32, 3, 2), (64, 2, 1)],
                ids=['c64_l4', 'c32_l3', 'c64_l2'])
def deployment(request, tmp_path_factory):
    from sevennet_finetuning_amd import model_build as mb
    ch, L, fam = request.param
    d = str(tmp_path_factory.mktemp(f'c{ch}l{L}'))
    mb.deploy_config(mb.sevennet_shaped_config(ch, L), d, seed=ch + L)
    return d, fam


def _oracle(model_dir, pos, cell, types):
    from oracle.neighbor import neighbor_list
    from oracle.nequip_ref import NequIPRef
    ref = NequIPRef(model_dir)
    ei, sh = neighbor_list(pos, cell, ref.cutoff)
    out = ref(torch.tensor(pos), torch.tensor(types), torch.tensor(ei), torch.tensor(sh),
              torch.tensor(cell))
    return {k: (v.numpy() if torch.is_tensor(v) else v) for k, v in out.items()}


def _run(model, pos, cell, types):
    from sevennet_finetuning_amd.neighbor import neighbor_list
    ei, sh = neighbor_list(pos, cell, model.cutoff)
    vec = pos[ei[1]] + sh @ cell - pos[ei[0]]
    t = lambda a, dt=torch.int32: torch.as_tensor(a, dtype=dt, device=DEV)  # noqa: E731
    r = model.energy_forces(t(types), t(ei[0]), t(ei[1]), t(vec, torch.float32))
    vol = abs(np.linalg.det(cell))
    return {'energy': float(r['energy']), 'forces': r['forces'].cpu().numpy(),
            'stress': r['virial'].cpu().numpy() / vol}


@pytest.mark.parametrize('name', ['mixed_2x1x1', 'si_rng0_2x2x1', 'mixed_3x3x3'])
def test_family_model_vs_oracle(deployment, name):
    """Energy, forces and stress of a channel-family deployment on the fused
    kernels against the fp64 oracle of the reference's model."""
    from sevennet_finetuning_amd.model import E3GNNModel
    d, fam = deployment
    m = E3GNNModel(d, device=DEV)
    assert m.family == fam   # the fused kernels serve it, not the generic engine
    pos, cell, types = system(name, m.chemical_symbols)
    got = _run(m, pos, cell, types)
    ref = _oracle(d, pos, cell, types)
    e = float(ref['energy'])
    assert abs(got['energy'] - e) <= 2e-6 * abs(e), (got['energy'], e)
    assert np.abs(got['forces'] - ref['forces']).max() <= 1e-4
    assert np.abs(got['stress'] - ref['stress']).max() <= 2e-6
    assert np.abs(ref['forces']).max() > 1e-3   # a real force field (10x the tolerance), not zeros


def test_family_model_equals_generic_engine(deployment, monkeypatch):
    """The fused family engine and the generic runtime-table engine (two
    independent HIP implementations) agree on a mixed-species box, and the
    family engine is bitwise repeatable."""
    from sevennet_finetuning_amd.model import E3GNNModel
    d, fam = deployment
    a = E3GNNModel(d, device=DEV)
    monkeypatch.setenv('E3GNN_GENERIC', '1')
    b = E3GNNModel(d, device=DEV)
    assert a.family == fam and b.family == -1
    pos, cell, types = system('mixed_3x3x3', a.chemical_symbols)
    ra, rb = _run(a, pos, cell, types), _run(b, pos, cell, types)
    assert abs(ra['energy'] - rb['energy']) <= 2e-6 * abs(rb['energy'])
    assert np.abs(ra['forces'] - rb['forces']).max() <= 5e-5
    again = _run(a, pos, cell, types)
    assert again['energy'] == ra['energy'] and np.array_equal(again['forces'], ra['forces'])


def test_family_model_decomposed_matches_serial(deployment, tmp_path):
    """Two ranks (gloo, both on the box's GPU) through the segment API and
    the per-layer halo exchanges (parallel.py) = the serial evaluation."""
    import socket

    import torch.multiprocessing as mp
    from _parallel_workers import worker
    from sevennet_finetuning_amd.model import E3GNNModel
    d, _ = deployment
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    out = str(tmp_path / 'fam2.npz')
    mp.spawn(worker, args=(2, port, 'mixed_3x3x3', 'hip', out, d), nprocs=2, join=True)
    got = np.load(out)
    m = E3GNNModel(d, device=DEV)
    pos, cell, types = system('mixed_3x3x3', m.chemical_symbols)
    one = _run(m, pos, cell, types)
    assert abs(float(got['energy']) - one['energy']) <= 2e-6 * abs(one['energy'])
    assert np.abs(got['forces'] - one['forces']).max() <= 1e-4
