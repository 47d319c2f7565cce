"""Device neighbour list (e3gnn_nlist_*, csrc/neighbor.hip) vs the host list
and the oracle's brute force: identical edges, order and integer shifts (bit
for bit), edge vectors within f32 rounding.  Needs an MI355X: ``pytest -m gpu``."""
import numpy as np
import pytest
import torch

from sevennet_finetuning_amd.neighbor import neighbor_list
from sevennet_finetuning_amd.structures import si_diamond

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def dnl():
    from sevennet_finetuning_amd.neighbor import DeviceNeighborList
    assert torch.cuda.is_available(), 'GPU tests need a HIP device'
    return DeviceNeighborList('cuda:0')


def run(dnl, pos, cell, rc=5.0, pbc=(True, True, True)):
    c, n, s, v = dnl(pos, cell, rc, pbc)
    return (np.stack([c.cpu().numpy(), n.cpu().numpy()]).astype(np.int64),
            s.cpu().numpy().astype(np.float64), v.cpu().numpy())


def host_vec(pos, cell, ei, sh):
    if cell is None:
        return (pos[ei[1]] - pos[ei[0]]).astype(np.float32)
    return ((pos[ei[1]] + sh @ cell) - pos[ei[0]]).astype(np.float32)


def check(dnl, pos, cell, rc=5.0, pbc=(True, True, True), brute=False):
    ei, sh, vec = run(dnl, pos, cell, rc, pbc)
    if brute:
        from oracle.neighbor import neighbor_list as ref
        ej, sj = ref(pos, cell, rc)
    else:
        ej, sj = neighbor_list(pos, cell, rc, pbc)
    assert np.array_equal(ei, ej)
    assert np.array_equal(sh, sj)
    if ei.shape[1]:
        assert np.abs(vec - host_vec(pos, cell, ei, sh)).max() <= 1e-5
    return ei, sh


@pytest.mark.parametrize('cells', [(1, 1, 1), (2, 2, 1), (3, 3, 3), (4, 3, 2)])
def test_si_boxes_vs_bruteforce(dnl, cells):
    pos, cell = si_diamond(cells, sigma=0.05)
    check(dnl, pos, cell, brute=True)


def test_triclinic_hfo2(dnl):
    d = np.load('tests/golden/hfo2_resdat.npz')
    check(dnl, d['pos'], d['cell'], brute=True)


def test_small_primitive_cell_many_images(dnl):
    """FCC primitive Si cell (2 atoms, heights < rc): every image within rc."""
    a = 5.43
    cell = 0.5 * a * np.array([[0, 1, 1], [1, 0, 1], [1, 1, 0]], dtype=np.float64)
    pos = np.array([[0, 0, 0], [0.25 * a, 0.25 * a, 0.25 * a]], dtype=np.float64)
    ei, _ = check(dnl, pos, cell, rc=6.0, brute=True)
    assert ei.shape[1] == 92  # 2 atoms x 46 neighbours within 6 A


def test_unwrapped_positions(dnl):
    """Atoms outside the cell (MD-style unwrapped coordinates): the shifts
    absorb the offsets, edges unchanged in geometry."""
    pos, cell = si_diamond((3, 3, 3), sigma=0.05)
    rng = np.random.default_rng(7)
    off = rng.integers(-3, 4, size=(len(pos), 3)).astype(np.float64) @ cell
    check(dnl, pos + off, cell)


def test_cluster_no_pbc(dnl):
    rng = np.random.default_rng(3)
    pos = rng.uniform(-6, 6, size=(300, 3))
    keep = [0]
    for i in range(1, len(pos)):
        if np.min(np.linalg.norm(pos[keep] - pos[i], axis=1)) > 1.6:
            keep.append(i)
    pos = pos[keep]
    ei, sh = check(dnl, pos, None, pbc=(False, False, False))
    assert not sh.any()
    # brute force over pairs
    d = np.linalg.norm(pos[:, None] - pos[None], axis=-1)
    ii, jj = np.nonzero((d < 5.0) & ~np.eye(len(pos), dtype=bool))
    assert np.array_equal(ei, np.stack([ii, jj]))


def test_isolated_and_empty(dnl):
    ei, _, _ = run(dnl, np.zeros((1, 3)), np.eye(3) * 20.0)
    assert ei.shape == (2, 0)
    ei, _, _ = run(dnl, np.zeros((0, 3)), np.eye(3) * 20.0)
    assert ei.shape == (2, 0)


def test_mixed_pbc_is_refused(dnl):
    from sevennet_finetuning_amd._lib import E3GNNError
    pos, cell = si_diamond((2, 2, 2), sigma=0.0)
    with pytest.raises(E3GNNError):
        dnl(pos, cell, 5.0, (True, True, False))


def test_bench_box_properties(dnl):
    """97,336-atom bench box: host list equality, 28 neighbours each, the
    (i, j, S) <-> (j, i, -S) symmetry, CSR order."""
    pos, cell = si_diamond((23, 23, 23), sigma=0.05)
    ei, sh = check(dnl, pos, cell)
    assert ei.shape[1] == 28 * len(pos)
    assert np.all(np.diff(ei[0]) >= 0)
    key = lambda i, j, s: ((i * len(pos) + j) * 64 + (s[:, 0] + 2) * 16 + (s[:, 1] + 2) * 4
                           + (s[:, 2] + 2))
    s = sh.astype(np.int64)
    assert np.array_equal(np.sort(key(ei[0], ei[1], s)), np.sort(key(ei[1], ei[0], -s)))


def test_energy_forces_from_device_list(dnl):
    """The device list feeds e3gnn_energy_forces directly: same energy and
    forces as with the host list."""
    from sevennet_finetuning_amd.model import E3GNNModel
    model = E3GNNModel(device='cuda:0')
    pos, cell = si_diamond((4, 4, 4), sigma=0.05)
    types = torch.full((len(pos),), model.chemical_symbols.index('Si'), dtype=torch.int32,
                       device='cuda:0')
    c, n, _, v = dnl(pos, cell, model.cutoff)
    a = model.energy_forces(types, c, n, v)
    ei, sh = neighbor_list(pos, cell, model.cutoff)
    vec = torch.tensor(host_vec(pos, cell, ei, sh), device='cuda:0')
    b = model.energy_forces(types, torch.tensor(ei[0], device='cuda:0'),
                            torch.tensor(ei[1], device='cuda:0'), vec)
    assert abs(float(a['energy']) - float(b['energy'])) <= 1e-6 * abs(float(b['energy']))
    assert (a['forces'] - b['forces']).abs().max().item() <= 1e-5
