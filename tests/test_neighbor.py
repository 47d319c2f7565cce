"""Host neighbor list (product) vs the oracle's brute force: identical edge
sets, order (sorted by centre) and integer shifts -- bit-exact integer work."""
import numpy as np
import pytest

from sevennet_finetuning_amd.neighbor import neighbor_list
from sevennet_finetuning_amd.structures import si_diamond


@pytest.mark.parametrize('cells', [(1, 1, 1), (2, 2, 1), (3, 3, 3), (4, 3, 2)])
def test_neighbor_list_matches_bruteforce(cells):
    from oracle.neighbor import neighbor_list as brute
    pos, cell = si_diamond(cells, sigma=0.05)
    ei, sh = neighbor_list(pos, cell, 5.0)
    ej, sj = brute(pos, cell, 5.0)
    assert np.array_equal(ei, ej)
    assert np.array_equal(sh, sj)
    assert np.all(np.diff(ei[0]) >= 0)


def test_neighbor_list_triclinic_and_empty():
    from oracle.neighbor import neighbor_list as brute
    d = np.load('tests/golden/hfo2_resdat.npz')
    ei, sh = neighbor_list(d['pos'], d['cell'], 5.0)
    ej, sj = brute(d['pos'], d['cell'], 5.0)
    assert np.array_equal(ei, ej) and np.array_equal(sh, sj)
    # an isolated atom in a big box has no edges
    ei, sh = neighbor_list(np.zeros((1, 3)), np.eye(3) * 20.0, 5.0)
    assert ei.shape == (2, 0)


def test_cell_list_path_large_box():
    """12x12x12 cells exercise the cell-list branch; symmetric full list."""
    pos, cell = si_diamond((12, 12, 12), sigma=0.05)
    ei, sh = neighbor_list(pos, cell, 5.0)
    assert ei.shape[1] == 28 * len(pos)
    fwd = set(zip(ei[0], ei[1], map(tuple, sh.astype(int))))
    rev = set(zip(ei[1], ei[0], map(tuple, (-sh).astype(int))))
    assert fwd == rev
