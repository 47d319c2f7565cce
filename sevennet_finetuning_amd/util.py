"""Host helpers mirroring sevenn/util.py (pretrained_name_to_path :316-329,
unlabeled_atoms_to_input :234-245) and dataload.unlabeled_atoms_to_graph
(sevenn/train/dataload.py:31-68)."""
import os

import numpy as np

from . import _keys as KEY
from .neighbor import neighbor_list

ASSETS = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'assets')
PRETRAINED = {'sevennet-0': 'sevennet0', '7net-0': 'sevennet0',
              'sevennet-0_11july2024': 'sevennet0', '7net-0_11july2024': 'sevennet0'}


def pretrained_name_to_path(name: str) -> str:
    key = name.lower()
    if key not in PRETRAINED:
        raise ValueError('Not a valid potential')
    return os.path.join(ASSETS, PRETRAINED[key])


def unlabeled_atoms_to_graph(atoms, cutoff: float):
    """Graph dict of an Atoms-like object, reference edge convention
    (edge_index[0] = i centre, edge_index[1] = j, edge_vec = r_j + S.cell - r_i,
    self-pairs only through a non-zero image), edges sorted by centre."""
    pos = np.asarray(atoms.get_positions(), dtype=np.float64)
    cell = np.asarray(atoms.get_cell(), dtype=np.float64).reshape(3, 3)
    pbc = tuple(bool(p) for p in atoms.get_pbc())
    edge_index, shift = neighbor_list(pos, cell, cutoff, pbc)
    edge_vec = pos[edge_index[1]] + shift @ cell - pos[edge_index[0]]
    z = np.asarray(atoms.get_atomic_numbers())
    return {
        KEY.NODE_FEATURE: z,
        KEY.ATOMIC_NUMBERS: z,
        KEY.POS: pos,
        KEY.EDGE_IDX: edge_index,
        KEY.EDGE_VEC: edge_vec,
        KEY.CELL: cell,
        KEY.CELL_SHIFT: shift,
        KEY.CELL_VOLUME: float(np.einsum('i,i', cell[0], np.cross(cell[1], cell[2]))),
        KEY.NUM_ATOMS: len(z),
        KEY.INFO: {},
    }


def unlabeled_atoms_to_input(atoms, cutoff: float):
    return unlabeled_atoms_to_graph(atoms, cutoff)
