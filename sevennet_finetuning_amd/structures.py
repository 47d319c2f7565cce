"""Synthetic periodic boxes used by the bench and the parity tests.

The Si diamond recipe is the one the survey used for the reference CPU
baseline and the known-answer values: a = 5.43 A, the
8-atom conventional cell with the four fcc sites first and their
(1/4,1/4,1/4) partners second, cells replicated with the basis innermost,
``np.random.default_rng(seed).normal(0, 0.05, (N, 3))`` A displacements,
positions wrapped into the box.
"""
import itertools

import numpy as np

SI_A = 5.43
_FCC = np.array([[0.0, 0.0, 0.0], [0.0, 0.5, 0.5], [0.5, 0.0, 0.5], [0.5, 0.5, 0.0]])
DIAMOND_BASIS = np.concatenate([_FCC, _FCC + 0.25])

# types drawn for the "mixed" variant: Li, P, S, Cl
MIXED_SYMBOLS = ('Li', 'P', 'S', 'Cl')


def si_diamond(cells, a=SI_A, sigma=0.05, seed=0):
    """Returns (pos [N,3] float64, cell [3,3] float64)."""
    cells = tuple(int(c) for c in cells)
    frac = np.array([np.array(ijk) + b
                     for ijk in itertools.product(*[range(c) for c in cells])
                     for b in DIAMOND_BASIS])
    pos = frac * a
    cell = np.diag(np.array(cells, dtype=np.float64) * a)
    if sigma:
        pos = pos + np.random.default_rng(seed).normal(0.0, sigma, pos.shape)
        pos = np.mod(pos, np.diag(cell))
    return pos, cell


def mixed_symbols(n, seed=1):
    rng = np.random.default_rng(seed)
    return [MIXED_SYMBOLS[i] for i in rng.integers(0, len(MIXED_SYMBOLS), n)]
