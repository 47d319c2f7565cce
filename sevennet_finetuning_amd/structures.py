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


def diamond_primitive(cells, a=SI_A, sigma=0.05, seed=0):
    """Fine-tune cells of SURVEY.md 8d config 5: the 2-atom fcc primitive
    diamond cell (vectors a/2 (0,1,1), (1,0,1), (1,1,0); basis 0 and
    (1/4,1/4,1/4) in fractional coordinates) replicated n1 x n2 x n3,
    N(0, sigma) displacements from ``default_rng(seed)``, wrapped back into
    the (triclinic) cell.  Returns (pos [N,3] float64, cell [3,3])."""
    cells = tuple(int(c) for c in cells)
    prim = 0.5 * a * np.array([[0.0, 1.0, 1.0], [1.0, 0.0, 1.0], [1.0, 1.0, 0.0]])
    frac = np.array([(np.array(ijk) + b) / np.array(cells)
                     for ijk in itertools.product(*[range(c) for c in cells])
                     for b in ([0.0, 0.0, 0.0], [0.25, 0.25, 0.25])])
    cell = prim * np.array(cells, dtype=np.float64)[:, None]
    pos = frac @ cell
    if sigma:
        pos = pos + np.random.default_rng(seed).normal(0.0, sigma, pos.shape)
        f = np.mod(pos @ np.linalg.inv(cell), 1.0)
        pos = f @ cell
    return pos, cell


def tile(pos, cell, reps):
    """Periodic supercell of (pos, cell): reps = (k1, k2, k3) copies along the
    lattice vectors, image-major (atom a of image m is row m * len(pos) + a).
    Every image has the same environment, so E(supercell) = k1 k2 k3 E(cell)
    and the forces repeat per image (the full-size parity property)."""
    reps = tuple(int(k) for k in reps)
    pos = np.asarray(pos, dtype=np.float64)
    cell = np.asarray(cell, dtype=np.float64)
    shifts = np.array(list(itertools.product(*[range(k) for k in reps])), dtype=np.float64)
    big = (shifts @ cell)[:, None, :] + pos[None]
    return big.reshape(-1, 3), cell * np.array(reps, dtype=np.float64)[:, None]


def morton_order(pos, cell, bin_width):
    """Permutation that sorts atoms by the Z-order (Morton) index of their
    spatial bin (bins of ~bin_width along each lattice vector), ascending atom
    id inside a bin -- the spatial sort LAMMPS applies (atom_modify sort), so
    that atoms close in space are close in memory."""
    pos = np.asarray(pos, dtype=np.float64)
    cell = np.asarray(cell, dtype=np.float64)
    frac = pos @ np.linalg.inv(cell)
    frac -= np.floor(frac)
    lens = np.linalg.norm(cell, axis=1)
    nb = np.maximum((lens / bin_width).astype(np.int64), 1)
    b = np.minimum((frac * nb).astype(np.int64), nb - 1)
    code = np.zeros(len(pos), dtype=np.int64)
    for bit in range(21):
        for k in range(3):
            code |= ((b[:, k] >> bit) & 1) << (3 * bit + k)
    return np.lexsort((np.arange(len(pos)), code))


def mixed_symbols(n, seed=1):
    rng = np.random.default_rng(seed)
    return [MIXED_SYMBOLS[i] for i in rng.integers(0, len(MIXED_SYMBOLS), n)]


# ASE's chemical_symbols order (index = atomic number), used for the
# chemical_symbols_to_index type map (sevennet_calculator.py:80-102)
CHEMICAL_SYMBOLS = (
    'X H He Li Be B C N O F Ne Na Mg Al Si P S Cl Ar K Ca Sc Ti V Cr Mn Fe Co Ni Cu Zn Ga Ge '
    'As Se Br Kr Rb Sr Y Zr Nb Mo Tc Ru Rh Pd Ag Cd In Sn Sb Te I Xe Cs Ba La Ce Pr Nd Pm Sm '
    'Eu Gd Tb Dy Ho Er Tm Yb Lu Hf Ta W Re Os Ir Pt Au Hg Tl Pb Bi Po At Rn Fr Ra Ac Th Pa U '
    'Np Pu Am Cm Bk Cf Es Fm Md No Lr Rf Db Sg Bh Hs Mt Ds Rg Cn Nh Fl Mc Lv Ts Og').split()


def atomic_number(symbol):
    return CHEMICAL_SYMBOLS.index(symbol)


class Atoms:
    """Minimal ase.Atoms stand-in (ASE is not installed here): the calculator
    only calls get_positions / get_cell / get_pbc / get_atomic_numbers."""

    def __init__(self, symbols=None, positions=None, cell=None, pbc=True, numbers=None):
        if numbers is None:
            numbers = [atomic_number(s) for s in symbols]
        self.numbers = np.asarray(numbers, dtype=np.int64)
        self.positions = np.asarray(positions, dtype=np.float64).reshape(-1, 3)
        self.cell = np.zeros((3, 3)) if cell is None else np.asarray(cell, dtype=np.float64)
        self.pbc = np.array([pbc] * 3 if np.isscalar(pbc) else pbc, dtype=bool)
        self.calc = None

    def __len__(self):
        return len(self.numbers)

    def get_positions(self):
        return self.positions.copy()

    def get_cell(self):
        return self.cell.copy()

    def get_pbc(self):
        return self.pbc.copy()

    def get_atomic_numbers(self):
        return self.numbers.copy()

    def get_chemical_symbols(self):
        return [CHEMICAL_SYMBOLS[z] for z in self.numbers]

    def get_volume(self):
        return abs(np.linalg.det(self.cell))

    def get_potential_energy(self):
        self.calc.calculate(self)
        return self.calc.results['energy']

    def get_forces(self):
        self.calc.calculate(self)
        return self.calc.results['forces']

    def get_stress(self):
        self.calc.calculate(self)
        return self.calc.results['stress']
