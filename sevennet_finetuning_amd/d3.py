"""DFT-D3 dispersion on the GPU -- SURVEY.md §8f row 4.

Python mirror of the reference's LAMMPS pair style ``d3``
(sevenn/pair_e3gnn/pair_d3.cu, pair_d3.h):

    pair_style d3 <rthr> <cn_thr> <damping> <functional>   -> PairD3(rthr, cn_thr, damping, functional)
    pair_coeff * * <element1> <element2> ...                 -> PairD3.coeff([...])
    PairD3::compute / update                                 -> PairD3.compute(pos, cell, types)

over the C ABI of libe3gnn_hip.so (``e3gnn_d3_create`` / ``e3gnn_d3_compute``,
kernels in csrc/d3.hip).  Units as LAMMPS metal: positions/cell in Angstrom,
energy eV, forces eV/A, virial eV (xx, yy, zz, xy, xz, yz); ``rthr`` and
``cn_thr`` are squared cutoffs in bohr^2 as in the reference (defaults of the
SevenNet-D3 recipes: 9000 and 1600).  ``D3Calculator`` wraps it ASE-style
(``energy``, ``free_energy``, ``forces``, ``stress`` with ASE's sign and
order).  The parameter tables are Grimme's published D3 data as the reference
ships them (assets/d3, exported by tools/export_d3_params.py).
"""
import ctypes
import json
import os

import numpy as np

from . import _lib
from .structures import CHEMICAL_SYMBOLS

ASSETS = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'assets', 'd3')
AU_TO_ANG = 0.52917726     # pair_d3.h:113
MAXC = 5
DAMPING = {'damp_zero': 1, 'damp_bj': 2, 'damp_zerom': 3, 'damp_bjm': 4}   # settings :279-282
_FUNC_KIND = {'damp_zero': 'zero', 'damp_bj': 'bj', 'damp_zerom': 'zerom', 'damp_bjm': 'bjm'}

_TABLES = None


def _tables():
    global _TABLES
    if _TABLES is None:
        d = np.load(os.path.join(ASSETS, 'd3_params.npz'))
        funcs = json.load(open(os.path.join(ASSETS, 'd3_functionals.json')))['functionals']
        _TABLES = ({k: d[k] for k in d.files}, funcs)
    return _TABLES


def element_tables(atomic_numbers):
    """Per-type D3 tables for LAMMPS types 1..nt = ``atomic_numbers``
    (PairD3::coeff :656-767: r2r4/rcov by element, r0ab in bohr, the C6
    reference grid with its coordination numbers, mxc = grid size)."""
    tab, _ = _tables()
    z = np.asarray(atomic_numbers, dtype=np.int64)
    if np.any(z < 1) or np.any(z > 94):
        raise ValueError('D3 parameters exist for elements 1..94 only')
    nt = len(z)
    c6 = np.zeros((nt, nt, MAXC, MAXC, 3), dtype=np.float32)
    mxc = np.zeros(nt, dtype=np.int32)
    rows = tab['c6ab']
    za, zb = rows[:, 1].astype(np.int64), rows[:, 2].astype(np.int64)
    ga, gb = (za - 1) // 100, (zb - 1) // 100          # grid index (get_limit_in_pars_array)
    ea, eb = za - 100 * ga, zb - 100 * gb
    for ia in range(nt):
        for ib in range(nt):
            sel = np.nonzero((ea == z[ia]) & (eb == z[ib]))[0]
            for r in sel:
                mxc[ia] = max(mxc[ia], ga[r] + 1)
                mxc[ib] = max(mxc[ib], gb[r] + 1)
                c6[ia, ib, ga[r], gb[r]] = (rows[r, 0], rows[r, 3], rows[r, 4])
                c6[ib, ia, gb[r], ga[r]] = (rows[r, 0], rows[r, 4], rows[r, 3])
    return {'rcov': tab['rcov'][z - 1].astype(np.float32),
            'r2r4': tab['r2r4'][z - 1].astype(np.float32),
            'r0ab': (tab['r0ab'][np.ix_(z - 1, z - 1)] / AU_TO_ANG).astype(np.float32),
            'mxc': mxc, 'c6ab': c6}


def functional_params(damping, functional_name):
    """(s6, s8, a1, a2, alp6, alp8) of PairD3::setfuncpar (:422-653)."""
    _, funcs = _tables()
    if damping not in DAMPING:
        raise ValueError(f'Unknown damping type {damping!r}: {sorted(DAMPING)}')
    table = funcs[_FUNC_KIND[damping]]
    key = functional_name.lower()
    if key not in table:
        raise ValueError(f'Functional name unknown: {functional_name!r}')
    p = table[key]
    return np.array([p['s6'], p['s18'], p['rs6'], p['rs18'], p['alp'], p['alp'] + 2.0],
                    dtype=np.float32)


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class PairD3:
    """pair_style d3 rthr cn_thr damping functional (+ pair_coeff * * elements)."""

    def __init__(self, rthr=9000.0, cn_thr=1600.0, damping='damp_bj', functional_name='pbe',
                 device=0):
        if damping == 'damp_zerom':
            raise NotImplementedError('damp_zerom: not implemented by the reference '
                                      '(pair_d3.cu:1550-1553)')
        self.rthr, self.cn_thr = float(rthr), float(cn_thr)
        self.damping, self.functional_name = damping, functional_name
        self.func = functional_params(damping, functional_name)
        self.device = int(device)
        self.lib = _lib.load()
        self.handle = None
        self.elements = None

    def coeff(self, elements):
        """pair_coeff * * El1 El2 ...: LAMMPS type t+1 is ``elements[t]``."""
        z = [e if isinstance(e, (int, np.integer)) else CHEMICAL_SYMBOLS.index(str(e).capitalize())
             for e in elements]
        t = element_tables(z)
        self.close()
        h = self.lib.e3gnn_d3_create(
            self.device, DAMPING[self.damping], _ptr(self.func), ctypes.c_float(self.rthr),
            ctypes.c_float(self.cn_thr), len(z), _ptr(t['rcov']), _ptr(t['r2r4']),
            _ptr(t['r0ab']), _ptr(t['mxc']), _ptr(np.ascontiguousarray(t['c6ab'])))
        if not h:
            raise _lib.E3GNNError(self.lib.e3gnn_last_error().decode())
        self.handle, self.elements, self._tables = h, list(z), t
        return self

    def compute(self, pos, cell, types, pbc=(True, True, True), stream=None):
        """types: 0-based indices into the coeff() element list.  Returns
        {'energy' eV, 'forces' [N,3] eV/A, 'virial' [6] eV (xx,yy,zz,xy,xz,yz)}."""
        if self.handle is None:
            raise _lib.E3GNNError('PairD3.coeff() has not been called')
        pos = np.ascontiguousarray(pos, dtype=np.float64).reshape(-1, 3)
        cell = np.ascontiguousarray(cell, dtype=np.float64).reshape(3, 3)
        types = np.ascontiguousarray(types, dtype=np.int32).reshape(-1)
        if types.shape[0] != pos.shape[0]:
            raise ValueError('types and positions disagree in length')
        pbc = np.ascontiguousarray([1 if p else 0 for p in pbc], dtype=np.int32)
        n = pos.shape[0]
        forces = np.zeros((n, 3), dtype=np.float64)
        energy = np.zeros(1, dtype=np.float64)
        virial = np.zeros(6, dtype=np.float64)
        if stream is None:
            import torch
            stream = torch.cuda.current_stream(self.device).cuda_stream
        _lib.check(self.lib.e3gnn_d3_compute(self.handle, n, _ptr(pos), _ptr(cell), _ptr(pbc),
                                             _ptr(types), _ptr(energy), _ptr(forces),
                                             _ptr(virial), stream))
        return {'energy': float(energy[0]), 'forces': forces, 'virial': virial}

    def close(self):
        if self.handle is not None:
            self.lib.e3gnn_d3_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class D3Calculator:
    """ASE-style calculator over PairD3.  Results: energy, free_energy,
    forces and stress = -virial / V in ASE order (xx, yy, zz, yz, xz, xy);
    no per-atom energies (the reference's pair style reports none either)."""

    implemented_properties = ['free_energy', 'energy', 'forces', 'stress']

    def __init__(self, damping='damp_bj', functional_name='pbe', rthr=9000.0, cn_thr=1600.0,
                 device=0):
        self.pair = PairD3(rthr, cn_thr, damping, functional_name, device)
        self.results = {}

    def calculate(self, atoms=None, properties=None, system_changes=None):
        z = np.asarray(atoms.get_atomic_numbers())
        elems = sorted(set(z.tolist()))
        if self.pair.elements != elems:
            self.pair.coeff(elems)
        types = np.searchsorted(np.asarray(elems), z)
        cell = np.asarray(atoms.get_cell(), dtype=np.float64).reshape(3, 3)
        pbc = np.asarray(atoms.get_pbc(), dtype=bool).reshape(-1)
        pos = np.asarray(atoms.get_positions(), dtype=np.float64)
        vol = abs(np.linalg.det(cell))
        molecule = not pbc.any()
        if molecule and not vol > 1e-12:
            # isolated molecule without a cell: any box works when no axis is
            # periodic (one bin per axis, no images); no stress
            ext = (pos.max(0) - pos.min(0)) if len(pos) else np.zeros(3)
            cell = np.diag(np.maximum(ext, 1.0) + 1.0)
        elif not vol > 1e-12:
            raise ValueError('D3: periodic axes need a non-singular cell')
        out = self.pair.compute(pos, cell, types, pbc)
        v = out['virial']
        self.results = {'energy': out['energy'], 'free_energy': out['energy'],
                        'forces': out['forces']}
        if not molecule:
            self.results['stress'] = -np.array([v[0], v[1], v[2], v[5], v[4], v[3]]) / vol
        return self.results
