"""DFT-D3 dispersion, numpy float64 restatement -- TEST INFRASTRUCTURE ONLY.

Follows the reference's LAMMPS pair style ``d3`` (sevenn/pair_e3gnn/pair_d3.cu,
CUDA, builds only inside LAMMPS: unbuildable here), term by term:

  units            positions and cell in bohr (AU_TO_ANG 0.52917726), energy in
                   hartree (AU_TO_EV 27.21138505) -- pair_d3.h:113-114
  atoms            wrapped into the cell, fractional a in [0, 1] -- load_atom_info :1182-1224
  images           tau = i a + j b + k c, |i| <= rep with rep = int(|sqrt(thr)/h|) + 1
                   (h = cell height along that axis), 0 along non-periodic axes
                   -- set_lattice_repetition_criteria :1026-1045, precalculate_tau_array :1230-1266
  CN               CN_i = sum_{j, T != self} 1 / (1 + exp(-K1 ((rcov_i + rcov_j) / r - 1))),
                   r^2 <= cn_thr, K1 = 16 -- kernel_get_coordination_number :1051-1104
  C6(CN_i, CN_j)   Gaussian-weighted mean of the reference C6 grid, K3 = -4, and
                   its CN derivatives; the nearest reference when all weights
                   underflow -- kernel_get_dC6_dCNij :808-887
  E (BJ)           -sum_pairs C6 (s6 / (r^6 + R0^6) + s8 3 r2r4_i r2r4_j / (r^8 + R0^8)),
                   R0 = a1 sqrt(3 r2r4_i r2r4_j) + a2 -- :1558-1768
  E (zero)         -sum_pairs C6 (s6 f6 / r^6 + 3 s8 r2r4_i r2r4_j f8 / r^8),
                   f_n = 1 / (1 + 6 (rs_n R0ab / r)^alp_n), alp6 = 14, alp8 = 16 -- :1273-1505
  pairs            unordered (i <= j) over images with r^2 <= rthr; the i == j
                   self-images (T != 0) count with weight 1/2
  forces           direct term + the C6(CN) chain dE/dCN_i * dCN_i/dr
                   -- kernel_get_forces_with_dC6 :1812-1976
  virial           sum over pair-images of (dE/dr r_hat) (x) r (LAMMPS order
                   xx, yy, zz, xy, xz, yz) -- update :2003-2024
  functionals      setfuncpar :422-653 (a1 = rs6, a2 = rs18, s8 = s18,
                   alp6 = alp, alp8 = alp + 2)

Parity is UNPINNED against the reference's own numbers: the reference ships no
D3 test, fixture or example output, and pair_d3.cu needs LAMMPS + CUDA.  This
restatement is checked for internal consistency (forces = -dE/dx and virial =
strain derivative by finite differences, translation/permutation invariance,
the C6 grid reproduced at the reference coordination numbers).
"""
import json
import os

import numpy as np

AU_TO_ANG = 0.52917726
AU_TO_EV = 27.21138505
K1 = 16.0
K3 = -4.0
MAXC = 5
ASSETS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                      'sevennet_finetuning_amd', 'assets', 'd3')


def load_tables(assets=ASSETS):
    d = np.load(os.path.join(assets, 'd3_params.npz'))
    funcs = json.load(open(os.path.join(assets, 'd3_functionals.json')))['functionals']
    return {k: d[k] for k in d.files}, funcs


def type_tables(elements_z, tables):
    """Per-type tables for atomic numbers ``elements_z`` (pair_d3.cu coeff
    :656-767, read_r0ab :354-367, read_c6ab :389-420)."""
    nt = len(elements_z)
    z = np.asarray(elements_z)
    r0ab = tables['r0ab'][np.ix_(z - 1, z - 1)] / AU_TO_ANG
    c6 = np.zeros((nt, nt, MAXC, MAXC, 3))
    mxc = np.zeros(nt, dtype=np.int64)
    for ref_c6, za, zb, cna, cnb in tables['c6ab']:
        za, zb = int(za), int(zb)
        ga, gb = (za - 1) // 100 + 1, (zb - 1) // 100 + 1   # grid index (get_limit_in_pars_array)
        ea, eb = za - (ga - 1) * 100, zb - (gb - 1) * 100
        ia = np.nonzero(z == ea)[0]
        ib = np.nonzero(z == eb)[0]
        if len(ia) == 0 or len(ib) == 0:
            continue
        ia, ib = ia[0], ib[0]
        mxc[ia] = max(mxc[ia], ga)
        mxc[ib] = max(mxc[ib], gb)
        c6[ia, ib, ga - 1, gb - 1] = (ref_c6, cna, cnb)
        c6[ib, ia, gb - 1, ga - 1] = (ref_c6, cnb, cna)
    return {'rcov': tables['rcov'][z - 1], 'r2r4': tables['r2r4'][z - 1], 'r0ab': r0ab,
            'c6ab': c6, 'mxc': mxc}


def functional(funcs, damping, name):
    kind = {'damp_zero': 'zero', 'damp_bj': 'bj', 'damp_zerom': 'zerom',
            'damp_bjm': 'bjm'}[damping]
    p = funcs[kind][name]
    return {'s6': p['s6'], 's8': p['s18'], 'a1': p['rs6'], 'a2': p['rs18'],
            'alp6': p['alp'], 'alp8': p['alp'] + 2.0}


def wrap_bohr(pos_ang, cell_ang):
    lat = np.asarray(cell_ang, dtype=np.float64) / AU_TO_ANG      # rows a, b, c
    frac = np.asarray(pos_ang, dtype=np.float64) / AU_TO_ANG @ np.linalg.inv(lat)
    frac = frac - np.floor(frac)          # the reference's while-loops: [0, 1)
    return frac @ lat, lat


def repetitions(lat, thr, pbc):
    rc = np.sqrt(thr)
    rep = []
    for k in range(3):
        cross = np.cross(lat[(k + 1) % 3], lat[(k + 2) % 3])
        h = abs(np.dot(cross, lat[k])) / np.linalg.norm(cross)
        rep.append(int(abs(rc / h)) + 1 if pbc[k] else 0)
    return rep


def translations(lat, rep):
    r = [np.arange(-m, m + 1) for m in rep]
    g = np.stack(np.meshgrid(*r, indexing='ij'), -1).reshape(-1, 3)
    return g @ lat, g


def _pairs(x, tau, thr, i_idx, j_idx):
    """All (i<=j pair, image) with r^2 <= thr, the self image of i == j excluded."""
    rij = x[j_idx][:, None, :] - x[i_idx][:, None, :] + tau[None, :, :]
    r2 = np.einsum('pti,pti->pt', rij, rij)
    keep = r2 <= thr
    self_img = (i_idx == j_idx)[:, None] & np.all(tau == 0.0, axis=1)[None, :]
    keep &= ~self_img
    p, t = np.nonzero(keep)
    return p, rij[p, t], r2[p, t]


def c6_and_derivs(tt, types, cn, i, j):
    c6tab = tt['c6ab'][types[i], types[j]]              # [P, 5, 5, 3]
    ref, cna, cnb = c6tab[..., 0], c6tab[..., 1], c6tab[..., 2]
    valid = ref > 0.0
    r = (cna - cn[i][:, None, None]) ** 2 + (cnb - cn[j][:, None, None]) ** 2
    w = np.where(valid, np.exp(K3 * r), 0.0)
    num = np.sum(w * ref, axis=(1, 2))
    den = np.sum(w, axis=(1, 2))
    dw_i = np.where(valid, w * 2.0 * K3 * (cn[i][:, None, None] - cna), 0.0)
    dw_j = np.where(valid, w * 2.0 * K3 * (cn[j][:, None, None] - cnb), 0.0)
    with np.errstate(invalid='ignore', divide='ignore'):
        c6 = num / den
        d_i = (np.sum(dw_i * ref, axis=(1, 2)) - c6 * np.sum(dw_i, axis=(1, 2))) / den
        d_j = (np.sum(dw_j * ref, axis=(1, 2)) - c6 * np.sum(dw_j, axis=(1, 2))) / den
    # all weights underflow: nearest reference, no derivative
    rr = np.where(valid, r, np.inf).reshape(len(i), -1)
    near = np.take_along_axis(ref.reshape(len(i), -1), np.argmin(rr, 1)[:, None], 1)[:, 0]
    small = ~(den > 1e-99)
    c6 = np.where(small, near, c6)
    d_i = np.where(small, 0.0, d_i)
    d_j = np.where(small, 0.0, d_j)
    return c6, d_i, d_j


def d3(pos_ang, cell_ang, types, tt, fp, damping='damp_bj', rthr=9000.0, cn_thr=1600.0,
       pbc=(True, True, True)):
    """Returns energy (eV), forces (eV/A, [N,3]), virial (eV, LAMMPS order
    xx,yy,zz,xy,xz,yz) and the coordination numbers."""
    if damping not in ('damp_bj', 'damp_bjm', 'damp_zero'):
        raise NotImplementedError(f'{damping}: not implemented by the reference either '
                                  '(pair_d3.cu:1550-1553)')
    types = np.asarray(types)
    x, lat = wrap_bohr(pos_ang, cell_ang)
    n = len(x)
    iu, ju = np.triu_indices(n)          # i <= j ...
    i_idx, j_idx = ju, iu                # ... as the reference's (iat >= jat) order
    tau_cn, _ = translations(lat, repetitions(lat, cn_thr, pbc))
    tau_vdw, _ = translations(lat, repetitions(lat, rthr, pbc))

    # coordination numbers
    p, rij, r2 = _pairs(x, tau_cn, cn_thr, i_idx, j_idx)
    a, b = i_idx[p], j_idx[p]
    r = np.sqrt(r2)
    rco = tt['rcov'][types[a]] + tt['rcov'][types[b]]
    ex = np.exp(-K1 * (rco / r - 1.0))
    damp = 1.0 / (1.0 + ex)
    cn = np.zeros(n)
    np.add.at(cn, a, damp)
    np.add.at(cn, b, np.where(a == b, 0.0, damp))

    # dispersion
    c6p, dci, dcj = c6_and_derivs(tt, types, cn, i_idx, j_idx)
    p, rij, r2 = _pairs(x, tau_vdw, rthr, i_idx, j_idx)
    a, b = i_idx[p], j_idx[p]
    c6, d6i, d6j = c6p[p], dci[p], dcj[p]
    half = np.where(a == b, 0.5, 1.0)
    r = np.sqrt(r2)
    r42 = tt['r2r4'][types[a]] * tt['r2r4'][types[b]]
    s6, s8 = fp['s6'], fp['s8']
    if damping == 'damp_zero':
        r0 = tt['r0ab'][types[a], types[b]]
        t6 = (fp['a1'] * r0 / r) ** fp['alp6']
        t8 = (fp['a2'] * r0 / r) ** fp['alp8']
        f6, f8 = 1.0 / (1.0 + 6.0 * t6), 1.0 / (1.0 + 6.0 * t8)
        e_rest = s6 * f6 / r ** 6 + 3.0 * s8 * r42 * f8 / r ** 8
        # d e_rest / dr
        de = (s6 * (-6.0 * f6 / r ** 7 + f6 * f6 * 6.0 * fp['alp6'] * t6 / r ** 7)
              + 3.0 * s8 * r42 * (-8.0 * f8 / r ** 9 + f8 * f8 * 6.0 * fp['alp8'] * t8 / r ** 9))
    else:
        R0 = fp['a1'] * np.sqrt(3.0 * r42) + fp['a2']
        t6 = 1.0 / (r ** 6 + R0 ** 6)
        t8 = 1.0 / (r ** 8 + R0 ** 8)
        e_rest = s6 * t6 + 3.0 * s8 * r42 * t8
        de = -(s6 * 6.0 * r ** 5 * t6 * t6 + 3.0 * s8 * r42 * 8.0 * r ** 7 * t8 * t8)
    energy = -np.sum(half * c6 * e_rest)
    dEdr = -half * c6 * de                               # dE/dr along r_ij = x_j - x_i + T
    fvec = dEdr[:, None] * rij / r[:, None]
    forces = np.zeros((n, 3))
    np.add.at(forces, a, fvec)                           # dE/dx_i = -dE/dr_ij
    np.add.at(forces, b, -fvec)
    vir = -np.einsum('pi,pj->ij', fvec, rij)             # -(dE/dr r_hat) (x) r
    dEdcn = np.zeros(n)                                  # dE/dCN
    np.add.at(dEdcn, a, -half * e_rest * d6i)
    np.add.at(dEdcn, b, -half * e_rest * d6j)

    # C6(CN) chain
    p, rij, r2 = _pairs(x, tau_cn, cn_thr, i_idx, j_idx)
    a, b = i_idx[p], j_idx[p]
    r = np.sqrt(r2)
    rco = tt['rcov'][types[a]] + tt['rcov'][types[b]]
    ex = np.exp(-K1 * (rco / r - 1.0))
    dcn_dr = -K1 * rco * ex / (r2 * (1.0 + ex) ** 2)      # d damp / dr
    w = np.where(a == b, dEdcn[a], dEdcn[a] + dEdcn[b])
    fvec = (w * dcn_dr)[:, None] * rij / r[:, None]
    np.add.at(forces, a, np.where((a == b)[:, None], 0.0, fvec))
    np.add.at(forces, b, np.where((a == b)[:, None], 0.0, -fvec))
    vir -= np.einsum('pi,pj->ij', fvec, rij)
    virial = np.array([vir[0, 0], vir[1, 1], vir[2, 2], vir[0, 1], vir[0, 2], vir[1, 2]])
    return {'energy': energy * AU_TO_EV, 'forces': forces * AU_TO_EV / AU_TO_ANG,
            'virial': virial * AU_TO_EV, 'cn': cn}
