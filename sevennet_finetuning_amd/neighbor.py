"""Host periodic neighbor list (cell list), reference edge convention.

Replaces the graph-building step before the hot path: ASE
``primitive_neighbor_list('ijDS')`` in the reference
(sevenn/train/dataload.py:31-68, :113-125) and the host loops of
pair_e3gnn.cpp:155-182.  Convention:

* edge_index[0] = i (centre, aggregation target), edge_index[1] = j
  (neighbor, gathered source);
* integer image shift S with r_ij = pos[j] + S @ cell - pos[i], |r_ij| < rc;
* every image is an edge, i == j only with S != 0 (periodic self images);
* edges sorted by (i, j, S) -- CSR by centre, which the HIP kernels require.
"""
import itertools

import numpy as np


def _heights(cell):
    vol = abs(np.linalg.det(cell))
    return np.array([vol / np.linalg.norm(np.cross(cell[(k + 1) % 3], cell[(k + 2) % 3]))
                     for k in range(3)])


def _brute(pos, cell, cutoff, pbc, centers=None):
    h = _heights(cell)
    ci = np.arange(len(pos)) if centers is None else np.asarray(centers, dtype=np.int64)
    reps = [int(np.ceil(cutoff / h[k])) if pbc[k] else 0 for k in range(3)]
    ii, jj, ss = [], [], []
    for s in itertools.product(*[range(-r, r + 1) for r in reps]):
        s = np.array(s, dtype=np.float64)
        d = pos[None, :, :] + (s @ cell)[None, None, :] - pos[ci, None, :]
        mask = np.einsum('ijk,ijk->ij', d, d) < cutoff * cutoff
        if not s.any():
            mask[np.arange(len(ci)), ci] = False
        i, j = np.nonzero(mask)
        i = ci[i]
        ii.append(i)
        jj.append(j)
        ss.append(np.broadcast_to(s, (len(i), 3)))
    return np.concatenate(ii), np.concatenate(jj), np.concatenate(ss)


def _cell_list(pos, cell, cutoff, centers=None):
    inv = np.linalg.inv(cell)
    frac = pos @ inv
    f0 = np.floor(frac)
    frac = frac - f0
    posw = frac @ cell
    nb = np.maximum((_heights(cell) / cutoff).astype(np.int64), 1)
    b3 = np.minimum((frac * nb).astype(np.int64), nb - 1)
    bid = (b3[:, 0] * nb[1] + b3[:, 1]) * nb[2] + b3[:, 2]
    order = np.argsort(bid, kind='stable')
    nbins = int(nb.prod())
    counts = np.bincount(bid, minlength=nbins)
    start = np.concatenate([[0], np.cumsum(counts)])
    m = int(counts.max())
    table = np.full((nbins, m), -1, dtype=np.int64)
    slot = np.arange(len(pos)) - start[bid[order]]
    table[bid[order], slot] = order
    ii, jj, ss = [], [], []
    rc2 = cutoff * cutoff
    idx = np.arange(len(pos)) if centers is None else np.asarray(centers, dtype=np.int64)
    for off in itertools.product((-1, 0, 1), repeat=3):
        nbc = b3[idx] + np.array(off)
        sh = np.floor_divide(nbc, nb)
        nbc = nbc - sh * nb
        nbid = (nbc[:, 0] * nb[1] + nbc[:, 1]) * nb[2] + nbc[:, 2]
        cand = table[nbid]                                  # [N, m]
        valid = cand >= 0
        c = np.where(valid, cand, 0)
        d = posw[c] + (sh.astype(np.float64) @ cell)[:, None, :] - posw[idx, None, :]
        ok = valid & (np.einsum('nmk,nmk->nm', d, d) < rc2)
        zero = ~sh.any(axis=1)
        ok &= ~((c == idx[:, None]) & zero[:, None])
        r, k = np.nonzero(ok)
        j = c[r, k]
        ii.append(idx[r])
        jj.append(j)
        ss.append(sh[r].astype(np.float64))
    i = np.concatenate(ii)
    j = np.concatenate(jj)
    s = np.concatenate(ss)
    s = s + f0[i] - f0[j]          # back to images of the unwrapped positions
    return i, j, s


def neighbor_list(pos, cell, cutoff, pbc=(True, True, True), centers=None):
    """Returns (edge_index int64 [2,E], shift float64 [E,3]) sorted by centre.
    ``centers``: optional subset of centre atoms (a rank's owned atoms in the
    domain decomposition); neighbours are still taken from every atom."""
    pos = np.ascontiguousarray(pos, dtype=np.float64)
    cell = np.ascontiguousarray(cell, dtype=np.float64)
    if all(pbc) and np.all(_heights(cell) >= 3 * cutoff):
        i, j, s = _cell_list(pos, cell, cutoff, centers)
    else:
        i, j, s = _brute(pos, cell, cutoff, pbc, centers)
    order = np.lexsort((s[:, 2], s[:, 1], s[:, 0], j, i))
    return (np.stack([i[order], j[order]]).astype(np.int64),
            np.ascontiguousarray(s[order]))
