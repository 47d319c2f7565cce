"""Brute-force periodic neighbor list (oracle copy) -- TEST INFRASTRUCTURE ONLY.

Edge convention of the reference (sevenn/train/dataload.py:113-125, ASE
``primitive_neighbor_list('ijDS', self_interaction=True)`` then dropping
i == j with zero shift): edge_index[0] = i (centre), edge_index[1] = j
(neighbor), shift S (integer image, so pos[j] + S @ cell - pos[i] = r_ij),
all images with |r_ij| < cutoff.  Edges sorted by i, then j, then S.
O(N^2 * images): for small cells only.
"""
import itertools

import numpy as np


def neighbor_list(pos, cell, cutoff, pbc=(True, True, True)):
    pos = np.asarray(pos, dtype=np.float64)
    cell = np.asarray(cell, dtype=np.float64)
    n = len(pos)
    vol = abs(np.linalg.det(cell))
    reps = []
    for k in range(3):
        if not pbc[k]:
            reps.append(0)
            continue
        cross = np.cross(cell[(k + 1) % 3], cell[(k + 2) % 3])
        height = vol / np.linalg.norm(cross)
        reps.append(int(np.ceil(cutoff / height)))
    ii, jj, ss = [], [], []
    for s in itertools.product(*[range(-r, r + 1) for r in reps]):
        s = np.array(s, dtype=np.float64)
        d = pos[None, :, :] + (s @ cell)[None, None, :] - pos[:, None, :]
        dist = np.linalg.norm(d, axis=-1)
        mask = dist < cutoff
        if not s.any():
            np.fill_diagonal(mask, False)
        i, j = np.nonzero(mask)
        ii.append(i)
        jj.append(j)
        ss.append(np.repeat(s[None, :], len(i), axis=0))
    i = np.concatenate(ii)
    j = np.concatenate(jj)
    s = np.concatenate(ss)
    order = np.lexsort((s[:, 2], s[:, 1], s[:, 0], j, i))
    return np.stack([i[order], j[order]]).astype(np.int64), s[order]
