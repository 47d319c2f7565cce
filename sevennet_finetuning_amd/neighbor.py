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


def _rij(pos_j, pos_i, S, cell):
    """r_ij = (pos_j + S cell) - pos_i, term by term in this order (elementwise
    f64, no fused multiply-add): the device list (csrc/neighbor.hip) evaluates
    the same expression, so the inclusion test agrees bit for bit."""
    S = np.asarray(S, dtype=np.float64)
    sc = [((S[..., 0] * cell[0, d]) + (S[..., 1] * cell[1, d])) + (S[..., 2] * cell[2, d])
          for d in range(3)]
    return np.stack([(pos_j[..., d] + sc[d]) - pos_i[..., d] for d in range(3)], axis=-1)


def _r2(d):
    return ((d[..., 0] * d[..., 0]) + (d[..., 1] * d[..., 1])) + (d[..., 2] * d[..., 2])


def _heights(cell):
    vol = abs(np.linalg.det(cell))
    return np.array([vol / np.linalg.norm(np.cross(cell[(k + 1) % 3], cell[(k + 2) % 3]))
                     for k in range(3)])


def _brute(pos, cell, cutoff, pbc, centers=None):
    h = _heights(cell) if any(pbc) else np.ones(3)
    ci = np.arange(len(pos)) if centers is None else np.asarray(centers, dtype=np.int64)
    reps = [int(np.ceil(cutoff / h[k])) if pbc[k] else 0 for k in range(3)]
    ii, jj, ss = [], [], []
    for s in itertools.product(*[range(-r, r + 1) for r in reps]):
        s = np.array(s, dtype=np.float64)
        d = _rij(pos[None, :, :], pos[ci, None, :], s, cell)
        mask = _r2(d) < cutoff * cutoff
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
        # image of the unwrapped positions: S = bin-image shift + f0[i] - f0[j]
        S = sh[:, None, :] + f0[idx][:, None, :] - f0[c]
        d = _rij(pos[c], pos[idx][:, None, :], S, cell)
        ok = valid & (_r2(d) < rc2)
        ok &= ~((c == idx[:, None]) & ~S.any(axis=2))
        r, k = np.nonzero(ok)
        ii.append(idx[r])
        jj.append(c[r, k])
        ss.append(S[r, k])
    return np.concatenate(ii), np.concatenate(jj), np.concatenate(ss)


def neighbor_list(pos, cell, cutoff, pbc=(True, True, True), centers=None):
    """Returns (edge_index int64 [2,E], shift float64 [E,3]) sorted by centre.
    ``centers``: optional subset of centre atoms (a rank's owned atoms in the
    domain decomposition); neighbours are still taken from every atom."""
    pos = np.ascontiguousarray(pos, dtype=np.float64)
    cell = np.zeros((3, 3)) if cell is None else np.ascontiguousarray(cell, dtype=np.float64)
    if all(pbc) and np.all(_heights(cell) >= 3 * cutoff):
        i, j, s = _cell_list(pos, cell, cutoff, centers)
    else:
        i, j, s = _brute(pos, cell, cutoff, pbc, centers)
    order = np.lexsort((s[:, 2], s[:, 1], s[:, 0], j, i))
    return (np.stack([i[order], j[order]]).astype(np.int64),
            np.ascontiguousarray(s[order]))


class DeviceNeighborList:
    """Neighbour list on the GPU (libe3gnn_hip.so ``e3gnn_nlist_*``), the same
    edges, order and integer shifts as ``neighbor_list`` (bit for bit).

    ``__call__(pos, cell, cutoff, pbc)`` returns device tensors
    ``(edge_center int32 [E], edge_nbr int32 [E], shift int32 [E, 3],
    edge_vec float32 [E, 3])``.  pbc must be all True or all False (the
    device list raises ``E3GNNError`` otherwise; ``neighbor_list`` covers the
    mixed case on the host)."""

    def __init__(self, device='cuda:0'):
        import torch
        from . import _lib
        self._torch, self._L = torch, _lib
        self.lib = _lib.load()
        self.device = torch.device(device)
        idx = self.device.index if self.device.index is not None else 0
        self._h = self.lib.e3gnn_nlist_create(idx)
        if not self._h:
            raise _lib.E3GNNError(self.lib.e3gnn_last_error().decode())

    def __del__(self):
        h, self._h = getattr(self, '_h', None), None
        if h:
            self.lib.e3gnn_nlist_free(h)

    def __call__(self, pos, cell, cutoff, pbc=(True, True, True)):
        import ctypes
        torch, L = self._torch, self._L
        dev = self.device
        pos = torch.as_tensor(pos).to(dev, torch.float64).contiguous()
        n = int(pos.shape[0])
        cellh = (ctypes.c_double * 9)(*np.asarray(cell, dtype=np.float64).reshape(-1).tolist()) \
            if cell is not None else (ctypes.c_double * 9)()
        pbch = (ctypes.c_int * 3)(*[int(bool(p)) for p in pbc])
        ne = ctypes.c_int64()
        s = torch.cuda.current_stream(dev).cuda_stream
        L.check(self.lib.e3gnn_nlist_build(self._h, n, pos.data_ptr(), cellh, pbch,
                                           float(cutoff), ctypes.byref(ne), s))
        E = ne.value
        center = torch.empty(E, dtype=torch.int32, device=dev)
        nbr = torch.empty(E, dtype=torch.int32, device=dev)
        shift = torch.empty(E, 3, dtype=torch.int32, device=dev)
        vec = torch.empty(E, 3, dtype=torch.float32, device=dev)
        L.check(self.lib.e3gnn_nlist_fetch(self._h, center.data_ptr(), nbr.data_ptr(),
                                           shift.data_ptr(), vec.data_ptr(), s))
        return center, nbr, shift, vec
