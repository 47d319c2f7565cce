"""Spatial domain decomposition of the energy/force path over torch.distributed.

The reference's multi-GPU path is ``pair_style e3gnn/parallel``
(pair_e3gnn_parallel.cpp): LAMMPS bricks own atoms, every rank evaluates the
edges whose centre it owns, and the node features of ghost atoms are exchanged
at every interaction-layer boundary (``pack/unpack_forward_comm_gnn``,
pair_e3gnn_parallel.cpp:803-870) with the reverse exchange of dE/dx_ghost in
the backward (``pack/unpack_reverse_comm_gnn``, :872-933), then the ghost
forces go back to their owners (LAMMPS reverse comm, newton on) and energy and
virial are summed over ranks.

Here, one process per GPU:

* ``brick_grid(world)`` splits the cell into px x py x pz bricks of fractional
  coordinates (2 -> 2x1x1, 4 -> 2x2x1, 8 -> 2x2x2), owner = brick of the
  wrapped position.
* ``build_rank_graph`` gives a rank its owned atoms (sorted by global id),
  their edges (neighbour list restricted to owned centres) and the ghost nodes
  = every non-owned neighbour, deduplicated by atom id (periodic images of one
  atom share a ghost row: features do not depend on the image; the image only
  enters the edge vector), ordered by (owner rank, id) so each peer's ghosts
  are one contiguous block.  A one-time handshake (all_to_all) tells every
  owner which of its rows each peer needs.
* ``Halo`` moves rows with one ``all_to_all_single`` per exchange (RCCL over
  xGMI with backend "nccl"; host-staged with "gloo"), packing and unpacking
  with the library's halo kernels.  Reverse exchanges accumulate per peer
  block in rank order (deterministic; no atomics).  Exchanges are started
  asynchronously and overlapped with the work that does not need them: the
  interior centres (owned atoms without ghost neighbours, ordered first) in
  the forward, the interior centres and owned rows in the backward
  (e3gnn_layer_forward_part / _backward_part).
* ``ParallelE3GNN.set_graph`` uploads a rank graph once per neighbour list;
  ``evaluate`` runs one evaluation: graph_set, 5 x (halo forward, layer
  forward), readout, 5 x (layer backward, halo reverse), forces, reverse of
  the ghost forces, one all_reduce of (energy, virial).

The per-rank compute is an *engine* with the segment interface of
include/e3gnn.h (``HipSegmentEngine`` wraps libe3gnn_hip.so; tests plug in a
CPU engine built on the oracle to check the decomposition itself).
"""
import time
from dataclasses import dataclass, field

import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from .neighbor import neighbor_list


# ------------------------------------------------------------------ partition
def brick_grid(world):
    """px >= py >= pz with px*py*pz = world, splitting the longest side first."""
    dims = [1, 1, 1]
    n = int(world)
    f = 2
    primes = []
    while n > 1:
        while n % f == 0:
            primes.append(f)
            n //= f
        f += 1
    for p in sorted(primes, reverse=True):
        k = int(np.argmin(dims))
        dims[k] *= p
    return tuple(sorted(dims, reverse=True))


def owners(pos, cell, grid):
    """Owner rank of every atom: brick of its wrapped fractional position."""
    frac = np.asarray(pos, dtype=np.float64) @ np.linalg.inv(np.asarray(cell, dtype=np.float64))
    frac -= np.floor(frac)
    g = np.asarray(grid, dtype=np.int64)
    b = np.minimum((frac * g).astype(np.int64), g - 1)
    return (b[:, 0] * g[1] + b[:, 1]) * g[2] + b[:, 2]


@dataclass
class RankGraph:
    """One rank's graph in the segment layout of e3gnn_graph_set."""
    rank: int
    world: int
    grid: tuple
    owned: np.ndarray            # global ids of owned atoms -> rows [0, n_local):
                                 # interior atoms first, then boundary, each by id
    ghosts: np.ndarray           # global ids of ghost rows [n_local, n_local + n_ghost)
    types: np.ndarray            # int32 [n_local + n_ghost]
    center: np.ndarray           # int32 [E] (sorted, < n_local)
    nbr: np.ndarray              # int32 [E] (< n_local + n_ghost)
    vec: np.ndarray              # float64 [E, 3] = x_j - x_i (+ image); engines cast
    recv_counts: np.ndarray      # ghosts received from each rank
    recv_rows: np.ndarray        # ghost rows, grouped by owner rank
    req_ids: np.ndarray          # global ids of those ghosts (what we ask the owners for)
    n_interior: int = 0          # owned rows [0, n_interior) have no ghost neighbour
    send_counts: np.ndarray = field(default=None)  # rows each peer asks of us
    send_rows: np.ndarray = field(default=None)    # our local rows, grouped by peer

    @property
    def n_local(self):
        return len(self.owned)

    @property
    def n_ghost(self):
        return len(self.ghosts)


def build_rank_graph(pos, cell, types, cutoff, grid, rank, pbc=(True, True, True)):
    """Local graph of ``rank`` (no communication; see ``handshake``).  Owned
    atoms whose neighbours are all owned (interior) come first, so the
    library can convolve them while the halo is in flight (e3gnn_set_interior)."""
    pos = np.asarray(pos, dtype=np.float64)
    cell = np.asarray(cell, dtype=np.float64)
    types = np.asarray(types)
    world = int(np.prod(grid))
    own = owners(pos, cell, grid)
    mine = np.nonzero(own == rank)[0]
    ei, sh = neighbor_list(pos, cell, cutoff, pbc=pbc, centers=mine)
    i, j = ei
    boundary = np.zeros(len(pos), dtype=bool)
    boundary[i[own[j] != rank]] = True
    owned = np.concatenate([mine[~boundary[mine]], mine[boundary[mine]]])
    n_interior = int((~boundary[mine]).sum())
    gj = np.unique(j[own[j] != rank])
    ghosts = gj[np.lexsort((gj, own[gj]))]
    lid = np.full(len(pos), -1, dtype=np.int64)
    lid[owned] = np.arange(len(owned))
    lid[ghosts] = len(owned) + np.arange(len(ghosts))
    # CSR by local centre row (stable: each centre keeps the (j, S) order)
    order = np.argsort(lid[i], kind='stable')
    i, j, sh = i[order], j[order], sh[order]
    vec = pos[j] + sh @ cell - pos[i]
    return RankGraph(
        rank=rank, world=world, grid=tuple(grid), owned=owned, ghosts=ghosts,
        types=np.concatenate([types[owned], types[ghosts]]).astype(np.int32),
        center=lid[i].astype(np.int32), nbr=lid[j].astype(np.int32),
        vec=vec,
        recv_counts=np.bincount(own[ghosts], minlength=world).astype(np.int64),
        recv_rows=(len(owned) + np.arange(len(ghosts))).astype(np.int64),
        req_ids=ghosts.astype(np.int64), n_interior=n_interior)


def handshake(rg, group=None, device='cpu'):
    """Tell every owner which of its atoms we need (global ids, one-time per
    graph); the owner turns them into its local rows."""
    w = rg.world
    if w == 1:
        rg.send_counts = np.zeros(1, dtype=np.int64)
        rg.send_rows = np.zeros(0, dtype=np.int64)
        return rg
    rc = torch.as_tensor(rg.recv_counts, dtype=torch.int64, device=device)
    sc = torch.empty_like(rc)
    dist.all_to_all_single(sc, rc, group=group)
    send_counts = sc.cpu().numpy()
    req = torch.as_tensor(rg.req_ids, dtype=torch.int64, device=device)
    ids = torch.empty(int(send_counts.sum()), dtype=torch.int64, device=device)
    dist.all_to_all_single(ids, req, output_split_sizes=send_counts.tolist(),
                           input_split_sizes=rg.recv_counts.tolist(), group=group)
    ids = ids.cpu().numpy()
    local_of = {int(g): r for r, g in enumerate(rg.owned)} if len(ids) < 4096 else None
    if local_of is not None:
        rows = np.array([local_of[int(g)] for g in ids], dtype=np.int64)
    else:   # vectorised: owned ids sorted, positions mapped back to rows
        srt = np.argsort(rg.owned)
        rows = srt[np.searchsorted(rg.owned, ids, sorter=srt)].astype(np.int64)
    if len(ids) and not np.array_equal(rg.owned[rows], ids):
        raise RuntimeError('halo handshake: a peer asked for an atom this rank does not own')
    rg.send_counts = send_counts
    rg.send_rows = rows
    return rg


def local_handshake(rgs):
    """``handshake`` for ALL ranks' graphs held by one process (the rank
    emulation of bench.py --rank-emulation, tests): every owner's send lists
    from its peers' requests, without a process group."""
    world = len(rgs)
    for r, rg in enumerate(rgs):
        counts, rows = np.zeros(world, dtype=np.int64), []
        srt = np.argsort(rg.owned)
        for p, q in enumerate(rgs):
            if p == r or q.req_ids.size == 0:
                rows.append(np.zeros(0, dtype=np.int64))
                continue
            lo = int(q.recv_counts[:r].sum())
            ids = q.req_ids[lo:lo + int(q.recv_counts[r])]   # q's ghosts owned by r, by id
            rr = srt[np.searchsorted(rg.owned, ids, sorter=srt)].astype(np.int64) if ids.size else \
                np.zeros(0, dtype=np.int64)
            if ids.size and not np.array_equal(rg.owned[rr], ids):
                raise RuntimeError('local handshake: a peer asked for an atom this rank does not own')
            counts[p] = ids.size
            rows.append(rr)
        rg.send_counts, rg.send_rows = counts, np.concatenate(rows)
    return rgs


# ------------------------------------------------------------------ halo
class Halo:
    """Forward (owner rows -> ghost rows) and reverse (ghost rows -> owner rows,
    accumulated) row exchanges of one RankGraph."""

    def __init__(self, rg, engine, group=None):
        self.rg, self.eng, self.group = rg, engine, group
        dev = engine.device
        self.staged = dist.is_initialized() and dist.get_backend(group) == 'gloo' \
            and torch.device(dev).type != 'cpu'
        i32 = lambda a: torch.as_tensor(np.asarray(a, dtype=np.int32), device=dev)
        self.send_rows = i32(rg.send_rows)
        self.recv_rows = i32(rg.recv_rows)
        self.sc = [int(x) for x in rg.send_counts]
        self.rc = [int(x) for x in rg.recv_counts]
        self.soff = np.concatenate([[0], np.cumsum(self.sc)]).astype(np.int64)

    def _a2a_start(self, out, inp, out_splits, in_splits):
        """Start an all_to_all (async on the device with RCCL: ordered after
        the pack on the current stream, waited for on the stream in finish)."""
        if self.staged:
            o = torch.empty(out.shape, dtype=out.dtype)
            w = dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits, group=self.group,
                                       async_op=True)
            return [w, o, out]
        w = dist.all_to_all_single(out, inp, out_splits, in_splits, group=self.group,
                                   async_op=True)
        return [w, None, out]

    @staticmethod
    def _a2a_wait(h):
        """Complete an all_to_all started by _a2a_start (idempotent)."""
        if h[0] is None:
            return
        w, o, out = h
        w.wait()
        if o is not None:
            out.copy_(o)
        h[0] = None

    def forward_start(self, kind, t):
        """Ghost rows of buffer (kind, t) <- their owners' rows: pack + start."""
        if self.rg.world == 1:
            return None
        dim = self.eng.dim(kind, t)
        sbuf = self.eng.empty(sum(self.sc), dim)
        rbuf = self.eng.empty(sum(self.rc), dim)
        self.eng.pack(kind, t, self.send_rows, sbuf)
        return (kind, t, rbuf, sbuf, self._a2a_start(rbuf, sbuf, self.rc, self.sc))

    def forward_finish(self, h):
        if h is None:
            return
        kind, t, rbuf, _, a2a = h
        self._a2a_wait(a2a)
        self.eng.unpack(kind, t, self.recv_rows, rbuf, accumulate=False)

    def reverse_start(self, kind, t):
        """Owner rows of buffer (kind, t) += the ghost rows peers hold: pack + start."""
        if self.rg.world == 1:
            return None
        dim = self.eng.dim(kind, t)
        sbuf = self.eng.empty(sum(self.rc), dim)
        rbuf = self.eng.empty(sum(self.sc), dim)
        self.eng.pack(kind, t, self.recv_rows, sbuf)
        return (kind, t, rbuf, sbuf, self._a2a_start(rbuf, sbuf, self.sc, self.rc))

    def reverse_finish(self, h):
        if h is None:
            return
        kind, t, rbuf, _, a2a = h
        self._a2a_wait(a2a)
        # one accumulate per peer block: unique rows inside a block, fixed order
        for p in range(self.rg.world):
            a, b = int(self.soff[p]), int(self.soff[p + 1])
            if b > a:
                self.eng.unpack(kind, t, self.send_rows[a:b], rbuf[a:b], accumulate=True)

    def forward(self, kind, t):
        self.forward_finish(self.forward_start(kind, t))

    def reverse(self, kind, t):
        self.reverse_finish(self.reverse_start(kind, t))


class LocalHalo(Halo):
    """A rank's exchanges emulated inside one process (bench.py
    --rank-emulation: one rank of a decomposition timed on one GPU): the
    packs and unpacks of the real Halo run unchanged on the rank's own rows,
    and each all_to_all is replaced by a device copy of the receive buffer's
    size from the send buffer (rows the rank does not have are left as they
    were).  The ghost VALUES are therefore not the peers': a timing rehearsal
    of one rank's compute and halo kernels, not a physics result."""

    staged = False

    def __init__(self, rg, engine, group=None):
        super().__init__(rg, engine, group)
        self.staged = False

    def _a2a_start(self, out, inp, out_splits, in_splits):
        n = min(out.shape[0], inp.shape[0])
        if n:
            out[:n].copy_(inp[:n])
        return [None, None, out]

    def forward_start(self, kind, t):
        # (world > 1 by construction: the emulated rank belongs to a grid)
        dim = self.eng.dim(kind, t)
        sbuf = self.eng.empty(sum(self.sc), dim)
        rbuf = self.eng.empty(sum(self.rc), dim)
        self.eng.pack(kind, t, self.send_rows, sbuf)
        return (kind, t, rbuf, sbuf, self._a2a_start(rbuf, sbuf, self.rc, self.sc))

    def reverse_start(self, kind, t):
        dim = self.eng.dim(kind, t)
        sbuf = self.eng.empty(sum(self.rc), dim)
        rbuf = self.eng.empty(sum(self.sc), dim)
        self.eng.pack(kind, t, self.recv_rows, sbuf)
        return (kind, t, rbuf, sbuf, self._a2a_start(rbuf, sbuf, self.sc, self.rc))

    def bytes_per_step(self, num_layers):
        """(sent, received) bytes of one evaluation's exchanges: the forward
        feature halos of layers 1..L-1, the reverse gradient halos of the same
        layers and the ghost forces"""
        s = r = 0
        for t in range(1, num_layers):
            d = self.eng.dim('x', t)
            s += sum(self.sc) * d * 4 + sum(self.rc) * d * 4      # forward + reverse
            r += sum(self.rc) * d * 4 + sum(self.sc) * d * 4
        s += sum(self.rc) * 3 * 4
        r += sum(self.sc) * 3 * 4
        return s, r


# ------------------------------------------------------------------ engines
class HipSegmentEngine:
    """libe3gnn_hip.so segment API (include/e3gnn.h) as a decomposition engine."""

    def __init__(self, model):
        self.m = model
        self.lib = model.lib
        self.ctx = model._ctx
        self.device = model.device
        self.num_layers = model.num_layers
        self._forces = None

    def _s(self):
        return self.m.stream_handle()

    def upload(self, rg):
        """Rank graph -> resident device tensors, once per neighbour-list build
        (the reference rebuilds its graph tensors per LAMMPS neighbour list,
        pair_e3gnn_parallel.cpp:258-314), so a step moves no host data."""
        dev = self.device
        t32 = lambda a: torch.as_tensor(np.asarray(a, dtype=np.int32), device=dev)
        self.n = rg.n_local + rg.n_ghost
        self.nl = rg.n_local
        self.n_ghost = rg.n_ghost
        self._in = (t32(rg.types), t32(rg.center), t32(rg.nbr),
                    torch.as_tensor(np.asarray(rg.vec, dtype=np.float32), device=dev))
        _lib.check(self.lib.e3gnn_set_interior(self.ctx, int(rg.n_interior)))

    def graph_set(self):
        """Per evaluation: CSR indices, transposed CSR, edge embedding and
        layer-0 features from the resident tensors (same work as the
        single-device e3gnn_energy_forces)."""
        ty, c, nb, v = self._in
        _lib.check(self.lib.e3gnn_graph_set(self.ctx, self.nl, self.n_ghost, int(c.numel()),
                                            ty.data_ptr(), c.data_ptr(), nb.data_ptr(),
                                            v.data_ptr(), self._s()))

    def dim(self, kind, t):
        return 3 if kind == 'force' else self.lib.e3gnn_feature_dim(self.ctx, t)

    def empty(self, n, dim):
        return torch.empty(n, dim, dtype=torch.float32, device=self.device)

    def _ptr(self, kind, t):
        if kind == 'x':
            return self.lib.e3gnn_feature_ptr(self.ctx, t)
        if kind == 'grad':
            return self.lib.e3gnn_grad_ptr(self.ctx, t)
        return self._forces.data_ptr()

    def pack(self, kind, t, idx, out):
        d = self.dim(kind, t)
        if idx.numel():
            _lib.check(self.lib.e3gnn_halo_pack(idx.data_ptr(), idx.numel(), d,
                                                self._ptr(kind, t), d, out.data_ptr(),
                                                self._s()))

    def unpack(self, kind, t, idx, src, accumulate):
        d = self.dim(kind, t)
        if idx.numel():
            _lib.check(self.lib.e3gnn_halo_unpack(idx.data_ptr(), idx.numel(), d,
                                                  src.data_ptr(), self._ptr(kind, t), d,
                                                  int(accumulate), self._s()))

    def layer_forward(self, t):
        _lib.check(self.lib.e3gnn_layer_forward(self.ctx, t, self._s()))

    def layer_forward_part(self, t, part):
        _lib.check(self.lib.e3gnn_layer_forward_part(self.ctx, t, part, self._s()))

    def layer_backward_part(self, t, part):
        _lib.check(self.lib.e3gnn_layer_backward_part(self.ctx, t, part, self._s()))

    def readout(self):
        e = torch.empty(1, device=self.device)
        ea = torch.empty(max(self.nl, 1), device=self.device)
        _lib.check(self.lib.e3gnn_readout(self.ctx, e.data_ptr(), ea.data_ptr(), self._s()))
        return e, ea[:self.nl]

    def layer_backward(self, t):
        _lib.check(self.lib.e3gnn_layer_backward(self.ctx, t, self._s()))

    def forces(self):
        self._forces = torch.empty(max(self.n, 1), 3, device=self.device)
        vir = torch.empty(6, device=self.device)
        _lib.check(self.lib.e3gnn_forces(self.ctx, self._forces.data_ptr(), vir.data_ptr(),
                                         None, self._s()))
        return self._forces, vir


# ------------------------------------------------------------------ driver
class ParallelE3GNN:
    """One energy/force/virial evaluation of a decomposed system.

    Mirrors the compute() loop of pair_e3gnn_parallel.cpp:316-519 with the
    TorchScript segments replaced by the engine's layer calls."""

    def __init__(self, engine, group=None):
        self.eng = engine
        self.group = group
        self.rg = None
        self.halo = None

    def set_graph(self, rg, emulate=False):
        """New neighbour list: handshake, halo index lists and the one-time
        upload of the rank graph; ``evaluate`` then moves no host data.
        ``emulate``: one rank of a decomposition in a single process (send
        lists from ``local_handshake``, exchanges as ``LocalHalo`` copies)."""
        if emulate:
            if rg.send_rows is None:
                raise ValueError('rank emulation: run local_handshake over all ranks first')
        elif rg.send_rows is None:
            handshake(rg, self.group, self._comm_device())
        self.rg = rg
        self.halo = (LocalHalo if emulate else Halo)(rg, self.eng, self.group)
        self.eng.upload(rg)

    def _comm_device(self):
        if dist.is_initialized() and dist.get_backend(self.group) == 'nccl':
            return self.eng.device
        return 'cpu'

    def _sync(self):
        if torch.device(self.eng.device).type == 'cuda':
            torch.cuda.synchronize(self.eng.device)

    def _exchange(self, start, finish, kind, t, timing):
        """Start an exchange (overlapped: the caller finishes it later).  With
        ``timing`` (a dict) the exchange's communication instead runs to
        completion on its own (pack + all_to_all), ranks aligned by a barrier
        and the device synchronised around it, and its wall time is added to
        timing['exchange_s'].  Either way the caller's ``finish`` does the
        unpack at the same point of the evaluation, so the result is the same
        (a reverse exchange accumulates into rows that the second part of the
        layer backward writes first)."""
        if timing is None:
            return start(kind, t)
        self._sync()
        if dist.is_initialized() and self.rg.world > 1:
            dist.barrier(group=self.group)
        t0 = time.perf_counter()
        h = start(kind, t)
        if h is not None:
            Halo._a2a_wait(h[4])
        self._sync()
        timing['exchange_s'] = timing.get('exchange_s', 0.0) + time.perf_counter() - t0
        timing['exchanges'] = timing.get('exchanges', 0) + 1
        return h

    def evaluate(self, timing=None):
        """One evaluation.  ``timing``: a dict to fill with the wall time of
        the halo exchanges run serially (no overlap; see ``_exchange``) and of
        the whole evaluation, so compute = total - exchange."""
        eng, halo, L = self.eng, self.halo, self.eng.num_layers
        t_begin = time.perf_counter()
        eng.graph_set()
        for t in range(L):
            if t > 0:
                # forward_comm of the layer-t features, overlapped with the
                # owned rows' work (interior centres)
                h = self._exchange(halo.forward_start, halo.forward_finish, 'x', t, timing)
                eng.layer_forward_part(t, 0)
                halo.forward_finish(h)
                eng.layer_forward_part(t, 1)
            else:
                eng.layer_forward(t)
        e_local, atomic = eng.readout()
        for t in reversed(range(L)):
            if t > 0:
                # ghost rows of dE/dx first, their reverse_comm overlapped with
                # the interior centres and owned rows
                eng.layer_backward_part(t, 0)
                h = self._exchange(halo.reverse_start, halo.reverse_finish, 'grad', t, timing)
                eng.layer_backward_part(t, 1)
                halo.reverse_finish(h)
            else:
                eng.layer_backward(t)
        forces, vir = eng.forces()
        # ghost forces -> owners (newton on)
        halo.reverse_finish(self._exchange(halo.reverse_start, halo.reverse_finish, 'force', 0,
                                           timing))
        tot = torch.cat([e_local.reshape(1), vir.reshape(6)]).to(torch.float64)
        if dist.is_initialized() and self.rg.world > 1:
            if self._comm_device() == 'cpu' and tot.device.type != 'cpu':
                h = tot.cpu()
                dist.all_reduce(h, group=self.group)
                tot = h.to(tot.device)
            else:
                dist.all_reduce(tot, group=self.group)
        if timing is not None:
            self._sync()
            timing['total_s'] = time.perf_counter() - t_begin
        nl = self.rg.n_local
        return {'energy': tot[0], 'virial': tot[1:7], 'forces': forces[:nl],
                'atomic_energy': atomic, 'owned': self.rg.owned}


def gather_all(res, n_atoms, group=None, device='cpu'):
    """Global forces / atomic energies on every rank (tests and tools only;
    ``device``: where the all_reduce runs, the GPU for backend "nccl")."""
    f = torch.zeros(n_atoms, 3, dtype=torch.float64, device=device)
    ea = torch.zeros(n_atoms, dtype=torch.float64, device=device)
    idx = torch.as_tensor(res['owned'], dtype=torch.int64, device=device)
    f[idx] = res['forces'].detach().to(device, torch.float64)
    ea[idx] = res['atomic_energy'].detach().to(device, torch.float64)
    if dist.is_initialized():
        dist.all_reduce(f, group=group)
        dist.all_reduce(ea, group=group)
    return f.cpu(), ea.cpu()
