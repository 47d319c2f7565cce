"""CPU segment engine for the decomposition tests (TEST INFRASTRUCTURE).

Implements the per-rank segment interface that ``parallel.ParallelE3GNN``
drives (graph_set / layer_forward / readout / layer_backward / forces +
pack/unpack of the 'x', 'grad' and 'force' buffers), computing each
interaction block with the oracle's functions (oracle/sevennet_ref.py, which
follows sevenn/nn/*) and the backward with torch autograd.  It lets the
world_size>1 gloo tests check the decomposition (ownership, ghosts, halo
exchanges, reverse accumulation, reductions) on CPU against the single-process
oracle.  Never used by the product path.
"""
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from oracle.sevennet_ref import SevenNet0Ref, e3nn_linear, irreps_dim, spherical_harmonics_l2  # noqa: E402


class CpuSegmentEngine:
    device = 'cpu'

    def __init__(self, dtype=torch.float64):
        self.ref = SevenNet0Ref(dtype=dtype)
        self.dtype = dtype
        self.num_layers = self.ref.nlayer

    # -- graph
    uploads = 0

    def upload(self, rg):
        self.uploads += 1
        self.nl, self.n = rg.n_local, rg.n_local + rg.n_ghost
        self.center = torch.as_tensor(rg.center, dtype=torch.int64)
        self.nbr = torch.as_tensor(rg.nbr, dtype=torch.int64)
        self._vec = torch.as_tensor(rg.vec, dtype=self.dtype).clone()
        self._types = torch.as_tensor(rg.types, dtype=torch.int64)

    def graph_set(self):
        r = self.ref
        self.vec = self._vec.clone().requires_grad_(True)
        self.emb = r.edge_embedding(self.vec.norm(dim=-1))
        self.sh = spherical_harmonics_l2(self.vec)
        nsp = len(r.symbols)
        onehot = torch.nn.functional.one_hot(self._types, nsp).to(self.dtype)
        x0 = (onehot @ r.t('onehot_to_feature_x.linear.weight').reshape(nsp, -1)) / math.sqrt(nsp)
        self.x = {0: x0.detach()}
        self.out = {}
        self.grad = {}
        self.dvec = torch.zeros_like(self.vec)

    def dim(self, kind, t):
        return 3 if kind == 'force' else irreps_dim(self.ref.irreps[t])

    def empty(self, n, dim):
        return torch.empty(n, dim, dtype=self.dtype)

    def _buf(self, kind, t):
        return {'x': lambda: self.x[t], 'grad': lambda: self.grad[t],
                'force': lambda: self.F}[kind]()

    def pack(self, kind, t, idx, out):
        out.copy_(self._buf(kind, t).detach()[idx.long()])

    def unpack(self, kind, t, idx, src, accumulate):
        b = self._buf(kind, t)
        with torch.no_grad():
            if accumulate:
                b[idx.long()] += src
            else:
                b[idx.long()] = src

    # -- blocks (oracle energy() loop body, sevenn/nn via oracle/sevennet_ref.py)
    def layer_forward(self, t):
        r, nl = self.ref, self.nl
        x = self.x[t]
        if t > 0:
            x = x.detach().requires_grad_(True)
            self.x[t] = x
        irr_x, irr_out = r.irreps[t], r.irreps[t + 1]
        last = t == r.nlayer - 1
        gin, _, _ = r.gate_irreps(irr_out)
        sc = e3nn_linear(x[:nl], irr_x, gin, r.p[f'{t}_self_connection_intro.linear.weight'])
        h = e3nn_linear(x, irr_x, irr_x, r.p[f'{t}_self_interaction_1.linear.weight'])
        agg, mid = r.convolution(t, h, self.emb, self.sh, self.nbr, self.center, irr_x,
                                 0 if last else 2)
        y = e3nn_linear(agg[:nl], mid, gin, r.p[f'{t}_self_interaction_2.linear.weight']) + sc
        out = r.gate(y, irr_out)
        self.out[t] = out
        nxt = torch.zeros(self.n, out.shape[1], dtype=self.dtype)
        nxt[:nl] = out.detach()
        self.x[t + 1] = nxt

    # halo-overlap parts: the oracle engine computes a block in one go (part 1
    # of the forward, part 0 of the backward), which keeps the driver's data
    # dependencies (ghost rows needed by forward part 1, produced by backward
    # part 0)
    def layer_forward_part(self, t, part):
        if part == 1:
            self.layer_forward(t)

    def layer_backward_part(self, t, part):
        if part == 0:
            self.layer_backward(t)

    def readout(self):
        r, nl, L = self.ref, self.nl, self.num_layers
        xl = self.x[L].detach().requires_grad_(True)
        self.x[L] = xl
        x = xl[:nl]
        hid = e3nn_linear(x, r.irreps[-1], [(x.shape[1] // 2, 0)],
                          r.p['reduce_input_to_hidden.linear.weight'])
        e_s = e3nn_linear(hid, [(hid.shape[1], 0)], [(1, 0)],
                          r.p['reduce_hidden_to_energy.linear.weight'])
        ty = self._types_local
        atomic = e_s[:, 0] * r.t('rescale_atomic_energy.scale')[ty] + \
            r.t('rescale_atomic_energy.shift')[ty]
        e = atomic.sum()
        (g,) = torch.autograd.grad(e, xl)
        self.grad[L] = g.clone()
        return e.detach().reshape(1), atomic.detach()

    def layer_backward(self, t):
        gout = self.grad[t + 1][:self.nl]
        ins = [self.x[t], self.vec] if t > 0 else [self.vec]
        gs = torch.autograd.grad(self.out[t], ins, grad_outputs=gout, allow_unused=True,
                                 retain_graph=True)
        if t > 0:
            self.grad[t] = gs[0].clone() if gs[0] is not None else torch.zeros_like(self.x[t])
        if gs[-1] is not None:
            self.dvec += gs[-1]

    def forces(self):
        g, v = self.dvec, self.vec.detach()
        F = torch.zeros(self.n, 3, dtype=self.dtype)
        F.index_add_(0, self.center, g)
        F.index_add_(0, self.nbr, -g)
        self.F = F
        vir = -torch.stack([(v[:, 0] * g[:, 0]).sum(), (v[:, 1] * g[:, 1]).sum(),
                            (v[:, 2] * g[:, 2]).sum(),
                            0.5 * (v[:, 0] * g[:, 1] + v[:, 1] * g[:, 0]).sum(),
                            0.5 * (v[:, 1] * g[:, 2] + v[:, 2] * g[:, 1]).sum(),
                            0.5 * (v[:, 0] * g[:, 2] + v[:, 2] * g[:, 0]).sum()])
        return F, vir


def make_engine(rg, dtype=torch.float64):
    eng = CpuSegmentEngine(dtype)
    eng._types_local = torch.as_tensor(rg.types[:rg.n_local], dtype=torch.int64)
    return eng
