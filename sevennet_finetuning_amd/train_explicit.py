"""Hand-scheduled derivatives of the fine-tune step (SURVEY.md §8f row 1,
BASELINE config 5) -- no autograd graph over the model.

The reference trains with a force loss: ``ForceStressOutputFromEdge`` takes
F = -dE/dr with ``create_graph=True`` (force_output.py:158-215) and the
trainer back-propagates the loss through that graph (trainer.py:155-222), a
second-order derivative that PyTorch's autograd expands into thousands of
small kernels (the step is launch-bound at the reference's batch sizes).
Here the same gradient is written out by hand:

  1. primal forward, intermediates kept (SevenNetTrainable.forward's math);
  2. first reverse (seed dE/d atomic = 1): f_e = dE/dr_e per edge, then
     forces F and stress S from the edges, as the reference does;
  3. the loss on (E, F, S) as leaves (the reference's loss definitions,
     autograd over a few small tensors) gives cE = dL/dE, cF, cS, hence the
     per-edge cotangent v_e = dL/df_e;
  4. since  dL/dtheta = sum_g cE_g dE_g/dtheta + d/dtheta <v, dE/dr>  and
     <v, dE/dr> is the directional derivative of E along v, a TANGENT forward
     along v (every activation q gets q' = dq/d eps, r -> r + eps v) followed
     by ONE reverse sweep over the primal+tangent pairs, seeded with cE on E
     and 1 on E', gives the parameter gradient (reverse-over-forward).

Every bilinear piece has a closed form: linears (e3nn Linear as dense
matrices, y' = x' W), the scaled-SiLU chain (phi, phi', phi''), the gate
(J y', J^T x, and the second-order term d/dy <x'bar, J(y) y'>), the edge
basis / spherical harmonics, and the convolution agg = C(h, Y, w), which is
trilinear: its tangent is C(h', Y, w) + C(h, Y', w) + C(h, Y, w') and its
dual reverse four conv backward launches (ExplicitStep.backward).  The conv
launches are the library's (e3gnn_conv_forward / _backward), the element-wise
pieces the HIP kernels of train_ops.hip on the GPU (torch on the CPU, where
the tests compare this module in float64 with autograd of the trainable
model).

Scope: SevenNet-0's architecture (nn.sevennet0_kinds, linear
self-connection, XPLOR cutoff, normalised or raw SH, silu gates); other
members of the family keep the autograd path.
"""
import ctypes
import math
import os

import numpy as np
import torch

from . import _keys as KEY
from . import conv_ops
from .conv_ops import ACC_DH, ACC_DW, ACC_DY


def supported(model):
    """True when the explicit derivatives cover this trainable model."""
    from .nn import sevennet0_kinds
    if sevennet0_kinds(model.manifest, conv_only=True) is None:
        return False
    # the explicit step drives the specialised SevenNet-0 kernels (out= / acc=
    # conv launches, the fused tangent forward and dual backward); a model on
    # the runtime-table backend keeps the autograd path
    if getattr(getattr(model, 'conv_backend', None), 'generic', False):
        return False
    if model.sc_type != 'linear' or model.cut.get('name', 'XPLOR') != 'XPLOR':
        return False
    # linear biases / the FCN readout: the autograd path (their derivatives
    # are not in the hand-scheduled sweep)
    if getattr(model, 'use_bias', False) or model.readout_cfg.get('type', 'linear') != 'linear':
        return False
    if model.lmax_edge != 2 or model.filter_parity != 1:
        return False
    for blk in model.blocks:
        _, scal, gated, (gate_p, _, natural) = blk['gate']
        if not natural or gate_p != 1 or any(t[2] != 1 for t in scal) or len(gated) > 2:
            return False
    return True


# ------------------------------------------------------------------ primitives
class _Prims:
    """Element-wise primitives: the HIP kernels of train_ops.hip for float32
    device tensors, torch formulas otherwise (CPU tests, float64)."""

    def __init__(self, model):
        self.c = float(model.silu_norm)
        self.lib = model._act_lib() if model.flat.is_cuda else None

    def _hip(self, x):
        return self.lib is not None and x.is_cuda and x.dtype == torch.float32

    # scaled SiLU: phi = c x s, phi' = c s (1 + x (1 - s)), phi'' = c s (1 - s) (2 + x (1 - 2 s))
    def _d(self, x):
        s = torch.sigmoid(x)
        d1 = self.c * s * (1 + x * (1 - s))
        d2 = self.c * s * (1 - s) * (2 + x * (1 - 2 * s))
        return d1, d2

    def act(self, x, out=None):
        if self._hip(x):
            y = torch.empty_like(x) if out is None else out
            conv_ops._act_call(self.lib, 0, x, out0=y, scale=self.c)
            return y
        return _put(out, self.c * x * torch.sigmoid(x))

    def act_jvp(self, x, xd, out=None):
        """phi'(x) x'"""
        if self._hip(x):
            y = torch.empty_like(x) if out is None else out
            conv_ops._act_call(self.lib, 1, x, g=xd.contiguous(), out0=y, scale=self.c)
            return y
        return _put(out, self._d(x)[0] * xd)

    def act_dual(self, x, xd, g, gd, out0=None, out1=None):
        """reverse of (phi(x), phi'(x) x'): (g phi' + g' phi'' x', g' phi')"""
        if self._hip(x):
            o0 = torch.empty_like(x) if out0 is None else out0
            o1 = torch.empty_like(x) if out1 is None else out1
            conv_ops._act_dual_call(self.lib, x, xd, g, gd, o0, o1, self.c)
            return o0, o1
        d1, d2 = self._d(x)
        return _put(out0, g * d1 + gd * d2 * xd), _put(out1, gd * d1)


class _Gemms:
    """Dense products of the step, ``C = beta C + alpha (A B [+ A2 B2])``, on the
    library's grouped matrix-core GEMM (e3gnn_gemm_grouped, csrc/tgemm.hip) for
    float32 device tensors -- independent products queued with ``add`` go out as
    ONE launch (plus one fixed-order split-K reduction) at ``flush`` -- and as
    torch GEMMs otherwise (CPU tests, float64).  Operands are 2-D views; a
    transposed view (``W.t()``) is passed as op(X) = X^T of its storage."""

    def __init__(self, model):
        # E3GNN_TRAIN_TGEMM=0: torch's GEMMs (A/B)
        on = model.flat.is_cuda and os.environ.get('E3GNN_TRAIN_TGEMM', '1') != '0'
        self.lib = model._act_lib() if on else None
        self.q = []
        self.ws = None
        self.max_probs = 12        # e3gnn_gemm_grouped's problems per launch
        # deferred split-K reductions (begin_defer .. finish_defer): the
        # slabs of every flush in their own workspace region, all reduced
        # by one e3gnn_gemm_reduce launch
        self.defer = None
        self.dws = []              # workspace chunks (one after the first step)
        self.dws_total = 0
        # a captured HIP graph keeps the raw addresses of the workspaces it
        # used: a buffer replaced by a larger one stays allocated for the
        # lifetime of this object (and so of every graph that captured it)
        self.retired = []

    def _hip(self, *ts):
        return self.lib is not None and all(t.is_cuda and t.dtype == torch.float32 for t in ts)

    @staticmethod
    def _op(x):
        """(ptr, ld, trans) of a 2-D view (r x k): row-major storage X[r][ld]
        (trans 0) or a transposed view of X[k][ld] (trans 1)"""
        r, k = x.shape
        s0, s1 = x.stride()
        if s1 == 1 or k == 1:
            return x.data_ptr(), (s0 if r > 1 else max(k, 1)), 0
        if s0 == 1 or r == 1:
            return x.data_ptr(), (s1 if k > 1 else max(r, 1)), 1
        return None

    # the library's GEMM reads each operand through one buffer descriptor with
    # 32-bit byte offsets (csrc/tgemm.hip TG_RECORDS): larger operands take
    # the torch path (e3gnn_gemm_grouped refuses them with E3GNN_ERR_ARG)
    MAX_OPERAND_BYTES = 0x7fff0000

    @classmethod
    def _fits(cls, *ts):
        for t in ts:
            if t is None:
                continue
            if any(st < 0 for st in t.stride()):
                return False
            span = 1 + sum((n - 1) * st for n, st in zip(t.shape, t.stride()) if n > 0)
            if span * t.element_size() > cls.MAX_OPERAND_BYTES:
                return False
        return True

    def add(self, C, A, B, alpha=1.0, beta=0, A2=None, B2=None, kr=None, wgrad=False):
        """kr: (int32 device tensor, row-tile stride) of per-tile k ranges (the
        dense matrices' block sparsity, e3gnn_gemm_desc::krange) or None;
        wgrad: C is a weight gradient read only after finish_defer (its split-K
        reduction may be deferred)"""
        if not self._hip(C, A, B, *(t for t in (A2, B2) if t is not None)) or \
                not self._fits(A, B, A2, B2):
            self.flush()   # (queued problems may produce this one's operands)
            # straight into C (no temporaries / copy kernels)
            torch.addmm(C, A, B, beta=1 if beta else 0, alpha=alpha, out=C)
            if A2 is not None:
                C.addmm_(A2, B2, alpha=alpha)
            return C
        ops = [self._op(A), self._op(B)] + ([self._op(A2), self._op(B2)] if A2 is not None else [])
        if any(o is None for o in ops) or C.stride(1) != 1:
            A, B = A.contiguous(), B.contiguous()
            A2 = A2.contiguous() if A2 is not None else None
            B2 = B2.contiguous() if B2 is not None else None
            ops = [self._op(A), self._op(B)] + ([self._op(A2), self._op(B2)] if A2 is not None else [])
            if C.stride(1) != 1:
                raise ValueError('GEMM output must be row-major')
        from . import _lib
        d = _lib.GemmDesc()
        d.a, d.lda, d.trans_a = ops[0]
        d.b, d.ldb, d.trans_b = ops[1]
        if A2 is not None:
            d.a2, d.lda2, d.trans_a2 = ops[2]
            d.b2, d.ldb2, d.trans_b2 = ops[3]
            d.k2 = int(A2.shape[1])
        d.c, d.ldc = C.data_ptr(), C.stride(0)
        d.m, d.n, d.k = int(C.shape[0]), int(C.shape[1]), int(A.shape[1])
        d.alpha, d.beta = float(alpha), int(bool(beta))
        if kr is not None:
            d.krange, d.krange_stride_m = kr[0].data_ptr(), kr[1]
        self._push(d, (C, A, B, A2, B2, kr), C.device, (C, A, B, A2, B2, float(alpha), int(bool(beta))),
                   wgrad)
        return C

    def add_lay(self, M, N, K, C, A, B, lay, A2=None, B2=None, K2=0, alpha=1.0, beta=0, wgrad=False):
        """one problem in the general layouts (e3gnn_gemm_layouts ``lay``); C, A,
        B, A2, B2 = (tensor, element offset) of the operand bases"""
        from . import _lib
        L = [(A, lay.a, M, K), (B, lay.b, N, K)] + ([(A2, lay.a2, M, K2), (B2, lay.b2, N, K2)] if K2 else [])
        if self.lib is None or not all(self._lay_fits(t[0], t[1], g, r, k) for t, g, r, k in L):
            self.flush()
            self._lay_torch(M, N, K, C, A, B, lay, A2, B2, K2, alpha, beta)
            return
        d = _lib.GemmDesc()
        ptr = lambda t: t[0].data_ptr() + 4 * t[1]   # noqa: E731 (float32)
        d.a, d.b, d.c = ptr(A), ptr(B), ptr(C)
        if K2:
            d.a2, d.b2 = ptr(A2), ptr(B2)
        d.m, d.n, d.k, d.k2 = int(M), int(N), int(K), int(K2)
        d.alpha, d.beta = float(alpha), int(bool(beta))
        d.layout = ctypes.addressof(lay)
        self._push(d, (C[0], A[0], B[0], A2, B2, lay), C[0].device, None, wgrad)

    @classmethod
    def _lay_fits(cls, x, off, g, rows, K):
        """largest byte offset of operand layout g (e3gnn_gemm_layout) over
        rows x K elements from element `off` of x, within one descriptor"""
        if rows <= 0 or K <= 0:
            return True
        if min(g.ld, g.kst, g.sst, g.rs) < 0 or max(g.ld, g.kst, g.sst) > 0x7fffffff:
            return False
        rep, ks = max(g.rep, 1), g.ks if g.ks > 0 else K
        top = ((rows - 1) // rep * g.ld + min(rows - 1, rep - 1) * g.rs + min(K - 1, ks - 1) * g.kst
               + (K - 1) // ks * g.sst)
        return (top + 1) * x.element_size() <= cls.MAX_OPERAND_BYTES

    @staticmethod
    def _lay_view(x, off, g, rows, K):
        """the (rows x K) operand of layout g as a torch view: element (i, k)
        at (i / rep) ld + (i % rep) rs + (k % ks) kst + (k / ks) sst"""
        rep, ks = max(g.rep, 1), g.ks if g.ks > 0 else K
        assert rows % rep == 0 and K % ks == 0
        v = x.as_strided((rows // rep, rep, K // ks, ks), (g.ld, g.rs, g.sst, g.kst), x.storage_offset() + off)
        return v.reshape(rows, K)

    def _lay_torch(self, M, N, K, C, A, B, lay, A2, B2, K2, alpha, beta):
        """add_lay's problem with torch GEMMs (operands the library's 32-bit
        descriptors cannot address, or no library): same sums, written into
        C's layout"""
        prod = self._lay_view(*A, lay.a, M, K) @ self._lay_view(*B, lay.b, N, K).t()
        if K2:
            prod = prod + self._lay_view(*A2, lay.a2, M, K2) @ self._lay_view(*B2, lay.b2, N, K2).t()
        Ct, co = C
        crep = max(lay.crep, 1)
        cv = Ct.as_strided((M // crep, crep, N), (lay.ldc, lay.crs, lay.cns), Ct.storage_offset() + co)
        prod = (alpha * prod).view(M // crep, crep, N)
        if beta:
            cv.add_(prod)
        else:
            cv.copy_(prod)

    def _push(self, d, keep, dev, info, wgrad=False):
        if len(self.q) == self.max_probs:
            self.flush()
        self.q.append((d, keep, dev, info, wgrad))

    def flush(self):
        if not self.q:
            return
        from . import _lib
        n = len(self.q)
        descs = (_lib.GemmDesc * n)(*[e[0] for e in self.q])
        need = int(self.lib.e3gnn_gemm_workspace_floats(n, descs))
        dev = self.q[0][2]
        stream = torch.cuda.current_stream(dev).cuda_stream
        split = [int(self.lib.e3gnn_gemm_workspace_floats(1, ctypes.byref(descs[i]))) for i in range(n)]
        # deferred only when every split problem of the launch is a weight
        # gradient (any other output is read by the next launches)
        if self.defer is not None and need > 0 and all(e[4] for e, w in zip(self.q, split) if w > 0):
            base = self._dws_take(need, dev)
            _lib.check(self.lib.e3gnn_gemm_grouped_ex(n, descs, base, need, 1, stream))
            off = 0
            for i, (e, w) in enumerate(zip(self.q, split)):
                if w > 0:
                    self.defer.append((descs[i], e[1], base + 4 * off))
                off += w
            self.q = []
            return
        if need > 0 and (self.ws is None or self.ws.numel() < need):
            if self.ws is not None:
                self.retired.append(self.ws)
            self.ws = torch.empty(max(need, 1 << 20), device=dev)
        ws = self.ws.data_ptr() if self.ws is not None else None
        _lib.check(self.lib.e3gnn_gemm_grouped(n, descs, ws, self.ws.numel() if self.ws is not None else 0,
                                               stream))
        self.q = []

    def _dws_take(self, need, dev):
        """the device address of `need` floats of deferred workspace (a new
        chunk when the current one is full; one chunk of the whole step's
        size from the next begin_defer on)"""
        buf, used = self.dws[-1] if self.dws else (None, 0)
        if buf is None or used + need > buf.numel():
            buf, used = torch.empty(max(need, self.dws_total, 1 << 20), device=dev), 0
            self.dws.append([buf, 0])
        self.dws[-1][1] = used + need
        return buf.data_ptr() + 4 * used

    def begin_defer(self):
        if self.lib is None:
            return
        self.flush()
        if len(self.dws) > 1:     # last step needed several chunks: one of the total
            self.dws_total = sum(u for _, u in self.dws)
            self.retired.extend(b for b, _ in self.dws)
            self.dws = []
        for c in self.dws:
            c[1] = 0
        self.defer = []

    def finish_defer(self):
        """the deferred split-K reductions, one launch (per 32 problems)"""
        if self.defer is None:
            return
        self.flush()
        pend, self.defer = self.defer, None
        if not pend:
            return
        from . import _lib
        n = len(pend)
        descs = (_lib.GemmDesc * n)(*[p[0] for p in pend])
        wss = (ctypes.c_void_p * n)(*[p[2] for p in pend])
        dev = pend[0][1][0].device
        _lib.check(self.lib.e3gnn_gemm_reduce(n, descs, wss, torch.cuda.current_stream(dev).cuda_stream))


def _put(out, v):
    if out is None:
        return v
    out.copy_(v)
    return out


_ONES = {}


def _wgrad(G, A, B, alpha=1.0):
    """G += alpha A^T B for a tall K (edges) and a small output: split over
    K-chunks as one batched GEMM and a sum (a single GEMM with K = 24k rows
    and a 64 x 64 output runs on 4 workgroups)"""
    K = A.shape[0]
    if K < 2048 or A.shape[1] * B.shape[1] > (1 << 17):
        G.addmm_(A.t(), B, alpha=alpha)
        return
    S = next((s for s in range(K // 384, 7, -1) if K % s == 0), 1)
    if S <= 1:
        G.addmm_(A.t(), B, alpha=alpha)
        return
    part = torch.bmm(A.view(S, K // S, -1).transpose(1, 2), B.view(S, K // S, -1))
    # the S partial products summed into G by one GEMM (ones[1, S] @ part)
    ones = _ONES.get((S, part.dtype, part.device))
    if ones is None:
        ones = _ONES[(S, part.dtype, part.device)] = torch.ones(1, S, dtype=part.dtype,
                                                                device=part.device)
    G.view(1, -1).addmm_(ones, part.view(S, -1), alpha=alpha)


class _Gate:
    """e3nn Gate of a block in the natural layout [s | g | gated_k], silu
    (scaled) on scalars and gates: x = [phi(s) | phi(g_k) b_k]."""

    def __init__(self, gate_irreps, prims):
        _, scal, gated, _ = gate_irreps
        self.ns = sum(t[0] for t in scal)
        self.ng = sum(t[0] for t in gated)
        self.gated = [(t[0], 2 * t[1] + 1) for t in gated]
        self.p = prims
        self.dims = conv_ops.gate_dims([t[:2] for t in scal], [t[:2] for t in gated]) if self.ng \
            else None

    def _split(self, y):
        s = y[:, :self.ns]
        g = y[:, self.ns:self.ns + self.ng]
        blks, off = [], self.ns + self.ng
        for m, d in self.gated:
            blks.append(y[:, off:off + m * d].reshape(-1, m, d))
            off += m * d
        return s, g, blks

    def _gsplit(self, g):
        return g.split([m for m, _ in self.gated], dim=1) if len(self.gated) > 1 else (g,)

    def _xsplit(self, x):
        # output row [s | blocks]
        out, off = [x[:, :self.ns]], self.ns
        for m, d in self.gated:
            out.append(x[:, off:off + m * d].reshape(-1, m, d))
            off += m * d
        return out

    def fwd(self, y, out=None):
        p = self.p
        if not self.ng:
            return p.act(y, out)
        if p._hip(y):
            o = torch.empty(y.shape[0], int(self.dims[3]), device=y.device) if out is None else out
            conv_ops._gate_call(p.lib, 0, self.dims, y.contiguous(), out0=o, scale=p.c)
            return o
        s, g, blks = self._split(y)
        ga = self._gsplit(p.act(g))
        outs = [p.act(s)] + [(a.unsqueeze(-1) * b).reshape(y.shape[0], -1) for a, b in zip(ga, blks)]
        return _put(out, torch.cat(outs, 1))

    def vjp(self, y, xb):
        """J^T x-bar"""
        p = self.p
        if not self.ng:
            return p.act_jvp(y, xb)
        if p._hip(y):
            o = torch.empty_like(y)
            conv_ops._gate_call(p.lib, 1, self.dims, y.contiguous(), go=xb.contiguous(), out0=o,
                                scale=p.c)
            return o
        s, g, blks = self._split(y)
        xs = self._xsplit(xb)
        d1g = p._d(g)[0]
        ga = self._gsplit(p.act(g))
        gds = self._gsplit(d1g)
        out = [p.act_jvp(s, xs[0])]
        gbar = [gd * (xk * b).sum(-1) for gd, xk, b in zip(gds, xs[1:], blks)]
        out += gbar
        out += [(a.unsqueeze(-1) * xk).reshape(y.shape[0], -1) for a, xk in zip(ga, xs[1:])]
        return torch.cat(out, 1)

    def jvp(self, y, yd, out=None):
        """J y'"""
        p = self.p
        if not self.ng:
            return p.act_jvp(y, yd, out)
        if p._hip(y):
            o = torch.empty(y.shape[0], int(self.dims[3]), device=y.device) if out is None else out
            conv_ops._gate_dual_call(p.lib, 0, self.dims, y, yd, out0=o, scale=p.c)
            return o
        s, g, blks = self._split(y)
        sd, gd, bds = self._split(yd)
        ga = self._gsplit(p.act(g))
        gjv = self._gsplit(p.act_jvp(g, gd))
        outs = [p.act_jvp(s, sd)]
        for a, aj, b, bd in zip(ga, gjv, blks, bds):
            outs.append((aj.unsqueeze(-1) * b + a.unsqueeze(-1) * bd).reshape(y.shape[0], -1))
        return _put(out, torch.cat(outs, 1))

    def dual_vjp(self, y, yd, xb, xbd, out0=None, out1=None):
        """reverse of (x, x') = (G(y), J(y) y'):
        y-bar = J^T x-bar + d/dy <x'-bar, J(y) y'>,  y'-bar = J^T x'-bar"""
        p = self.p
        if not self.ng:
            return p.act_dual(y, yd, xb, xbd, out0, out1)
        if p._hip(y):
            yb = torch.empty_like(y) if out0 is None else out0
            ydb = torch.empty_like(y) if out1 is None else out1
            conv_ops._gate_dual_call(p.lib, 1, self.dims, y, yd, xb, xbd, out0=yb, out1=ydb,
                                     scale=p.c)
            return yb, ydb
        yb = self.vjp(y, xb)
        ydb = self.vjp(y, xbd)
        # second-order term
        s, g, blks = self._split(y)
        sd, gd, bds = self._split(yd)
        xs = self._xsplit(xbd)
        d1s, d2s = p._d(s)
        d1g, d2g = p._d(g)
        out = [xs[0] * d2s * sd]
        d1gs, d2gs, gds = self._gsplit(d1g), self._gsplit(d2g), self._gsplit(gd)
        gpart, bpart = [], []
        for d1, d2, gdk, xk, b, bd in zip(d1gs, d2gs, gds, xs[1:], blks, bds):
            gpart.append(d2 * gdk * (xk * b).sum(-1) + d1 * (xk * bd).sum(-1))
            bpart.append((xk * (d1 * gdk).unsqueeze(-1)).reshape(y.shape[0], -1))
        h = torch.cat(out + gpart + bpart, 1)
        return _put(out0, yb + h), _put(out1, ydb)


# ------------------------------------------------------------------ edge geometry
class _Geometry:
    """r, u, Y = SH(u) (e3nn 'component', lmax 2, of the unit or raw vector;
    nn.spherical_harmonics) and emb = Bessel(r) * XPLOR(r) (nn._edge_basis),
    with the tangent along a direction v and the transposes the reverse
    sweeps need."""

    def __init__(self, model, prims):
        from .nn import _sh_map
        self.rc = float(model.cutoff)
        self.ron = float(model.r_on)
        self.normalize = bool(model.sh_normalize)
        self._map = lambda dev, dt: _sh_map(2, dev, dt)   # noqa: E731
        self.lib = prims.lib   # float32 device tensors: the HIP kernels (e3gnn_edge_geometry*)

    def _hip(self, vec):
        return self.lib is not None and vec.is_cuda and vec.dtype == torch.float32

    def _args(self, g):
        return (g['E'], g['vec'].data_ptr(), g['coeffs'].data_ptr(), self.rc, self.ron)

    @staticmethod
    def _stream(t):
        return torch.cuda.current_stream(t.device).cuda_stream

    def _env(self, r):
        rc2, ron2 = self.rc * self.rc, self.ron * self.ron
        d3 = (rc2 - ron2) ** 3
        s = torch.clamp(r * r, min=ron2)
        env = (rc2 - s) ** 2 * (2.0 * s + (rc2 - 3.0 * ron2)) / d3
        # d env / dr = 6 (rc2 - s)(ron2 - s) / d3 * ds/dr, ds/dr = 2r above r_on, 0 below
        denv = torch.where(r * r > ron2, 12.0 * r * (rc2 - s) * (ron2 - s) / d3, torch.zeros_like(r))
        return env, denv

    def forward(self, vec, coeffs, emb_out=None):
        if self._hip(vec):
            from . import _lib
            vec, coeffs = vec.contiguous(), coeffs.contiguous()
            E = int(vec.shape[0])
            Y = torch.empty(E, 9, device=vec.device)
            emb = torch.empty(E, 8, device=vec.device) if emb_out is None else emb_out
            g = {'E': E, 'vec': vec, 'coeffs': coeffs, 'Y': Y, 'emb': emb}
            _lib.check(self.lib.e3gnn_edge_geometry(*self._args(g), int(not self.normalize),
                                                    Y.data_ptr(), emb.data_ptr(), self._stream(vec)))
            return g
        g = self._forward_torch(vec, coeffs)
        if emb_out is not None:
            emb_out.copy_(g['emb'])
        return g

    def _forward_torch(self, vec, coeffs):
        r = torch.linalg.norm(vec, dim=-1)
        u = vec / r.unsqueeze(-1) if self.normalize else vec
        mono = torch.cat([torch.ones_like(u[:, :1]), u, (u.unsqueeze(-1) * u.unsqueeze(-2)).reshape(-1, 9)], 1)
        Y = mono @ self._map(vec.device, vec.dtype)
        env, denv = self._env(r)
        cr = coeffs * r.unsqueeze(-1)
        sn, cs = torch.sin(cr), torch.cos(cr)
        k = 2.0 / self.rc
        ur = r.unsqueeze(-1)
        b = k * sn / ur
        emb = b * env.unsqueeze(-1)
        # d emb / dr
        db = k * (coeffs * cs * ur - sn) / (ur * ur)
        demb = db * env.unsqueeze(-1) + b * denv.unsqueeze(-1)
        return {'r': r, 'u': u, 'Y': Y, 'emb': emb, 'demb': demb, 'env': env, 'denv': denv,
                'sn': sn, 'cs': cs, 'E': int(vec.shape[0]), 'vec': vec, 'coeffs': coeffs}

    def sh_vjp_u(self, G, u):
        """dE/du from dE/dY"""
        gm = G @ self._map(G.device, G.dtype).t()          # E x 13 (monomials)
        q = gm[:, 4:].reshape(-1, 3, 3)
        return gm[:, 1:4] + ((q + q.transpose(1, 2)) @ u.unsqueeze(-1)).squeeze(-1)

    def vjp(self, g, Yb, embb):
        """dE/dvec from dE/dY and dE/demb"""
        if 'u' not in g:
            from . import _lib
            fij = torch.empty(g['E'], 3, device=Yb.device)
            _lib.check(self.lib.e3gnn_edge_geometry_vjp(
                *self._args(g), int(not self.normalize), Yb.contiguous().data_ptr(),
                embb.contiguous().data_ptr(), fij.data_ptr(), self._stream(Yb)))
            return fij
        u, r = g['u'], g['r']
        ub = self.sh_vjp_u(Yb, u)
        rb = (embb * g['demb']).sum(-1)
        if self.normalize:
            uhat = u
            vb = (ub - uhat * (uhat * ub).sum(-1, keepdim=True)) / r.unsqueeze(-1)
        else:
            uhat = u / r.unsqueeze(-1)
            vb = ub
        return vb + uhat * rb.unsqueeze(-1)

    def tangent(self, g, S, cF, cS, embd_out):
        """(Y', emb' -> embd_out, r') along the loss cotangent of the edge
        forces: v_e = cF[centre] - cF[nbr] minus the stress term (forces F_i
        = sum_{centre i} f_e - sum_{nbr i} f_e, stress from the edges)"""
        center, nbr, batch = S['center'], S['nbr'], S['batch']
        if 'u' not in g:
            from . import _lib
            aux = S['graph'].aux
            E = g['E']
            Yd = torch.empty(E, 9, device=cF.device)
            rd = torch.empty(E, device=cF.device)
            cS_, vol = (cS.contiguous(), S['vol'].contiguous()) if cS is not None else (None, None)
            ptr = lambda t: t.data_ptr() if t is not None else None   # noqa: E731
            _lib.check(self.lib.e3gnn_edge_geometry_jvp(
                *self._args(g), int(not self.normalize), aux['center'].data_ptr(),
                aux['nbr'].data_ptr(), batch.contiguous().data_ptr(), cF.contiguous().data_ptr(),
                ptr(cS_), ptr(vol), Yd.data_ptr(), embd_out.data_ptr(), rd.data_ptr(),
                self._stream(cF)))
            return Yd, rd
        v = cF[center] - cF[nbr]
        if cS is not None:
            vol = S['vol']
            c = cS[batch[nbr]] / vol[batch[nbr]].unsqueeze(-1)
            r = S['vec']
            v = v - torch.stack([c[:, 0] * r[:, 0] + c[:, 5] * r[:, 2],
                                 c[:, 1] * r[:, 1] + c[:, 3] * r[:, 0],
                                 c[:, 2] * r[:, 2] + c[:, 4] * r[:, 1]], 1)
        Yd, embd, rd = self.jvp(g, v)
        embd_out.copy_(embd)
        return Yd, rd

    def jvp(self, g, v):
        """(Y', emb') along the direction v"""
        u, r = g['u'], g['r']
        uhat = u if self.normalize else u / r.unsqueeze(-1)
        rd = (uhat * v).sum(-1)
        ud = (v - uhat * rd.unsqueeze(-1)) / r.unsqueeze(-1) if self.normalize else v
        quad = (ud.unsqueeze(-1) * u.unsqueeze(-2) + u.unsqueeze(-1) * ud.unsqueeze(-2)).reshape(-1, 9)
        mono = torch.cat([torch.zeros_like(u[:, :1]), ud, quad], 1)
        Yd = mono @ self._map(v.device, v.dtype)
        embd = g['demb'] * rd.unsqueeze(-1)
        return Yd, embd, rd

    def coeff_grad(self, g, embb, embdb, rd, coeffs):
        """d/dc of <emb-bar, emb> + <emb'-bar, emb'>"""
        if 'u' not in g:
            from . import _lib
            per = torch.empty(g['E'], 8, device=embb.device)
            _lib.check(self.lib.e3gnn_edge_geometry_coeff_grad(
                *self._args(g), embb.contiguous().data_ptr(), embdb.contiguous().data_ptr(),
                rd.contiguous().data_ptr(), per.data_ptr(), self._stream(embb)))
            return per.sum(0)
        k = 2.0 / self.rc
        env, denv = g['env'].unsqueeze(-1), g['denv'].unsqueeze(-1)
        sn, cs = g['sn'], g['cs']
        de_dc = k * cs * env
        ddr_dc = k * (-coeffs * sn * env + cs * denv)
        return (embb * de_dc + embdb * ddr_dc * rd.unsqueeze(-1)).sum(0)


# ------------------------------------------------------------------ dense linears
class _DenseBank:
    """Every e3nn Linear of the model as a dense (din x dout) matrix in ONE
    buffer, built from the flat parameters with one gather / scale / scatter
    (nn._Linear's dense form), and the map back: flat_grad[u] += alpha *
    sum over the 2l+1 copies of u of the dense gradient (a padded gather and a
    row sum -- no atomics, deterministic)."""

    def __init__(self, model, entries, divisors=None):
        # entries: (key, _Linear, parameter name); divisors: key -> parameter
        # name of a scalar the whole matrix (and its gradient) is divided by
        # (a frozen convolution denominator folded into si2)
        self.model = model
        self.views = {}
        pos, src, scl, self.shapes = [], [], [], {}
        off = 0
        upos, usrc, uscl = [], [], []
        dsrc, udsrc = [], []
        self.pnames, ucount = [], []   # per entry: its parameter, its flat elements
        divisors = divisors or {}
        for key, lin, pname in entries:
            self.pnames.append(pname)
            ucount.append(sum(lin.irreps_in[i][0] * lin.irreps_out[j][0] for i, j in lin.ins))
            dv = model.slices[divisors[key]][0] if key in divisors else -1
            din, dout = lin.in_off[-1], lin.out_off[-1]
            poff = model.slices[pname][0]
            woff = 0
            for i, j in lin.ins:
                mi = lin.irreps_in[i][0]
                mo, d = lin.irreps_out[j][0], 2 * lin.irreps_in[i][1] + 1
                u, v, m = np.meshgrid(np.arange(mi), np.arange(mo), np.arange(d), indexing='ij')
                p = off + (lin.in_off[i] + u * d + m) * dout + lin.out_off[j] + v * d + m
                pos.append(p.ravel())
                src.append((poff + woff + u * mo + v).ravel())
                scl.append(np.full(u.size, lin.alpha[j]))
                dsrc.append(np.full(u.size, dv))
                # reverse map: flat element (u, v) <- its d dense positions
                pr = p.reshape(mi * mo, d)
                pad = np.full((mi * mo, 5), -1, dtype=np.int64)
                pad[:, :d] = pr
                upos.append(pad)
                usrc.append(poff + woff + np.arange(mi * mo))
                uscl.append(np.full(mi * mo, lin.alpha[j]))
                udsrc.append(np.full(mi * mo, dv))
                woff += mi * mo
            self.shapes[key] = (off, din, dout)
            off += din * dout
        self.total = off
        dev, dt = model.flat.device, model.flat.dtype
        self.pos = torch.as_tensor(np.concatenate(pos), device=dev)
        self.src = torch.as_tensor(np.concatenate(src), device=dev)
        self.scl = torch.as_tensor(np.concatenate(scl), device=dev, dtype=dt)
        up = np.concatenate(upos)
        up[up < 0] = off                    # the zero slot after the buffer
        self.upos = torch.as_tensor(up, device=dev)
        self.usrc = torch.as_tensor(np.concatenate(usrc), device=dev)
        self.uscl = torch.as_tensor(np.concatenate(uscl), device=dev, dtype=dt)
        self.uent = np.repeat(np.arange(len(entries)), ucount)   # entry of each reverse row
        self._mask_key, self._rows = None, None
        self.buf = torch.zeros(off, device=dev, dtype=dt)
        self.gbuf = torch.zeros(off + 1, device=dev, dtype=dt)
        # divisor sources: index into [flat; 1.0] (the extra slot: no divisor)
        self.div = bool(divisors)
        if self.div:
            nf = model.flat.numel()
            d, ud = np.concatenate(dsrc), np.concatenate(udsrc)
            self.dsrc = torch.as_tensor(np.where(d < 0, nf, d), device=dev)
            self.udsrc = torch.as_tensor(np.where(ud < 0, nf, ud), device=dev)
            self.flat1 = torch.ones(nf + 1, device=dev, dtype=dt)

    def _flat1(self):
        """[flat; 1.0]: the divisor table"""
        self.flat1[:-1].copy_(self.model.flat.detach())
        return self.flat1

    def build(self):
        flat = self.model.flat.detach()
        vals = flat[self.src] * self.scl
        if self.div:
            vals.div_(self._flat1()[self.dsrc])
        self.buf.index_put_((self.pos,), vals)
        return {k: self.buf[o:o + a * b].view(a, b) for k, (o, a, b) in self.shapes.items()}

    def grads(self):
        self.gbuf.zero_()
        return {k: self.gbuf[o:o + a * b].view(a, b) for k, (o, a, b) in self.shapes.items()}

    def _trainable_rows(self):
        """Reverse-map rows of the linears that require grad (None: all do).
        A frozen linear gets no gradient, as under autograd -- the flat
        gradient buffer is what the all-reduce, grad norms and the optimizer
        read.  Re-derived when a parameter's requires_grad flips."""
        key = tuple(self.model.param(n).requires_grad for n in self.pnames)
        if key != self._mask_key:
            self._mask_key = key
            keep = np.asarray(key)[self.uent]
            self._rows = None if keep.all() else torch.as_tensor(
                np.nonzero(keep)[0], device=self.usrc.device)
        return self._rows

    def flush(self, flat_grad):
        rows = self._trainable_rows()
        if rows is None:
            upos, usrc, uscl = self.upos, self.usrc, self.uscl
            udsrc = self.udsrc if self.div else None
        else:
            if rows.numel() == 0:
                return
            upos, usrc, uscl = self.upos[rows], self.usrc[rows], self.uscl[rows]
            udsrc = self.udsrc[rows] if self.div else None
        vals = self.gbuf[upos].sum(1) * uscl
        if self.div:
            vals.div_(self._flat1()[udsrc])
        flat_grad.index_add_(0, usrc, vals)


# ------------------------------------------------------------------ the step
class ExplicitStep:
    """Forces, stress and the loss gradient of one batch for a trainable
    SevenNet-0 (nn.SevenNetTrainable), accumulating dL/dtheta into
    model.flat_grad.  See the module docstring."""

    def __init__(self, model):
        if not supported(model):
            raise ValueError('the explicit fine-tune derivatives cover SevenNet-0\'s architecture only')
        self.m = model
        self.p = _Prims(model)
        self.gm = _Gemms(model)
        self.geo = _Geometry(model, self.p)
        self.gates = [_Gate(b['gate'], self.p) for b in model.blocks]
        ent = []
        for t, blk in enumerate(model.blocks):
            ent += [(f'sc{t}', blk['sc'], f'{t}_self_connection_intro.linear.weight'),
                    (f'si1{t}', blk['si1'], f'{t}_self_interaction_1.linear.weight'),
                    (f'si2{t}', blk['si2'], f'{t}_self_interaction_2.linear.weight')]
        ent += [('r1', model.readout1, 'reduce_input_to_hidden.linear.weight'),
                ('r2', model.readout2, 'reduce_hidden_to_energy.linear.weight')]
        # si2 (mid irreps -> gate input) is block-diagonal by l: ~10x zeros in
        # its dense matrix.  Its products per instruction block (strided views,
        # E3GNN_TRAIN_SI2_BLOCKS=1) measured SLOWER at the fine-tune batch size
        # (10.05-10.2 vs 8.14 ms per step, same box): three small strided GEMMs
        # cost more than one dense one.  Default: one dense product per use.
        self.si2_blocks = []
        dense_si2 = os.environ.get('E3GNN_TRAIN_SI2_BLOCKS', '0') != '1'
        for t, blk in enumerate(model.blocks):
            lin = blk['si2']
            bl = [(lin.in_off[i], lin.in_off[i] + lin.irreps_in[i][0] * (2 * lin.irreps_in[i][1] + 1),
                   lin.out_off[j], lin.out_off[j] + lin.irreps_out[j][0] * (2 * lin.irreps_out[j][1] + 1))
                  for i, j in lin.ins]
            if dense_si2:
                bl = [(0, lin.in_off[-1], 0, lin.out_off[-1])]
            cover = sorted({(a, b) for a, b, _, _ in bl})
            gaps, pos = [], 0
            for a, b in cover:
                if a > pos:
                    gaps.append((pos, a))
                pos = max(pos, b)
            if pos < lin.in_off[-1]:
                gaps.append((pos, lin.in_off[-1]))
            self.si2_blocks.append((bl, gaps))
        self.dense_si2 = dense_si2
        # frozen convolution denominators (the default) are folded into si2:
        # agg / den W = agg (W / den), and the si2 gradient divided by den in
        # the flush -- no division launches on the activations
        dens = [f'{t}_convolution.denominator' for t in range(len(model.blocks))]
        self.fold_den = not any(model.param(d).requires_grad for d in dens)
        self.bank = _DenseBank(model, ent, {f'si2{t}': d for t, d in enumerate(dens)}
                               if self.fold_den else None)
        self._lins = {key: lin for key, lin, _ in ent}
        self._lb_cache = {}
        # E3GNN_TRAIN_IRREPS=0: the dense products (zero-block ranges only)
        self._irreps = os.environ.get('E3GNN_TRAIN_IRREPS', '1') != '0'
        self._dims = {key: (lin.in_off[-1], lin.out_off[-1]) for key, lin, _ in ent}
        self._kr_cache = {}
        # the radial MLP weights of every block, scaled by 1/sqrt(fan-in)
        # (e3nn FullyConnectedNet), gathered into one buffer by one launch
        idx, scl, self.mlp_views = [], [], []
        off = 0
        for t in range(len(model.blocks)):
            views = []
            for li in range(3):
                o, cnt, shape = model.slices[f'{t}_convolution.weight_nn.layer{li}.weight']
                idx.append(np.arange(o, o + cnt))
                scl.append(np.full(cnt, 1.0 / math.sqrt(shape[0])))
                views.append((off, shape))
                off += cnt
            self.mlp_views.append(views)
        dev, dt = model.flat.device, model.flat.dtype
        self.mlp_idx = torch.as_tensor(np.concatenate(idx), device=dev)
        self.mlp_scl = torch.as_tensor(np.concatenate(scl), device=dev, dtype=dt)
        self.mlp_buf = torch.empty(off, device=dev, dtype=dt)
        # layer 2 of the forward / tangent chains on bf16x6 matrix cores
        # (e3gnn_radial_mlp_forward_p): the W2 piece images, rebuilt by one
        # launch with the weights (E3GNN_TRAIN_MLP_BF16=0: the f32 chains)
        self.w2p = None
        self._w2p_of = {}
        widths = [views[2][1][1] for views in self.mlp_views]
        if (self.p._hip(self.mlp_buf) and os.environ.get('E3GNN_TRAIN_MLP_BF16', '1') != '0'
                and all(w % 16 == 0 for w in widths) and len(widths) <= 8):
            lib = self.p.lib
            nb = [int(lib.e3gnn_radial_mlp_w2_piece_bytes(w)) for w in widths]
            offs = np.concatenate([[0], np.cumsum(nb)]).astype(np.int64)
            self.w2p_buf = torch.empty(int(offs[-1]), device=dev, dtype=torch.uint8)
            self.w2p = [self.w2p_buf.data_ptr() + int(o) for o in offs[:-1]]
            self.w2p_widths = (ctypes.c_int32 * len(widths))(*widths)

    def _mlp_weights(self):
        """[(W0, W1, W2) per block], each scaled by 1/sqrt(fan-in), views of one
        buffer filled by one gather-multiply (16-byte aligned when the counts
        are multiples of 4)"""
        torch.mul(self.m.flat.detach()[self.mlp_idx], self.mlp_scl, out=self.mlp_buf)
        Ws = [tuple(self.mlp_buf[o:o + int(np.prod(sh))].view(*sh) for o, sh in views)
              for views in self.mlp_views]
        self._w2p_of = {}
        if self.w2p is not None:
            from . import _lib
            n = len(Ws)
            srcs = (ctypes.c_void_p * n)(*[W[2].data_ptr() for W in Ws])
            imgs = (ctypes.c_void_p * n)(*self.w2p)
            _lib.check(self.p.lib.e3gnn_radial_mlp_w2_pieces(n, srcs, self.w2p_widths, imgs,
                                                             self._stream(self.mlp_buf)))
            self._w2p_of = {W[2].data_ptr(): q for W, q in zip(Ws, self.w2p)}
        return Ws

    def _P(self, name):
        return self.m.param(name)

    def _mm(self, C, A, B, alpha=1.0, beta=0, A2=None, B2=None, kr=None):
        """one product now (its result is needed next)"""
        self.gm.add(C, A, B, alpha, beta, A2, B2, kr=kr)
        self.gm.flush()
        return C

    # ---- the linears per l-block in the e3nn irreps layout (e3gnn_gemm_layouts):
    # rows (node, m) of [node][mul][2l+1] blocks against the m = 0 diagonal of
    # the dense matrices -- no zero blocks and no zeros between the m copies
    # (the dense products spent 2l + 1 times the work on those); weight
    # gradients summed over K = (m, node) segments into the m = 0 diagonal of
    # the dense gradient (the bank's flush sums the diagonal positions)
    def _lblocks(self, key):
        """[(l, d, in_lo, mul_in, out_lo, mul_out)] of key's linear, its input
        and output irreps merged by l (sorted by l: consecutive)"""
        if key in self._lb_cache:
            return self._lb_cache[key]
        lin = self._lins[key]
        def merged(irreps, offs):
            out = {}
            for i, (mul, l, _) in enumerate(irreps):
                d = 2 * l + 1
                if l in out:
                    lo, m0 = out[l]
                    assert lo + m0 * d == offs[i], 'irreps of one l not contiguous'
                    out[l] = (lo, m0 + mul)
                else:
                    out[l] = (offs[i], mul)
            return out
        ins = merged(lin.irreps_in, lin.in_off)
        outs = merged(lin.irreps_out, lin.out_off)
        ls = sorted({lin.irreps_in[i][1] for i, j in lin.ins})
        res = [(l, 2 * l + 1, ins[l][0], ins[l][1], outs[l][0], outs[l][1]) for l in ls]
        self._lb_cache[key] = res
        return res

    def _irr(self, *ts):
        return self._irreps and self.gm._hip(*ts)

    def _lin(self, C, A, key, A2=None, key2=None, trans=False, beta=0, flush=True):
        """C = A op(D[key]) [+ A2 op(D[key2])], op = identity or transpose, one
        problem per l-block (the dense product with its zero-block ranges on
        other devices / dtypes)"""
        D = self.S['D']
        if not self._irr(C, A, *([A2] if A2 is not None else [])):
            B = D[key].t() if trans else D[key]
            B2 = None if key2 is None else (D[key2].t() if trans else D[key2])
            kr = self._kr((key, trans), None if key2 is None else (key2, trans))
            self.gm.add(C, A, B, beta=beta, A2=A2, B2=B2, kr=kr)
            if flush:
                self.gm.flush()
            return C
        from . import _lib
        rows = int(A.shape[0])
        outs = {}
        for Ai, k in [(A, key)] + ([(A2, key2)] if A2 is not None else []):
            Dk = D[k]
            dout = int(Dk.shape[1])
            for (l, d, in_lo, mi, out_lo, mo) in self._lblocks(k):
                if trans:   # C[:, in] += A[:, out] D[in, out]^T: k over the output block
                    ent = (Ai, out_lo, mo, Dk, in_lo * dout + out_lo, d * dout, d)
                    outs.setdefault((l, in_lo, mi, d), []).append(ent)
                else:
                    ent = (Ai, in_lo, mi, Dk, in_lo * dout + out_lo, d, d * dout)
                    outs.setdefault((l, out_lo, mo, d), []).append(ent)
        for (l, c_lo, N, d), ps in outs.items():
            assert len(ps) <= 2
            lay = _lib.GemmLayouts()
            ops = []
            for (Ai, a_lo, K, Dk, b_off, b_ld, b_kst), La, Lb in zip(ps, (lay.a, lay.a2), (lay.b, lay.b2)):
                La.ld, La.rep, La.rs, La.kst, La.ks, La.sst = Ai.stride(0), d, 1, d, K, 0
                Lb.ld, Lb.rep, Lb.rs, Lb.kst, Lb.ks, Lb.sst = b_ld, 1, 0, b_kst, K, 0
                ops.append(((Ai, a_lo), (Dk, b_off), K))
            lay.ldc, lay.crep, lay.crs, lay.cns = C.stride(0), d, 1, d
            extra = {}
            if len(ops) > 1:
                extra = dict(A2=ops[1][0], B2=ops[1][1], K2=ops[1][2])
            self.gm.add_lay(rows * d, N, ops[0][2], (C, c_lo), ops[0][0], ops[0][1], lay, beta=beta, **extra)
        if flush:
            self.gm.flush()
        return C

    def _lin_grad(self, G, X, Y, key):
        """G += X^T Y, G the dense gradient of key's matrix, on its l-blocks"""
        if not self._irr(G, X, Y):
            self.gm.add(G, X.t(), Y, beta=1, kr=self._kr(None, grad=key), wgrad=True)
            return
        from . import _lib
        rows = int(X.shape[0])
        dout = int(G.shape[1])
        for (l, d, in_lo, mi, out_lo, mo) in self._lblocks(key):
            lay = _lib.GemmLayouts()
            # element (u, (m, node)) = X[node][in_lo + u d + m]
            lay.a.ld, lay.a.rep, lay.a.rs, lay.a.kst, lay.a.ks, lay.a.sst = d, 1, 0, X.stride(0), rows, 1
            lay.b.ld, lay.b.rep, lay.b.rs, lay.b.kst, lay.b.ks, lay.b.sst = d, 1, 0, Y.stride(0), rows, 1
            lay.ldc, lay.crep, lay.crs, lay.cns = d * dout, 1, 0, d
            self.gm.add_lay(mi, mo, d * rows, (G, in_lo * dout + out_lo), (X, in_lo), (Y, out_lo), lay,
                            beta=1, wgrad=True)

    # ---- block sparsity of the dense linear matrices (e3gnn_gemm_desc::krange)
    def _lin_blocks(self, key, trans=False):
        """(row range, column range) of every nonzero block of key's dense
        matrix (din x dout; trans: of its transpose)"""
        lin = self._lins[key]
        out = []
        for i, j in lin.ins:
            r = (lin.in_off[i], lin.in_off[i] + lin.irreps_in[i][0] * (2 * lin.irreps_in[i][1] + 1))
            c = (lin.out_off[j], lin.out_off[j] + lin.irreps_out[j][0] * (2 * lin.irreps_out[j][1] + 1))
            out.append((c, r) if trans else (r, c))
        return out

    def _kr(self, part1, part2=None, grad=None):
        """per-tile k ranges of a product with the dense matrices on its right:
        part1 / part2 = (key, trans) of C = A op(D) [+ A2 op(D2)] -- for each
        64-column tile of C the hull of the k rows of op(D) that are nonzero in
        it; grad = key: C = A^T B is key's dense gradient (din x dout), tiles
        that meet no block get an empty range (nothing is added there).
        (device int32 tensor, row-tile stride), cached."""
        ck = (part1, part2, grad)
        if ck in self._kr_cache:
            return self._kr_cache[ck]
        T = 64
        if grad is not None:
            bl = self._lin_blocks(grad)
            din, dout = self._dims[grad]
            tm, tn = -(-din // T), -(-dout // T)
            tab = np.zeros((tm, tn, 4), dtype=np.int32)
            for a in range(tm):
                for b in range(tn):
                    if any(r0 < (a + 1) * T and r1 > a * T and c0 < (b + 1) * T and c1 > b * T
                           for (r0, r1), (c0, c1) in bl):
                        tab[a, b, 1] = 1 << 30          # the whole K
            res = (torch.as_tensor(tab.ravel(), device=self.m.flat.device), tn)
        else:
            def hull(key, trans, ncol):
                bl = self._lin_blocks(key, trans)
                out = np.zeros((-(-ncol // T), 2), dtype=np.int32)
                for b in range(out.shape[0]):
                    rows = [(r0, r1) for (r0, r1), (c0, c1) in bl if c0 < (b + 1) * T and c1 > b * T]
                    if rows:
                        out[b] = (min(r for r, _ in rows), max(r for _, r in rows))
                return out
            d1 = self._dims[part1[0]]
            ncol = d1[0] if part1[1] else d1[1]
            tab = np.zeros((-(-ncol // T), 4), dtype=np.int32)
            tab[:, :2] = hull(part1[0], part1[1], ncol)
            if part2 is not None:
                tab[:, 2:] = hull(part2[0], part2[1], ncol)
            res = (torch.as_tensor(tab.ravel(), device=self.m.flat.device), 0)
        self._kr_cache[ck] = res
        return res

    # ---- si2 products over its instruction blocks (views, no copies)
    def _si2_fwd(self, t, A, Dm, out):
        """out += A Dm (the gate-input rows)"""
        for i0, i1, o0, o1 in self.si2_blocks[t][0]:
            out[:, o0:o1].addmm_(A[:, i0:i1], Dm[i0:i1, o0:o1])

    def _si2_t(self, t, A, Dm):
        """A Dm^T (cotangent rows of the mid irreps)"""
        if self.dense_si2:
            return self._lin(torch.empty(A.shape[0], Dm.shape[0], device=A.device, dtype=A.dtype),
                             A, f'si2{t}', trans=True)
        bl, gaps = self.si2_blocks[t]
        out = torch.empty(A.shape[0], Dm.shape[0], device=A.device, dtype=A.dtype)
        seen = set()
        for i0, i1, o0, o1 in bl:
            out[:, i0:i1].addmm_(A[:, o0:o1], Dm[i0:i1, o0:o1].t(),
                                 beta=1.0 if (i0, i1) in seen else 0.0)
            seen.add((i0, i1))
        for a, b in gaps:
            out[:, a:b].zero_()
        return out

    def _si2_wgrad(self, t, Gm, A, B):
        """Gm += A^T B on si2's blocks (the other entries of the dense gradient
        map to no weight)"""
        for i0, i1, o0, o1 in self.si2_blocks[t][0]:
            Gm[i0:i1, o0:o1].addmm_(A[:, i0:i1].t(), B[:, o0:o1])

    # ---- the radial MLP chains: one HIP launch each (e3gnn_radial_mlp_*) on
    # float32 device tensors, the same GEMMs + element-wise steps otherwise
    def _mlp_hip(self, t):
        return self.p._hip(t)

    @staticmethod
    def _stream(t):
        return torch.cuda.current_stream(t.device).cuda_stream

    def _mlp_fwd(self, e, Ws, a1p, a2p, A1, H1, A2, H2, WT):
        """forward chain (a1p None) or the tangent chain along e' = ``e``"""
        W0, W1, W2 = Ws
        if self._mlp_hip(e) and W2.shape[1] % 16 == 0:
            from . import _lib
            ptr = lambda t: t.data_ptr() if t is not None else None   # noqa: E731
            _lib.check(self.p.lib.e3gnn_radial_mlp_forward_p(
                int(e.shape[0]), int(W2.shape[1]), e.data_ptr(), W0.data_ptr(), W1.data_ptr(),
                W2.data_ptr(), self._w2p_of.get(W2.data_ptr()), ptr(a1p), ptr(a2p), A1.data_ptr(),
                H1.data_ptr(), A2.data_ptr(), H2.data_ptr(), WT.data_ptr(), self.p.c, self._stream(e)))
            return
        torch.mm(e, W0, out=A1)
        if a1p is None:
            self.p.act(A1, out=H1)
        else:
            self.p.act_jvp(a1p, A1, out=H1)
        torch.mm(H1, W1, out=A2)
        if a2p is None:
            self.p.act(A2, out=H2)
        else:
            self.p.act_jvp(a2p, A2, out=H2)
        torch.mm(H2, W2, out=WT)

    def _mlp_rev(self, wb, Ws, a1, a2, embb):
        """embb += the reverse chain of wb (first reverse)"""
        W0, W1, W2 = Ws
        if self._mlp_hip(wb) and W2.shape[1] % 16 == 0:
            from . import _lib
            _lib.check(self.p.lib.e3gnn_radial_mlp_backward_p(
                int(wb.shape[0]), int(W2.shape[1]), wb.contiguous().data_ptr(), W0.data_ptr(),
                W1.data_ptr(), W2.data_ptr(), self._w2p_of.get(W2.data_ptr()), a1.data_ptr(), a2.data_ptr(),
                None, None, None, None, embb.data_ptr(), self.p.c, self._stream(wb)))
            return
        a2b = self.p.act_jvp(a2, wb @ W2.t())
        a1b = self.p.act_jvp(a1, a2b @ W1.t())
        embb.addmm_(a1b, W0.t())

    def _mlp_dual(self, WB, Ws, A1, A2, A2B, A1B, EMBB):
        """reverse of the (primal, tangent) chains: A2B, A1B ([2E, 64]) and
        EMBB += (A1, A2: stacked [primal; tangent] pre-activations)"""
        W0, W1, W2 = Ws
        E = A1.shape[0] // 2
        if self._mlp_hip(WB) and W2.shape[1] % 16 == 0:
            from . import _lib
            _lib.check(self.p.lib.e3gnn_radial_mlp_backward_p(
                E, int(W2.shape[1]), WB.data_ptr(), W0.data_ptr(), W1.data_ptr(), W2.data_ptr(),
                self._w2p_of.get(W2.data_ptr()), A1[:E].data_ptr(), A2[:E].data_ptr(), A1[E:].data_ptr(),
                A2[E:].data_ptr(), A2B.data_ptr(), A1B.data_ptr(), EMBB.data_ptr(), self.p.c,
                self._stream(WB)))
            return
        H2B = WB @ W2.t()
        self.p.act_dual(A2[:E], A2[E:], H2B[:E], H2B[E:], out0=A2B[:E], out1=A2B[E:])
        H1B = A2B @ W1.t()
        self.p.act_dual(A1[:E], A1[E:], H1B[:E], H1B[E:], out0=A1B[:E], out1=A1B[E:])
        EMBB.addmm_(A1B, W0.t())

    def _G(self, name):
        """the gradient view of a parameter (a slice of flat_grad), or None when frozen"""
        p = self.m.param(name)
        if not p.requires_grad:
            return None
        off, n, shape = self.m.slices[name]
        return self.m.flat_grad[off:off + n].view(shape)

    # ---------------------------------------------------------------- 1 + 2
    def forward(self, data, graph=None):
        """Primal forward and first reverse.  Returns the model's output dict
        (energy per graph, forces, stress) -- the loss's inputs.

        Activations live in STACKED buffers, primal rows first and their
        tangents (filled by backward()) after them -- [emb; emb'], [a1; a1'],
        [h1; h1'], ..., [x; x'], [agg; agg'] (/den unless folded into si2), [y; y'] -- so the reverse
        sweep forms each weight gradient x^T y-bar + x'^T y'-bar and each input
        gradient [y-bar; y'-bar] W^T as ONE GEMM."""
        m = self.m
        dev = m.flat.device
        dt = m.dtype
        types = data[KEY.NODE_FEATURE].to(dev).long()
        n = int(types.shape[0])
        ei = data[KEY.EDGE_IDX].to(dev).long()
        vec = data[KEY.EDGE_VEC].to(dev, dt).detach()
        batch = data[KEY.BATCH].to(dev).long() if KEY.BATCH in data else \
            torch.zeros(n, dtype=torch.long, device=dev)
        nb = int(data[KEY.NUM_ATOMS].numel()) if KEY.NUM_ATOMS in data else 1
        center, nbr = ei[0], ei[1]
        perm = None
        if graph is None:
            from .train import edges_marked_sorted
            if (not edges_marked_sorted(data) and center.numel() > 1
                    and bool((center[1:] < center[:-1]).any())):
                perm = torch.argsort(center, stable=True)
                center, nbr = center[perm], nbr[perm]
            graph = conv_ops.ConvGraph(n, center, nbr, m.conv_backend)
        vec_k = vec[perm] if perm is not None else vec
        E = int(vec_k.shape[0])
        S = self.S = {'n': n, 'E': E, 'nb': nb, 'types': types, 'batch': batch, 'center': center,
                      'nbr': nbr, 'graph': graph, 'vec': vec_k}
        coeffs = self._P('edge_embedding.basis_function.coeffs').detach()
        EMB = torch.empty(2 * E, 8, device=dev, dtype=dt)
        g = self.geo.forward(vec_k, coeffs, emb_out=EMB[:E])
        S['geo'] = g
        S['EMB'] = EMB
        D = S['D'] = self.bank.build()
        MW = self._mlp_weights()
        P = lambda name: self._P(name).detach()   # noqa: E731
        emb_w = P('onehot_to_feature_x.linear.weight').view(m.nsp, -1)
        X = torch.empty(2 * n, emb_w.shape[1], device=dev, dtype=dt)
        torch.mul(emb_w[types], 1.0 / math.sqrt(m.nsp), out=X[:n])
        X[n:].zero_()                          # x0 does not depend on the edge vectors
        blocks = []
        be = m.conv_backend
        new = lambda *shape: torch.empty(*shape, device=dev, dtype=dt)   # noqa: E731
        for t, blk in enumerate(m.blocks):
            pre = f'{t}_convolution'
            W0, W1, W2 = MW[t]
            x = X[:n]
            H = new(2 * n, D[f'si1{t}'].shape[1])
            self._lin(H[:n], x, f'si1{t}')
            A1, H1 = new(2 * E, W0.shape[1]), new(2 * E, W0.shape[1])
            A2, H2 = new(2 * E, W1.shape[1]), new(2 * E, W1.shape[1])
            WT = new(2 * E, W2.shape[1])
            self._mlp_fwd(EMB[:E], (W0, W1, W2), None, None, A1[:E], H1[:E], A2[:E], H2[:E], WT[:E])
            den = P(f'{pre}.denominator')
            AGG = new(2 * n, D[f'si2{t}'].shape[0])
            be.forward(blk['kind'], graph, H[:n], g['Y'], WT[:E], out=AGG[:n])
            if not self.fold_den:            # (folded: D[si2] is si2 / den)
                AGG[:n].div_(den)
            Yg = new(2 * n, D[f'si2{t}'].shape[1])
            if self.dense_si2:                              # x sc + agg si2: one product
                self._lin(Yg[:n], x, f'sc{t}', A2=AGG[:n], key2=f'si2{t}')
            else:
                self._mm(Yg[:n], x, D[f'sc{t}'])            # (GEMM into the output, then
                self._si2_fwd(t, AGG[:n], D[f'si2{t}'], Yg[:n])  # accumulate: no bias copy)
            Xn = new(2 * n, self.gates[t].dims[3] if self.gates[t].ng else Yg.shape[1])
            self.gates[t].fwd(Yg[:n], out=Xn[:n])
            blocks.append({'X': X, 'H': H, 'A1': A1, 'H1': H1, 'A2': A2, 'H2': H2, 'WT': WT,
                           'W': (W0, W1, W2), 'den': den, 'AGG': AGG, 'Y': Yg})
            X = Xn
        S['blocks'] = blocks
        S['XL'] = X
        hid = self._mm(new(n, D['r1'].shape[1]), X[:n], D['r1'])
        e = self._mm(new(n, 1), hid, D['r2'])[:, 0]
        scale = P('rescale_atomic_energy.scale')[types]
        atomic = e * scale + P('rescale_atomic_energy.shift')[types]
        S.update(hid=hid, e=e, scale=scale)
        energy = torch.zeros(nb, device=dev, dtype=atomic.dtype).index_add(0, batch, atomic)

        # ---- first reverse: dE/dr per edge (seed dE/d atomic = 1)
        xb = self._mm(new(n, D['r1'].shape[0]), scale.unsqueeze(-1) * D['r2'][:, 0].unsqueeze(0),
                      D['r1'].t())
        Yb = torch.empty_like(g['Y'])         # the last block's launch assigns, the others add
        embb = torch.zeros_like(g['emb'])
        for t in range(len(blocks) - 1, -1, -1):
            b, blk = blocks[t], m.blocks[t]
            yb = self.gates[t].vjp(b['Y'][:n], xb)
            ab = self._si2_t(t, yb, D[f'si2{t}'])
            if not self.fold_den:
                ab.div_(b['den'])
            hb, _, wb = be.backward(blk['kind'], graph, b['H'][:n], g['Y'], b['WT'][:E], ab,
                                    need_h=t > 0, dY_out=Yb,
                                    acc=ACC_DY if t < len(blocks) - 1 else 0)
            self._mlp_rev(wb, b['W'], b['A1'][:E], b['A2'][:E], embb)
            if t > 0:
                xb = self._lin(new(n, hb.shape[1]), hb, f'si1{t}', A2=yb, key2=f'sc{t}', trans=True)
        fij = self.geo.vjp(g, Yb, embb)                    # dE/dr_e, centre-sorted order
        S['fij'] = fij
        aux = graph.aux
        if 'row_ptr' in aux and fij.is_cuda and fij.dtype == torch.float32:
            from . import _lib
            force = torch.empty(n, 3, device=dev)
            _lib.check(self.p.lib.e3gnn_edge_forces_to_atoms(
                n, aux['row_ptr'].data_ptr(), aux['src_ptr'].data_ptr(), aux['src_perm'].data_ptr(),
                fij.data_ptr(), force.data_ptr(), torch.cuda.current_stream(dev).cuda_stream))
        else:
            force = torch.zeros(n, 3, device=dev, dtype=fij.dtype).index_add(
                0, torch.cat([center, nbr]), torch.cat([fij, -fij]))
        voigt = vec_k.repeat(1, 2) * torch.cat([fij, fij.roll(-1, dims=1)], dim=1)
        s_graph = torch.zeros(nb, 6, device=dev, dtype=fij.dtype).index_add(0, batch[nbr], voigt)
        out = dict(data)
        out[KEY.ATOMIC_ENERGY] = atomic.unsqueeze(-1)
        out[KEY.PRED_TOTAL_ENERGY] = energy.requires_grad_(True)
        out[KEY.PRED_FORCE] = force.requires_grad_(True)
        if KEY.CELL_VOLUME in data:
            vol = data[KEY.CELL_VOLUME].to(dev, m.dtype).view(-1)
            S['vol'] = vol
            out[KEY.PRED_STRESS] = (torch.neg(s_graph) / vol.unsqueeze(-1)).detach().requires_grad_(True)
        self.out = out
        return out

    # ---------------------------------------------------------------- 4
    def backward(self, cE, cF, cS=None):
        """Accumulate dL/dtheta into model.flat_grad from the loss cotangents
        of the energies (per graph), forces and stress (per graph, or None)."""
        m, S = self.m, self.S
        D, g = S['D'], S['geo']
        n, E = S['n'], S['E']
        types, batch, center, nbr = S['types'], S['batch'], S['center'], S['nbr']
        be, graph = m.conv_backend, S['graph']
        dt = m.dtype
        dev = types.device
        cE = cE.to(dt) if cE is not None else torch.zeros(S['nb'], device=dev, dtype=dt)
        cF = cF.to(dt) if cF is not None else torch.zeros(n, 3, device=dev, dtype=dt)
        # ---- tangent forward along v_e = dL/df_e (second halves of the stacked
        # buffers; fused: the backend's one-launch tangent forward / dual
        # backward of the convolution; the generic engine's backend composes them)
        fused = hasattr(be, 'dual_backward') and hasattr(be, 'tangent_forward')
        EMB = S['EMB']
        Yd, rd = self.geo.tangent(g, S, cF, cS.to(dt) if cS is not None else None, EMB[E:])
        blocks = S['blocks']
        Y = g['Y']
        for t, blk in enumerate(m.blocks):
            b = blocks[t]
            k = blk['kind']
            A1, H1, A2, H2, WT = b['A1'], b['H1'], b['A2'], b['H2'], b['WT']
            self._mlp_fwd(EMB[E:], b['W'], A1[:E], A2[:E], A1[E:], H1[E:], A2[E:], H2[E:], WT[E:])
            h, w = b['H'][:n], WT[:E]
            AGG, Yg = b['AGG'], b['Y']
            aggd = AGG[n:]                       # C(h, Y', w) + C(h, Y, w') + C(h', Y, w)
            X = b['X']
            if t > 0:
                self._lin(b['H'][n:], X[n:], f'si1{t}')
            hd = b['H'][n:] if t > 0 else None   # x0' = 0: no h' term
            if fused:
                be.tangent_forward(k, graph, h, hd, Y, Yd, w, WT[E:], out=aggd)
            else:
                be.forward(k, graph, h, Yd, w, out=aggd)
                be.forward(k, graph, h, Y, WT[E:], out=aggd, acc=True)
                if hd is not None:
                    be.forward(k, graph, hd, Y, w, out=aggd, acc=True)
            if not self.fold_den:
                aggd.div_(b['den'])
            if self.dense_si2:
                if t > 0:
                    self._lin(Yg[n:], X[n:], f'sc{t}', A2=AGG[n:], key2=f'si2{t}')
                else:                            # x0' = 0
                    self._lin(Yg[n:], AGG[n:], f'si2{t}')
            else:
                if t > 0:
                    self._mm(Yg[n:], X[n:], D[f'sc{t}'])
                else:
                    Yg[n:].zero_()
                self._si2_fwd(t, AGG[n:], D[f'si2{t}'], Yg[n:])
            Xn = blocks[t + 1]['X'] if t + 1 < len(blocks) else S['XL']
            self.gates[t].jvp(Yg[:n], Yg[n:], out=Xn[n:])
        XL = S['XL']
        hidd = self._mm(torch.empty(n, D['r1'].shape[1], device=dev, dtype=dt), XL[n:], D['r1'])
        ed = self._mm(torch.empty(n, 1, device=dev, dtype=dt), hidd, D['r2'])[:, 0]

        # ---- one reverse sweep over (primal, tangent); seeds cE on E, 1 on E'
        G = self.bank.grads()
        # the weight gradients (G, read only by the bank's flush below) take
        # their split-K reductions in one launch at the end of the sweep
        self.gm.begin_defer()
        scale = S['scale']
        atb = cE[batch]                       # d L / d atomic
        gsc = self._G('rescale_atomic_energy.scale')
        if gsc is not None:
            gsc.index_add_(0, types, atb * S['e'] + ed)
        gsh = self._G('rescale_atomic_energy.shift')
        if gsh is not None:
            gsh.index_add_(0, types, atb)
        # [e-bar; e'-bar] = [cE scale; scale]
        EB = torch.cat([atb * scale, scale]).unsqueeze(-1)
        HID = torch.cat([S['hid'], hidd])
        HIDB = EB * D['r2'][:, 0].unsqueeze(0)
        XB = torch.empty(2 * n, D['r1'].shape[0], device=dev, dtype=dt)
        self.gm.add(G['r2'], HID.t(), EB, beta=1, wgrad=True)
        self.gm.add(G['r1'], XL.t(), HIDB, beta=1, wgrad=True)
        self.gm.add(XB, HIDB, D['r1'].t())    # [x-bar; x'-bar] of the last block's output
        self.gm.flush()
        EMBB = torch.zeros(2 * E, 8, device=dev, dtype=dt)
        new = lambda *shape: torch.empty(*shape, device=dev, dtype=dt)   # noqa: E731
        dYs = new(E, 9)                       # scratch for the unused dY outputs
        for t in range(len(blocks) - 1, -1, -1):
            b, blk = blocks[t], m.blocks[t]
            k = blk['kind']
            pre = f'{t}_convolution'
            Yg, AGG, X, H = b['Y'], b['AGG'], b['X'], b['H']
            YB = new(2 * n, Yg.shape[1])
            self.gates[t].dual_vjp(Yg[:n], Yg[n:], XB[:n], XB[n:], out0=YB[:n], out1=YB[n:])
            if self.dense_si2:
                # independent products of y-bar, one launch: si2's and sc's weight
                # gradients and agg-bar
                AGGB = new(2 * n, D[f'si2{t}'].shape[0])
                self._lin_grad(G[f'si2{t}'], AGG, YB, f'si2{t}')
                self._lin(AGGB, YB, f'si2{t}', trans=True, flush=False)
                self._lin_grad(G[f'sc{t}'], X, YB, f'sc{t}')
                self.gm.flush()
            else:
                self._si2_wgrad(t, G[f'si2{t}'], AGG, YB)
                AGGB = self._si2_t(t, YB, D[f'si2{t}'])
                self._mm(G[f'sc{t}'], X.t(), YB, beta=1)
            gden = self._G(f'{pre}.denominator')
            if gden is not None:
                gden.sub_(torch.dot(AGGB.view(-1), AGG.view(-1)) / b['den'])
            AB = AGGB if self.fold_den else AGGB / b['den']
            ab, adb = AB[:n], AB[n:]
            h, hd = H[:n], H[n:]
            WT = b['WT']
            w, wd = WT[:E], WT[E:]
            # trilinear agg = C(h, Y, w): B(h', Y', w'; c) = (B_h(Y', w'), B_Y(h', w'), B_w(h', Y'))
            # (the accumulating launches add into HB / WB; dY is not needed: Y and
            # Y' do not depend on the parameters)
            HB, WB = new(2 * n, H.shape[1]), new(2 * E, WT.shape[1])
            hb, wb, hdb, wdb = HB[:n], WB[:E], HB[n:], WB[E:]
            if fused:                         # the four products below in one launch
                be.dual_backward(k, graph, h, hd if t > 0 else None, Y, Yd, w, wd, ab, adb,
                                 hb, hdb if t > 0 else None, wb, wdb)
            else:
                be.backward(k, graph, h, Y, w, ab, dh_out=hb, dw_out=wb, dY_out=dYs)  # B_h(Y,w;a), B_w(h,Y;a)
                be.backward(k, graph, h, Yd, w, adb, dh_out=hb, dw_out=wb, dY_out=dYs,
                            acc=ACC_DH | ACC_DW)                                     # + B_h(Y',w), B_w(h,Y')
                be.backward(k, graph, h, Y, wd, adb, dh_out=hb, dw_out=wdb, dY_out=dYs,
                            acc=ACC_DH)                                              # + B_h(Y,w'); w'-bar
                if t > 0:
                    be.backward(k, graph, hd, Y, w, adb, dh_out=hdb, dw_out=wb, dY_out=dYs,
                                acc=ACC_DW)                                          # h'-bar; + B_w(h',Y)
            if t == 0:
                HB[n:].zero_()                # x0' = 0: no h' (its rows meet zero rows of X)
            # radial MLP, primal and tangent rows together
            W0, W1, W2 = b['W']
            A2B, A1B = new(2 * E, W1.shape[1]), new(2 * E, W0.shape[1])
            self._mlp_dual(WB, b['W'], b['A1'], b['A2'], A2B, A1B, EMBB)
            # the block's remaining products are independent: one launch (+ the
            # split-K reduction of the edge-summed weight gradients, K = 2E)
            for li, (rows, cot, Wl) in enumerate(((EMB, A1B, W0), (b['H1'], A2B, W1), (b['H2'], WB, W2))):
                gw = self._G(f'{pre}.weight_nn.layer{li}.weight')
                if gw is not None:
                    self.gm.add(gw, rows.t(), cot, 1.0 / math.sqrt(Wl.shape[0]), beta=1, wgrad=True)
            # self-interaction 1 (sc-bar = y-bar, added above) and the input cotangent
            self._lin_grad(G[f'si1{t}'], X, HB, f'si1{t}')
            XB = new(2 * n, D[f'si1{t}'].shape[0])
            self._lin(XB, HB, f'si1{t}', A2=YB, key2=f'sc{t}', trans=True, flush=False)
            self.gm.flush()
        # embedding (x0 = W[types] / sqrt(nsp)) and the radial basis coefficients
        gemb = self._G('onehot_to_feature_x.linear.weight')
        if gemb is not None:
            gemb.view(m.nsp, -1).index_add_(0, types, XB[:n] / math.sqrt(m.nsp))
        gco = self._G('edge_embedding.basis_function.coeffs')
        if gco is not None:
            coeffs = self._P('edge_embedding.basis_function.coeffs').detach()
            gco.add_(self.geo.coeff_grad(g, EMBB[:E], EMBB[E:], rd, coeffs))
        self.gm.finish_defer()
        self.bank.flush(m.flat_grad)
