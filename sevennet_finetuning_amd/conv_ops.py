"""Differentiable (to second order) convolution op on the HIP kernels.

The reference computes, inside ``IrrepsConvolution.forward``
(sevenn/nn/convolution.py:104-123),

    msg[e] = TP(x[edge_index[1][e]], Y[e], w[e])       e3nn uvu TensorProduct
    agg[i] = sum_{e: edge_index[0][e] = i} msg[e]       message_gather :19-32

and the fine-tune step differentiates it twice: once for the forces
(``autograd.grad(..., create_graph=self.training)``, force_output.py:158-215)
and once more for the parameter gradients of the force/stress loss
(trainer.py:155-222).  ``agg(h, Y, w)`` is trilinear, so with
``s = <g, agg(h, Y, w)>`` every derivative is one of two launches of
libe3gnn_hip.so with permuted operands:

    forward   F(h, Y, w)        = agg                         e3gnn_conv_forward
    backward  B(h, Y, w, g)     = (ds/dh, ds/dY, ds/dw)       e3gnn_conv_backward

and the derivative of B against cotangents (a_h, a_Y, a_w) is

    d/dg = F(a_h, Y, w) + F(h, a_Y, w) + F(h, Y, a_w)
    d/dh = B(h, a_Y, w, g).dh + B(h, Y, a_w, g).dh
    d/dY = B(a_h, Y, w, g).dY + B(h, Y, a_w, g).dY
    d/dw = B(a_h, Y, w, g).dw + B(h, a_Y, w, g).dw

(each B call supplies two of the six terms).  There is no CPU fallback: the
default backend is the library, and a missing library raises ``E3GNNError``.
"""
import ctypes

import torch

from . import _lib


class ConvGraph:
    """Edge CSR of one (batched) graph on the device: ``edge_center`` sorted
    non-decreasing (the aggregation target, edge_index[0]), ``edge_nbr`` the
    gathered source (edge_index[1]), plus the transposed CSR the dE/dh sum
    uses.  Built once per batch and shared by the five interaction blocks."""

    def __init__(self, n_nodes, edge_center, edge_nbr, backend):
        self.n_nodes = int(n_nodes)
        self.n_edges = int(edge_center.shape[0])
        self.edge_center = edge_center
        self.edge_nbr = edge_nbr
        self.backend = backend
        self.aux = backend.build(self)

    def rebuild(self, edge_center, edge_nbr):
        """Same sizes, new edges, into the SAME device buffers (a captured HIP
        graph keeps reading them): the per-step update of a graphed step."""
        if int(edge_center.shape[0]) != self.n_edges:
            raise ValueError('rebuild needs the same edge count')
        self.edge_center, self.edge_nbr = edge_center, edge_nbr
        self.backend.build(self, into=self.aux)


class HipConvBackend:
    """The kernels of libe3gnn_hip.so (include/e3gnn.h, training ops)."""

    def __init__(self):
        self.lib = _lib.load()
        self.small_max = int(self.lib.e3gnn_conv_graph_small_max_nodes())
        self.small_max_e = int(self.lib.e3gnn_conv_graph_small_max_edges())
        self.dims = {}
        for kind in (0, 1, 2):
            a, b, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
            _lib.check(self.lib.e3gnn_conv_dims(kind, a, b, c))
            self.dims[kind] = (a.value, b.value, c.value)

    @staticmethod
    def _stream(t):
        return torch.cuda.current_stream(t.device).cuda_stream

    def build(self, g, into=None):
        dev = g.edge_center.device
        if dev.type != 'cuda':
            raise _lib.E3GNNError(f'the HIP conv op needs device tensors, got {dev}')
        n, E = g.n_nodes, g.n_edges
        if into is None:
            aux = {'center': g.edge_center.to(torch.int32).contiguous(),
                   'nbr': g.edge_nbr.to(torch.int32).contiguous(),
                   'row_ptr': torch.empty(n + 1, dtype=torch.int32, device=dev),
                   'src_ptr': torch.empty(n + 1, dtype=torch.int32, device=dev),
                   'src_perm': torch.empty(max(E, 1), dtype=torch.int32, device=dev),
                   'scratch': torch.empty(n + 1, dtype=torch.int32, device=dev)}
        else:
            aux = into
            c, j = g.edge_center, g.edge_nbr
            if (c.dtype == torch.int64 and j.dtype == torch.int64 and c.is_contiguous() and j.is_contiguous()
                    and c.device == dev and n <= self.small_max and E <= self.small_max_e):
                # one launch: the int32 copies, the CSRs and the validation
                _lib.check(self.lib.e3gnn_conv_graph_i64(
                    n, E, c.data_ptr(), j.data_ptr(), aux['center'].data_ptr(), aux['nbr'].data_ptr(),
                    aux['row_ptr'].data_ptr(), aux['src_ptr'].data_ptr(), aux['src_perm'].data_ptr(),
                    aux['scratch'].data_ptr(), self._stream(aux['center'])))
                return aux
            aux['center'].copy_(c)
            aux['nbr'].copy_(j)
        _lib.check(self.lib.e3gnn_conv_graph(
            n, E, aux['center'].data_ptr(), aux['nbr'].data_ptr(), aux['row_ptr'].data_ptr(),
            aux['src_ptr'].data_ptr(), aux['src_perm'].data_ptr(), aux['scratch'].data_ptr(),
            self._stream(aux['center'])))
        return aux

    def _check(self, kind, g, h, Y, w):
        dx, dw, _ = self.dims[kind]
        for name, t, shape in (('h', h, (g.n_nodes, dx)), ('Y', Y, (g.n_edges, 9)),
                               ('w', w, (g.n_edges, dw))):
            if tuple(t.shape) != shape or t.dtype != torch.float32 or not t.is_cuda:
                raise _lib.E3GNNError(f'conv kind {kind}: {name} must be float32 {shape} on '
                                      f'the GPU, got {t.dtype} {tuple(t.shape)} on {t.device}')

    def forward(self, kind, g, h, Y, w, out=None, acc=False):
        """agg; ``acc``: add into ``out`` instead of overwriting it"""
        self._check(kind, g, h, Y, w)
        if acc and out is None:
            raise _lib.E3GNNError('conv forward: acc needs an output buffer')
        h, Y, w = h.contiguous(), Y.contiguous(), w.contiguous()
        agg = _out(out, (g.n_nodes, self.dims[kind][2]), h.device)
        a = g.aux
        _lib.check(self.lib.e3gnn_conv_forward_acc(
            kind, g.n_nodes, a['row_ptr'].data_ptr(), a['nbr'].data_ptr(), h.data_ptr(),
            Y.data_ptr(), w.data_ptr(), agg.data_ptr(), int(bool(acc)), self._stream(h)))
        return agg

    def backward(self, kind, g, h, Y, w, gagg, need_h=True, dh_out=None, dw_out=None,
                 dY_out=None, acc=0):
        """(dh, dY, dw); ``dh_out`` / ``dw_out`` / ``dY_out``: contiguous
        float32 buffers of the right shape to write dh / dw / dY into (the
        explicit fine-tune derivatives stack primal and tangent rows); ``acc``
        bits ACC_DH / ACC_DY / ACC_DW add into those buffers instead"""
        self._check(kind, g, h, Y, w)
        for bit, buf in ((ACC_DH, dh_out), (ACC_DY, dY_out), (ACC_DW, dw_out)):
            if acc & bit and buf is None:
                raise _lib.E3GNNError('conv backward: accumulation needs its output buffer')
        if acc & ACC_DH and not need_h:
            raise _lib.E3GNNError('conv backward: ACC_DH without need_h')
        dx, dwd, dm = self.dims[kind]
        h, Y, w = h.contiguous(), Y.contiguous(), w.contiguous()
        gagg = gagg.to(torch.float32).contiguous()
        if tuple(gagg.shape) != (g.n_nodes, dm):
            raise _lib.E3GNNError(f'conv kind {kind}: gagg must be {(g.n_nodes, dm)}')
        dev = h.device
        E = g.n_edges
        dY = _out(dY_out, (E, 9), dev)
        dw = _out(dw_out, (E, dwd), dev)
        dh = _out(dh_out, (g.n_nodes, dx), dev) if need_h else None
        dxc = torch.empty(E, dx, device=dev) if need_h and E else None
        a = g.aux
        _lib.check(self.lib.e3gnn_conv_backward_acc(
            kind, g.n_nodes, E, a['row_ptr'].data_ptr(), a['nbr'].data_ptr(),
            a['src_ptr'].data_ptr(), a['src_perm'].data_ptr(), h.data_ptr(), Y.data_ptr(),
            w.data_ptr(), gagg.data_ptr(), dh.data_ptr() if dh is not None else None,
            dY.data_ptr(), dw.data_ptr(), dxc.data_ptr() if dxc is not None else None,
            int(acc), self._stream(h)))
        return dh, dY, dw


    def tangent_forward(self, kind, g, h, hd, Y, Yd, w, wd, out, acc=False):
        """agg' = C(h, Y', w) + C(h, Y, w') + C(h', Y, w) into ``out`` (added
        with ``acc``); ``hd`` None: no h' term (e3gnn_conv_tangent_forward)"""
        self._check(kind, g, h, Y, w)
        self._check(kind, g, hd if hd is not None else h, Yd, wd)
        out = _out(out, (g.n_nodes, self.dims[kind][2]), h.device)
        a = g.aux
        _lib.check(self.lib.e3gnn_conv_tangent_forward(
            kind, g.n_nodes, a['row_ptr'].data_ptr(), a['nbr'].data_ptr(), h.data_ptr(),
            hd.data_ptr() if hd is not None else None, Y.data_ptr(), Yd.data_ptr(), w.data_ptr(),
            wd.data_ptr(), out.data_ptr(), int(bool(acc)), self._stream(h)))
        return out

    def dual_backward(self, kind, g, h, hd, Y, Yd, w, wd, ga, gad, dh_out, dhd_out, dw_out,
                      dwd_out):
        """The reverse of (agg, agg') for cotangents (ga, gad): writes
        dh = B_h(Y,w;ga) + B_h(Y',w;gad) + B_h(Y,w';gad), dh' = B_h(Y,w;gad),
        dw = B_w(h,Y;ga) + B_w(h,Y';gad) + B_w(h',Y;gad), dw' = B_w(h,Y;gad)
        (``hd`` / ``dhd_out`` None together: no h'); e3gnn_conv_dual_backward"""
        self._check(kind, g, h, Y, w)
        self._check(kind, g, hd if hd is not None else h, Yd, wd)
        if (hd is None) != (dhd_out is None):
            raise _lib.E3GNNError("dual conv backward: h' and dh' go together")
        dx, dwd, dm = self.dims[kind]
        n, E, dev = g.n_nodes, g.n_edges, h.device
        for t in (ga, gad):
            if tuple(t.shape) != (n, dm) or t.dtype != torch.float32 or not t.is_contiguous():
                raise _lib.E3GNNError(f'conv kind {kind}: cotangents must be contiguous float32 '
                                      f'{(n, dm)}')
        dh_out, dw_out, dwd_out = (_out(dh_out, (n, dx), dev), _out(dw_out, (E, dwd), dev),
                                   _out(dwd_out, (E, dwd), dev))
        if dhd_out is not None:
            dhd_out = _out(dhd_out, (n, dx), dev)
        dxc = torch.empty((2 if hd is not None else 1) * max(E, 1), dx, device=dev)
        a = g.aux
        ptr = lambda t: t.data_ptr() if t is not None else None   # noqa: E731
        _lib.check(self.lib.e3gnn_conv_dual_backward(
            kind, n, E, a['row_ptr'].data_ptr(), a['nbr'].data_ptr(), a['src_ptr'].data_ptr(),
            a['src_perm'].data_ptr(), h.data_ptr(), ptr(hd), Y.data_ptr(), Yd.data_ptr(),
            w.data_ptr(), wd.data_ptr(), ga.data_ptr(), gad.data_ptr(), dh_out.data_ptr(),
            ptr(dhd_out), dw_out.data_ptr(), dwd_out.data_ptr(), dxc.data_ptr(), self._stream(h)))
        return dh_out, dhd_out, dw_out, dwd_out


# accumulation bits of HipConvBackend.backward (e3gnn_conv_backward_acc)
ACC_DH, ACC_DY, ACC_DW = 1, 2, 4


def _out(buf, shape, device):
    """a caller's output buffer (checked), or a new one"""
    if buf is None:
        return torch.empty(*shape, device=device)
    if tuple(buf.shape) != tuple(shape) or buf.dtype != torch.float32 or not buf.is_contiguous():
        raise _lib.E3GNNError(f'output buffer must be contiguous float32 {tuple(shape)}, got '
                              f'{buf.dtype} {tuple(buf.shape)}')
    return buf


class GenericHipConvBackend(HipConvBackend):
    """Runtime path tables (gtp.hip, e3gnn_gtp_*): the convolution of any
    nequip-family block (irreps with parity, lmax <= 2), one table per block;
    ``kind`` is the block index.  Same build / forward / backward contract as
    the SevenNet-0 kernels, so the double-backward op above serves it too."""
    generic = True

    def __init__(self, tables=None):
        self.lib = _lib.load()
        self.dims, self.ydims, self.handles = {}, {}, []
        if tables is not None:
            self.configure(tables)

    def configure(self, tables):
        """tables: per block (paths int32 [P, 8], dx, dy, dw, dm) (nn.path_table)."""
        import numpy as np
        self._free()
        for k, (paths, dx, dy, dw, dm) in enumerate(tables):
            arr = np.ascontiguousarray(paths, dtype=np.int32)
            h = self.lib.e3gnn_gtp_create(len(arr), arr.ctypes.data, dx, dy, dw, dm)
            if not h:
                raise _lib.E3GNNError(f'gtp block {k}: {self.lib.e3gnn_last_error().decode()}')
            self.handles.append(h)
            self.dims[k] = (dx, dw, dm)
            self.ydims[k] = dy

    def _free(self):
        for h in getattr(self, 'handles', []):
            self.lib.e3gnn_gtp_free(h)
        self.handles = []

    def __del__(self):
        try:
            self._free()
        except Exception:
            pass

    def _check(self, kind, g, h, Y, w):
        dx, dw, _ = self.dims[kind]
        for name, t, shape in (('h', h, (g.n_nodes, dx)), ('Y', Y, (g.n_edges, self.ydims[kind])),
                               ('w', w, (g.n_edges, dw))):
            if tuple(t.shape) != shape or t.dtype != torch.float32 or not t.is_cuda:
                raise _lib.E3GNNError(f'gtp block {kind}: {name} must be float32 {shape} on the '
                                      f'GPU, got {t.dtype} {tuple(t.shape)} on {t.device}')

    def forward(self, kind, g, h, Y, w):
        self._check(kind, g, h, Y, w)
        h, Y, w = h.contiguous(), Y.contiguous(), w.contiguous()
        agg = torch.empty(g.n_nodes, self.dims[kind][2], device=h.device)
        a = g.aux
        _lib.check(self.lib.e3gnn_gtp_forward(
            self.handles[kind], g.n_nodes, a['row_ptr'].data_ptr(), a['nbr'].data_ptr(),
            h.data_ptr(), Y.data_ptr(), w.data_ptr(), agg.data_ptr(), self._stream(h)))
        return agg

    def backward(self, kind, g, h, Y, w, gagg, need_h=True):
        self._check(kind, g, h, Y, w)
        dx, dwd, dm = self.dims[kind]
        h, Y, w = h.contiguous(), Y.contiguous(), w.contiguous()
        gagg = gagg.to(torch.float32).contiguous()
        if tuple(gagg.shape) != (g.n_nodes, dm):
            raise _lib.E3GNNError(f'gtp block {kind}: gagg must be {(g.n_nodes, dm)}')
        dev, E = h.device, g.n_edges
        dY = torch.empty(E, self.ydims[kind], device=dev)
        dw = torch.empty(E, dwd, device=dev)
        dh = torch.empty(g.n_nodes, dx, device=dev) if need_h else None
        dxc = torch.empty(E, dx, device=dev) if need_h and E else None
        a = g.aux
        _lib.check(self.lib.e3gnn_gtp_backward(
            self.handles[kind], g.n_nodes, E, a['row_ptr'].data_ptr(), a['nbr'].data_ptr(),
            a['src_ptr'].data_ptr(), a['src_perm'].data_ptr(), h.data_ptr(), Y.data_ptr(),
            w.data_ptr(), gagg.data_ptr(), dh.data_ptr() if dh is not None else None,
            dY.data_ptr(), dw.data_ptr(), dxc.data_ptr() if dxc is not None else None,
            self._stream(h)))
        return dh, dY, dw

    # The one-launch tangent forward / dual backward exist for SevenNet-0's
    # three compile-time kinds only (kind there is 0/1/2, here a block index):
    # refuse instead of running the wrong kernel (train_explicit.supported()
    # keeps runtime-table models on the autograd path).
    def tangent_forward(self, *a, **k):
        raise _lib.E3GNNError('GenericHipConvBackend has no fused tangent forward: '
                              'runtime-table models train through autograd')

    def dual_backward(self, *a, **k):
        raise _lib.E3GNNError('GenericHipConvBackend has no fused dual backward: '
                              'runtime-table models train through autograd')


def _add(acc, t):
    if t is None:
        return acc
    return t if acc is None else acc + t


class _ConvForward(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, Y, w, kind, graph):
        ctx.save_for_backward(h, Y, w)
        ctx.kind, ctx.graph = kind, graph
        return graph.backend.forward(kind, graph, h, Y, w)

    @staticmethod
    def backward(ctx, g):
        h, Y, w = ctx.saved_tensors
        dh, dY, dw = _ConvBackward.apply(h, Y, w, g, ctx.kind, ctx.graph)
        return dh, dY, dw, None, None


class _ConvBackward(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, Y, w, g, kind, graph):
        ctx.save_for_backward(h, Y, w, g)
        ctx.kind, ctx.graph = kind, graph
        return graph.backend.backward(kind, graph, h, Y, w, g)

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, ah, aY, aw):
        h, Y, w, g = ctx.saved_tensors
        k, gr = ctx.kind, ctx.graph
        be = gr.backend
        gg = gh = gY = gw = None
        if ah is not None:
            gg = _add(gg, be.forward(k, gr, ah, Y, w))
            _, t_Y, t_w = be.backward(k, gr, ah, Y, w, g, need_h=False)
            gY, gw = _add(gY, t_Y), _add(gw, t_w)
        if aY is not None:
            gg = _add(gg, be.forward(k, gr, h, aY, w))
            t_h, _, t_w = be.backward(k, gr, h, aY, w, g)
            gh, gw = _add(gh, t_h), _add(gw, t_w)
        if aw is not None:
            gg = _add(gg, be.forward(k, gr, h, Y, aw))
            t_h, t_Y, _ = be.backward(k, gr, h, Y, aw, g)
            gh, gY = _add(gh, t_h), _add(gY, t_Y)
        return gh, gY, gw, gg, None, None


def conv(h, Y, w, kind, graph):
    """Raw (un-normalised) aggregated messages of one interaction block."""
    return _ConvForward.apply(h, Y, w, kind, graph)


# ------------------------------------------------------------------ scaled SiLU
def _act_call(lib, op, x, g=None, gg=None, out0=None, out1=None, scale=1.0):
    p = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
    _lib.check(lib.e3gnn_act(op, x.numel(), p(x), p(g), p(gg), p(out0), p(out1),
                             ctypes.c_float(scale), torch.cuda.current_stream(x.device).cuda_stream))


class _Act(torch.autograd.Function):
    # the INPUT tensors are saved (not their contiguous copies): the double
    # backward must reach the original x through them
    @staticmethod
    def forward(ctx, x, scale, lib):
        xc = x.contiguous()
        y = torch.empty_like(xc)
        _act_call(lib, 0, xc, out0=y, scale=scale)
        ctx.save_for_backward(x)
        ctx.scale, ctx.lib = scale, lib
        return y

    @staticmethod
    def backward(ctx, g):
        x, = ctx.saved_tensors
        return _ActBackward.apply(x, g, ctx.scale, ctx.lib), None, None


class _ActBackward(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g, scale, lib):
        xc, gc = x.contiguous(), g.contiguous()
        dx = torch.empty_like(xc)
        _act_call(lib, 1, xc, g=gc, out0=dx, scale=scale)
        ctx.save_for_backward(x, g)
        ctx.scale, ctx.lib = scale, lib
        return dx

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, gg):
        x, g = ctx.saved_tensors
        xc, gc, ggc = x.contiguous(), g.contiguous(), gg.contiguous()
        need_x, need_g = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        dx = torch.empty_like(xc) if need_x else None
        dg = torch.empty_like(xc) if need_g else None
        if need_x or need_g:
            _act_call(ctx.lib, 2, xc, g=gc, gg=ggc, out0=dx, out1=dg, scale=ctx.scale)
        return dx, dg, None, None


def scaled_silu(x, scale, lib):
    """scale * silu(x) on the HIP kernels of libe3gnn_hip.so (e3gnn_act),
    differentiable twice (the fine-tune step's force loss)."""
    return _Act.apply(x, float(scale), lib)


# ------------------------------------------------------------------ gate
def _gate_call(lib, op, dims, y, go=None, q=None, out0=None, out1=None, scale=1.0):
    p = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
    _lib.check(lib.e3gnn_gate(op, y.shape[0], dims.ctypes.data, p(y), p(go), p(q), p(out0),
                              p(out1), ctypes.c_float(scale),
                              torch.cuda.current_stream(y.device).cuda_stream))


class _Gate(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, dims, scale, lib):
        yc = y.contiguous()
        o = torch.empty(y.shape[0], int(dims[3]), device=y.device, dtype=y.dtype)
        _gate_call(lib, 0, dims, yc, out0=o, scale=scale)
        ctx.save_for_backward(y)
        ctx.dims, ctx.scale, ctx.lib = dims, scale, lib
        return o

    @staticmethod
    def backward(ctx, go):
        y, = ctx.saved_tensors
        return _GateBackward.apply(y, go, ctx.dims, ctx.scale, ctx.lib), None, None, None


class _GateBackward(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, go, dims, scale, lib):
        yc, gc = y.contiguous(), go.contiguous()
        dy = torch.empty_like(yc)
        _gate_call(lib, 1, dims, yc, go=gc, out0=dy, scale=scale)
        ctx.save_for_backward(y, go)
        ctx.dims, ctx.scale, ctx.lib = dims, scale, lib
        return dy

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, q):
        y, go = ctx.saved_tensors
        yc, gc, qc = y.contiguous(), go.contiguous(), q.contiguous()
        need_y, need_go = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        dgo = torch.empty_like(gc) if need_go else None
        dyy = torch.empty_like(yc) if need_y else None
        if need_y or need_go:
            _gate_call(ctx.lib, 2, ctx.dims, yc, go=gc, q=qc, out0=dgo, out1=dyy,
                       scale=ctx.scale)
        return dyy, dgo, None, None, None


def _act_dual_call(lib, x, xd, g, gd, og, ogd, scale):
    """e3gnn_act_dual: reverse of (act(x), act'(x) xd) (train_explicit.py)"""
    c = lambda t: t.contiguous()   # noqa: E731
    x, xd, g, gd = c(x), c(xd), c(g), c(gd)
    _lib.check(lib.e3gnn_act_dual(x.numel(), x.data_ptr(), xd.data_ptr(), g.data_ptr(),
                                  gd.data_ptr(), og.data_ptr(), ogd.data_ptr(), ctypes.c_float(scale),
                                  torch.cuda.current_stream(x.device).cuda_stream))


def _gate_dual_call(lib, op, dims, y, yd, xb=None, xdb=None, out0=None, out1=None, scale=1.0):
    """e3gnn_gate_dual: op 0 out0 = J yd; op 1 out0 = J^T xb + d/dy <xdb, J yd>,
    out1 = J^T xdb (train_explicit.py)"""
    p = lambda t: t.contiguous().data_ptr() if t is not None else None  # noqa: E731

    def o(t, name):   # outputs are written in place: a contiguous copy would be lost
        if t is None:
            return None
        if not t.is_contiguous():
            raise _lib.E3GNNError(f'e3gnn_gate_dual: {name} must be contiguous')
        return t.data_ptr()
    _lib.check(lib.e3gnn_gate_dual(op, y.shape[0], dims.ctypes.data, p(y), p(yd), p(xb), p(xdb),
                                   o(out0, 'out0'), o(out1, 'out1'), ctypes.c_float(scale),
                                   torch.cuda.current_stream(y.device).cuda_stream))


def gate_dims(scal, gated):
    """dims vector of e3gnn_gate for Gate irreps (scalars, gated (mul, l))."""
    import numpy as np
    ns = sum(m for m, _ in scal)
    ng = sum(m for m, _ in gated)
    if len(gated) > 2:
        raise ValueError('the fused gate takes at most two gated irreps')
    din = ns + ng + sum(m * (2 * l + 1) for m, l in gated)
    dout = ns + sum(m * (2 * l + 1) for m, l in gated)
    d = [ns, ng, din, dout, len(gated)]
    off_in, off_out = ns + ng, ns
    for m, l in gated:
        d += [off_in, off_out, m, 2 * l + 1]
        off_in += m * (2 * l + 1)
        off_out += m * (2 * l + 1)
    d += [0] * (13 - len(d))
    return np.asarray(d, dtype=np.int32)


def gate(y, dims, scale, lib):
    """e3nn Gate (scale * silu on scalars and gates) on the HIP kernels,
    differentiable twice."""
    return _Gate.apply(y, dims, float(scale), lib)
