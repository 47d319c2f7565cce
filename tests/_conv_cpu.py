"""CPU test double of conv_ops.HipConvBackend (TEST INFRASTRUCTURE).

Implements the same three methods (build / forward / backward) with the
oracle's uvu tensor product (oracle/sevennet_ref.py, convolution.py:104-123)
and torch autograd for the operand gradients, in any dtype.  Used to check the
host logic of the trainable model and trainer on the CPU, and -- in float64 --
as the reference the HIP training path is compared with on the GPU.
"""
import numpy as np
import torch

from oracle.cg import tp_cg
from oracle.sevennet_ref import conv_instructions

X_FIRST = [(128, 0)]
X_MID = [(128, 0), (64, 1), (32, 2)]
KINDS = {0: (X_FIRST, 2), 1: (X_MID, 2), 2: (X_MID, 0)}


class CpuConvBackend:
    def __init__(self):
        self.dims = {}
        self.tables = {}
        for kind, (irr, lmax) in KINDS.items():
            ins, mid, perm = conv_instructions(irr, lmax)
            dx = sum(m * (2 * l + 1) for m, l in irr)
            self.dims[kind] = (dx, sum(i[3] for i in ins), sum(m * (2 * l + 1) for m, l in mid))
            self.tables[kind] = (irr, ins, perm)

    def build(self, g, into=None):
        return {} if into is None else into

    def forward(self, kind, g, h, Y, w, out=None, acc=False):
        agg = self._forward(kind, g, h, Y, w)
        if out is not None:
            if acc:
                return out.add_(agg)
            out.copy_(agg)
            return out
        assert not acc
        return agg

    def _forward(self, kind, g, h, Y, w):
        irr, ins, perm = self.tables[kind]
        xs = h[g.edge_nbr.long()]
        e = xs.shape[0]
        x_off = np.cumsum([0] + [m * (2 * l + 1) for m, l in irr])
        sh_off = [0, 1, 4, 9]
        outs = [None] * len(ins)
        woff = 0
        for k, (i, l2, l3, mul) in enumerate(ins):
            l1 = irr[i][1]
            xi = xs[:, x_off[i]:x_off[i + 1]].reshape(e, mul, 2 * l1 + 1)
            y = Y[:, sh_off[l2]:sh_off[l2 + 1]]
            c = torch.as_tensor(tp_cg(l1, l2, l3), dtype=h.dtype)
            m = torch.einsum('eui,ej,ijk->euk', xi, y, c) * w[:, woff:woff + mul].unsqueeze(-1)
            woff += mul
            outs[perm[k]] = m.reshape(e, -1)
        msg = torch.cat(outs, dim=1)
        return torch.zeros(g.n_nodes, msg.shape[1], dtype=h.dtype).index_add(
            0, g.edge_center.long(), msg)

    def backward(self, kind, g, h, Y, w, gagg, need_h=True, dh_out=None, dw_out=None,
                 dY_out=None, acc=0):
        with torch.enable_grad():
            hh, YY, ww = (t.detach().requires_grad_(True) for t in (h, Y, w))
            s = (self._forward(kind, g, hh, YY, ww) * gagg.detach()).sum()
            dh, dY, dw = torch.autograd.grad(s, [hh, YY, ww], allow_unused=True)
        zero = torch.zeros_like
        dh = dh if dh is not None else zero(h)
        dY = dY if dY is not None else zero(Y)
        dw = dw if dw is not None else zero(w)
        # accumulation bits as conv_ops.ACC_DH / ACC_DY / ACC_DW
        def put(buf, v, bit):
            if buf is None:
                assert not acc & bit
                return v
            return buf.add_(v) if acc & bit else buf.copy_(v)
        dw = put(dw_out, dw, 4)
        dY = put(dY_out, dY, 2)
        if need_h:
            dh = put(dh_out, dh, 1)
        return (dh if need_h else None), dY, dw


def _tangent_forward(self, kind, g, h, hd, Y, Yd, w, wd, out, acc=False):
    """the fused tangent forward as its three trilinear terms (the HIP
    e3gnn_conv_tangent_forward's definition)"""
    t = self._forward(kind, g, h, Yd, w) + self._forward(kind, g, h, Y, wd)
    if hd is not None:
        t = t + self._forward(kind, g, hd, Y, w)
    return out.add_(t) if acc else out.copy_(t)


def _dual_backward(self, kind, g, h, hd, Y, Yd, w, wd, ga, gad, dh_out, dhd_out, dw_out, dwd_out):
    """the fused dual backward as four backward products (the HIP
    e3gnn_conv_dual_backward's definition)"""
    dh, _, dw = self.backward(kind, g, h, Y, w, ga)
    t_h, _, t_w = self.backward(kind, g, h, Yd, w, gad)
    dh, dw = dh + t_h, dw + t_w
    t_h, _, dwd = self.backward(kind, g, h, Y, wd, gad)
    dh = dh + t_h
    if hd is not None:
        dhd, _, t_w = self.backward(kind, g, hd, Y, w, gad)
        dw = dw + t_w
        dhd_out.copy_(dhd)
    dh_out.copy_(dh)
    dw_out.copy_(dw)
    dwd_out.copy_(dwd)
    return dh_out, dhd_out, dw_out, dwd_out


CpuConvBackend.tangent_forward = _tangent_forward
CpuConvBackend.dual_backward = _dual_backward


class GenericCpuConvBackend:
    """CPU double of conv_ops.GenericHipConvBackend: the runtime path tables
    (nn.path_table rows: l1, l2, l3, mul, x/Y/w/agg offsets) evaluated with
    the oracle's coupling tables, any dtype."""
    generic = True

    def __init__(self):
        self.dims, self.tables = {}, {}

    def configure(self, tables):
        for k, (paths, dx, dy, dw, dm) in enumerate(tables):
            self.dims[k] = (dx, dw, dm)
            self.tables[k] = (np.asarray(paths), dm)

    def build(self, g, into=None):
        return {} if into is None else into

    def forward(self, kind, g, h, Y, w):
        paths, dm = self.tables[kind]
        xs = h[g.edge_nbr.long()]
        e = xs.shape[0]
        msg = torch.zeros(e, dm, dtype=h.dtype)
        for l1, l2, l3, mul, xo, yo, wo, mo in paths.tolist():
            xi = xs[:, xo:xo + mul * (2 * l1 + 1)].reshape(e, mul, 2 * l1 + 1)
            c = torch.as_tensor(tp_cg(l1, l2, l3), dtype=h.dtype)
            m = torch.einsum('eui,ej,ijk->euk', xi, Y[:, yo:yo + 2 * l2 + 1], c) * \
                w[:, wo:wo + mul].unsqueeze(-1)
            msg = msg.index_add(1, torch.arange(mo, mo + mul * (2 * l3 + 1)), m.reshape(e, -1))
        return torch.zeros(g.n_nodes, dm, dtype=h.dtype).index_add(0, g.edge_center.long(), msg)

    _forward = forward
    backward = CpuConvBackend.backward
