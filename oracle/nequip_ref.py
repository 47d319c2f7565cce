"""Plain-PyTorch CPU restatement of the reference's ``nequip``-type E(3)
equivariant model for ANY deployment manifest of this build -- irreps with
parity, lmax <= 2, XPLOR or polynomial cutoff, normalised or raw spherical
harmonics, ``linear`` or ``nequip`` self-connection, parity-dependent gate
activations.  The HfO2 example deployment (sevenn 0.8.6) and SevenNet-0
(0.9.1) are both instances.

TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py.  Never imported by the
product package.

Reference modules (pipeline order, sevenn/model_build.py:186-445):

  EdgePreprocess            nn/edge_embedding.py:24-77
  BesselBasis               :80-116      PolynomialCutoff :119-145
  XPLORCutoff               :148-173     SphericalEncoding :177-198
                            (e3nn SH, component norm; ``normalize`` is False for
                            checkpoints older than the ``_normalize_sph`` key,
                            util.py:143-144)
  OnehotEmbedding + embed   nn/node_embedding.py:15-48, nn/linear.py:14-49
  per block (interaction_blocks.py:22-86):
    SelfConnectionIntro     nn/self_connection.py:11-38  (e3nn
                            FullyConnectedTensorProduct(x, one-hot), 'nequip')
    SelfConnectionLinearIntro :42-62 ('linear')
    IrrepsLinear si1        nn/linear.py:46-49
    IrrepsConvolution       nn/convolution.py:36-123 (instructions: every
                            (x irrep, filter irrep, output) with the output in
                            the block's output irreps, :72-95; mid irreps
                            stable-sorted by (l, p); uvu; / denominator)
    IrrepsLinear si2, SelfConnectionOutro :106-109
    EquivariantGate         nn/equivariant_gate.py:13-61 (scalars: act_scalar by
                            parity; gates: act_gate)
  readout linears           model_build.py:374-395, or FCN_e3nn
                            (readout_as_fcn, :396-408; nn/linear.py:94-129)
  biases (use_bias_in_linear) e3nn o3.Linear(biases=True): + b on 0e outputs of
                            the embedding, si1, si2 and readout linears
                            (model_build.py:194, :386, :393;
                            interaction_blocks.py:58, :80)
  (SpeciesWise)Rescale      nn/scale.py:12-73, AtomReduce nn/linear.py:53-90
  ForceStressOutput         nn/force_output.py:74-130

e3nn conventions restated: ``Irreps.sort`` orders irreps by (l, p) with odd
before even (0o < 0e < 1o < 1e); ``o3.Linear`` blocks connect equal (l, p),
weight (mul_in, mul_out) row-major per (i_in, i_out) in i_in-major order, path
weight 1/sqrt(sum of mul_in into i_out); ``FullyConnectedTensorProduct`` with a
scalar operand: per (i_x, i_out) of equal irrep a (mul_x, mul_op, mul_out)
block, path weight 1/sqrt(sum of mul_x * mul_op into i_out); uvu TP coupling
= wigner_3j * sqrt(2 l3 + 1) (oracle/cg.py).
"""
import json
import math
import os

import numpy as np
import torch

from .cg import tp_cg


def parse_irreps(s):
    """'4x0o+4x1e' -> [(4, 0, -1), (4, 1, 1)]"""
    out = []
    for term in str(s).split('+'):
        mul, ir = term.strip().split('x')
        out.append((int(mul), int(ir[:-1]), 1 if ir[-1] == 'e' else -1))
    return out


def dim(irreps):
    return sum(m * (2 * l + 1) for m, l, _ in irreps)


def offsets(irreps):
    return np.cumsum([0] + [m * (2 * l + 1) for m, l, _ in irreps]).tolist()


def simplify(irreps):
    out = []
    for m, l, p in irreps:
        if out and out[-1][1:] == (l, p):
            out[-1] = (out[-1][0] + m, l, p)
        else:
            out.append((m, l, p))
    return out


def gate_irreps(irreps_out):
    """EquivariantGate (equivariant_gate.py:30-51) + e3nn Gate: scalars (the
    l = 0 irreps of the output), one gate scalar per gated channel (parity +1
    when 0e is among the scalars, else -1, :41), the gated irreps; e3nn's Gate
    stable-sorts [scalars | gates | gated] by (l, p) and merges neighbours.
    Returns (irreps_in, scalars, gated, gate parity, offset of every piece in
    the sorted row)."""
    scal = [(m, l, p) for m, l, p in irreps_out if l == 0]
    gated = [(m, l, p) for m, l, p in irreps_out if l > 0]
    ng = sum(m for m, _, _ in gated)
    gp = 1 if (0, 1) in [(l, p) for _, l, p in scal] else -1
    pieces = scal + ([(ng, 0, gp)] if ng else []) + gated
    order = sorted(range(len(pieces)), key=lambda i: pieces[i][1:])
    offs, off = [0] * len(pieces), 0
    for i in order:
        offs[i] = off
        off += pieces[i][0] * (2 * pieces[i][1] + 1)
    return simplify([pieces[i] for i in order]), scal, gated, gp, offs


def conv_instructions(irreps_x, lmax_filter, filter_parity, irreps_out):
    """convolution.py:72-95: (i_x, l2, l3, p3, mul) in weight order; the mid
    irreps are these outputs stable-sorted by (l3, p3); perm[k] = slot of k."""
    allowed = {(l, p) for _, l, p in irreps_out}
    ins = []
    for i, (mul, l1, p1) in enumerate(irreps_x):
        for l2 in range(lmax_filter + 1):
            p2 = filter_parity ** l2
            for l3 in range(abs(l1 - l2), l1 + l2 + 1):
                if (l3, p1 * p2) in allowed:
                    ins.append((i, l2, l3, p1 * p2, mul))
    order = sorted(range(len(ins)), key=lambda k: (ins[k][2], ins[k][3], k))
    perm = [0] * len(ins)
    for slot, k in enumerate(order):
        perm[k] = slot
    mid = [(ins[k][4], ins[k][2], ins[k][3]) for k in order]
    return ins, mid, perm


def spherical_harmonics(vec, lmax, normalize):
    """e3nn SphericalHarmonics, component normalisation, l <= 2
    (edge_embedding.py:177-198): the l-th block is a homogeneous polynomial of
    degree l in the (optionally normalised) vector."""
    u = vec / vec.norm(dim=-1, keepdim=True) if normalize else vec
    x, y, z = u[:, 0], u[:, 1], u[:, 2]
    s3, s5 = math.sqrt(3.0), math.sqrt(5.0)
    parts = [torch.ones_like(x)]
    if lmax >= 1:
        parts += [s3 * x, s3 * y, s3 * z]
    if lmax >= 2:
        parts += [s5 * s3 * x * z, s5 * s3 * x * y, s5 * (y * y - 0.5 * (x * x + z * z)),
                  s5 * s3 * y * z, s5 * 0.5 * s3 * (z * z - x * x)]
    return torch.stack(parts, dim=-1)


def e3nn_linear(x, irreps_in, irreps_out, w_flat):
    n = x.shape[0]
    ins = [(i, j) for i, (_, li, pi) in enumerate(irreps_in)
           for j, (_, lo, po) in enumerate(irreps_out) if (li, pi) == (lo, po)]
    fan = {}
    for i, j in ins:
        fan[j] = fan.get(j, 0) + irreps_in[i][0]
    io, oo = offsets(irreps_in), offsets(irreps_out)
    outs = [torch.zeros(n, m, 2 * l + 1, dtype=x.dtype) for m, l, _ in irreps_out]
    woff = 0
    for i, j in ins:
        mi, l, _ = irreps_in[i]
        mo = irreps_out[j][0]
        w = torch.as_tensor(w_flat[woff:woff + mi * mo].reshape(mi, mo), dtype=x.dtype)
        woff += mi * mo
        xi = x[:, io[i]:io[i + 1]].reshape(n, mi, 2 * l + 1)
        outs[j] = outs[j] + torch.einsum('zui,uw->zwi', xi, w) / math.sqrt(fan[j])
    assert woff == w_flat.size, (woff, w_flat.size)
    return torch.cat([o.reshape(n, -1) for o in outs], dim=1)


def add_bias(y, irreps_out, b):
    """e3nn o3.Linear(biases=True) (IrrepsLinear biases=use_bias_in_linear,
    model_build.py:194, :237, :386, :393): + b on the channels of every 0e
    output irrep, in output order"""
    if b is None:
        return y
    b = torch.as_tensor(b, dtype=y.dtype).reshape(-1)
    oo = offsets(irreps_out)
    parts, k = [], 0
    for j, (m, l, p) in enumerate(irreps_out):
        blk = y[:, oo[j]:oo[j + 1]]
        if (l, p) == (0, 1):
            blk = blk + b[k:k + m]
            k += m
        parts.append(blk)
    assert k == b.numel(), (k, b.numel())
    return torch.cat(parts, dim=1)


def fctp_scalar(x, irreps_in, onehot, irreps_out, w_flat):
    """FullyConnectedTensorProduct(x, nsp x 0e -> irreps_out)
    (self_connection.py:11-38): per (i_x, i_out) of equal irrep a
    (mul_x, nsp, mul_out) weight block."""
    n, nsp = x.shape[0], onehot.shape[1]
    ins = [(i, j) for i, (_, li, pi) in enumerate(irreps_in)
           for j, (_, lo, po) in enumerate(irreps_out) if (li, pi) == (lo, po)]
    fan = {}
    for i, j in ins:
        fan[j] = fan.get(j, 0) + irreps_in[i][0] * nsp
    io = offsets(irreps_in)
    outs = [torch.zeros(n, m, 2 * l + 1, dtype=x.dtype) for m, l, _ in irreps_out]
    woff = 0
    for i, j in ins:
        mi, l, _ = irreps_in[i]
        mo = irreps_out[j][0]
        w = torch.as_tensor(w_flat[woff:woff + mi * nsp * mo].reshape(mi, nsp, mo), dtype=x.dtype)
        woff += mi * nsp * mo
        xi = x[:, io[i]:io[i + 1]].reshape(n, mi, 2 * l + 1)
        outs[j] = outs[j] + torch.einsum('zui,zs,usw->zwi', xi, onehot, w) / math.sqrt(fan[j])
    assert woff == w_flat.size, (woff, w_flat.size)
    return torch.cat([o.reshape(n, -1) for o in outs], dim=1)


class NequIPRef:
    """Energy / forces / stress of a deployment (manifest.json + weights.bin)."""

    def __init__(self, model_dir, dtype=torch.float64):
        with open(os.path.join(model_dir, 'manifest.json')) as f:
            self.man = man = json.load(f)
        flat = np.fromfile(os.path.join(model_dir, 'weights.bin'), dtype='<f4')
        self.p = {t['name']: flat[t['offset']:t['offset'] + t['numel']].reshape(t['shape']).copy()
                  for t in man['tensors']}
        self.dtype = dtype
        self.symbols = man['chemical_symbols']
        self.nsp = len(self.symbols)
        self.cutoff = float(man['cutoff'])
        self.cut = man['cutoff_function']
        self.irreps = [parse_irreps(s) for s in man['irreps_manual']]
        self.conv_out = [parse_irreps(s) for s in man['conv_irreps_out']] \
            if 'conv_irreps_out' in man else self.irreps[1:]
        self.nlayer = int(man['num_convolution_layer'])
        self.lmax_edge = int(man.get('lmax_edge', man['lmax']))
        self.filter_parity = -1 if man['is_parity'] else 1
        self.sh_normalize = bool(man.get('sh_normalize', True))
        self.sc_type = man.get('self_connection_type', 'linear')
        norm = man.get('act_norm', {'silu': man['silu_norm']})
        self.silu_norm = float(norm['silu'])
        self.tanh_norm = float(norm.get('tanh', 1.0))
        a_s = man.get('act_scalar', 'silu')
        a_g = man.get('act_gate', 'silu')
        self.act_scalar = a_s if isinstance(a_s, dict) else {'e': a_s, 'o': 'tanh'}
        self.act_gate = a_g if isinstance(a_g, dict) else {'e': a_g, 'o': 'tanh'}
        last = self.irreps[-1]
        self.hidden = int(man.get('readout_hidden', sum(m for m, _, _ in last) // 2))

    def t(self, name):
        return torch.as_tensor(self.p[name], dtype=self.dtype)

    def lin(self, x, irreps_in, irreps_out, name):
        """IrrepsLinear `name` (weight, + bias when the deployment has one)"""
        y = e3nn_linear(x, irreps_in, irreps_out, self.p[f'{name}.linear.weight'])
        return add_bias(y, irreps_out, self.p.get(f'{name}.linear.bias'))

    def act(self, name, x):
        if name == 'silu':
            return torch.nn.functional.silu(x) * self.silu_norm
        if name == 'tanh':
            return torch.tanh(x) * self.tanh_norm
        raise ValueError(name)

    def readout_fcn(self, x):
        """FCN_e3nn readout (nn/linear.py:94-129): e3nn FullyConnectedNet
        [dim] + hidden + [1], h <- c act(h W_k / sqrt(fan_in)) between layers
        (c = normalize2mom(act), the manifest's act_norm), no activation last"""
        ro = self.man['readout']
        f = {'relu': torch.relu, 'silu': torch.nn.functional.silu, 'tanh': torch.tanh,
             'sigmoid': torch.sigmoid, 'abs': torch.abs,
             'elu': torch.nn.functional.elu}[ro['act']]
        c = float(ro['act_norm'])
        h = x
        nh = len(ro['hidden'])
        for k in range(nh + 1):
            w = self.t(f'readout_FCN.fcn.layer{k}.weight')
            h = h @ (w / math.sqrt(w.shape[0]))
            if k < nh:
                h = f(h) * c
        return h

    def edge_embedding(self, r):
        rc = self.cutoff
        ur = r.unsqueeze(-1)
        bessel = (2.0 / rc) * torch.sin(self.t('edge_embedding.basis_function.coeffs') * ur) / ur
        if self.cut['name'] == 'poly_cut':   # edge_embedding.py:131-145
            p = float(self.cut['p'])
            x = r / rc
            env = (1.0 - (p + 1.0) * (p + 2.0) / 2.0 * x ** p + p * (p + 2.0) * x ** (p + 1)
                   - p * (p + 1.0) / 2.0 * x ** (p + 2))
            env = env * (x < 1.0)
        else:                                # XPLOR, :163-173
            ron = float(self.cut['cutoff_on'])
            r2 = r * r
            env = torch.where(r < ron, torch.ones_like(r),
                              (rc * rc - r2) ** 2 * (rc * rc + 2 * r2 - 3 * ron * ron)
                              / (rc * rc - ron * ron) ** 3)
        return bessel * env.unsqueeze(-1)

    def gate(self, y, irreps_out):
        _, scal, gated, gp, offs = gate_irreps(irreps_out)
        n = y.shape[0]
        outs = []
        for k, (m, l, p) in enumerate(scal):
            outs.append(self.act(self.act_scalar['e' if p == 1 else 'o'],
                                 y[:, offs[k]:offs[k] + m]))
        if gated:
            ng = sum(m for m, _, _ in gated)
            o = offs[len(scal)]
            g = self.act(self.act_gate['e' if gp == 1 else 'o'], y[:, o:o + ng])
            goff = 0
            for k, (m, l, _) in enumerate(gated):
                d = 2 * l + 1
                o = offs[len(scal) + 1 + k]
                blk = y[:, o:o + m * d].reshape(n, m, d)
                outs.append((g[:, goff:goff + m].unsqueeze(-1) * blk).reshape(n, -1))
                goff += m
        return torch.cat(outs, dim=1)

    def convolution(self, t, x, emb, sh, src, dst, irreps_x, irreps_out):
        pre = f'{t}_convolution'
        hid = [int(h) for h in self.man['weight_nn_hidden_neurons']]
        h = emb
        dims = [emb.shape[1]] + hid
        for k in range(len(hid)):
            h = self.act('silu', h @ (self.t(f'{pre}.weight_nn.layer{k}.weight') / math.sqrt(dims[k])))
        w = h @ (self.t(f'{pre}.weight_nn.layer{len(hid)}.weight') / math.sqrt(dims[-1]))
        ins, mid, perm = conv_instructions(irreps_x, self.lmax_edge, self.filter_parity, irreps_out)
        assert w.shape[1] == sum(i[4] for i in ins)
        xs = x[src]
        e = xs.shape[0]
        xo = offsets(irreps_x)
        outs = [None] * len(ins)
        woff = 0
        for k, (i, l2, l3, _, mul) in enumerate(ins):
            l1 = irreps_x[i][1]
            xi = xs[:, xo[i]:xo[i + 1]].reshape(e, mul, 2 * l1 + 1)
            y = sh[:, l2 * l2:(l2 + 1) ** 2]
            c = torch.as_tensor(tp_cg(l1, l2, l3), dtype=self.dtype)
            msg = torch.einsum('eui,ej,ijk->euk', xi, y, c) * w[:, woff:woff + mul].unsqueeze(-1)
            woff += mul
            outs[perm[k]] = msg.reshape(e, -1)
        msg = torch.cat(outs, dim=1)
        agg = torch.zeros(x.shape[0], msg.shape[1], dtype=self.dtype).index_add(0, dst, msg)
        return agg / self.t(f'{pre}.denominator')[0], mid

    def energy(self, pos, types, edge_index, shift, cell, with_stress=True):
        dt = self.dtype
        pos, cell = pos.to(dt), cell.to(dt)
        strain = torch.zeros(3, 3, dtype=dt, requires_grad=with_stress)
        sym = 0.5 * (strain + strain.t())
        pos_s = pos + pos @ sym
        cell_s = cell + cell @ sym
        src, dst = edge_index[0], edge_index[1]
        vec = pos_s[dst] - pos_s[src] + shift.to(dt) @ cell_s
        emb = self.edge_embedding(vec.norm(dim=-1))
        sh = spherical_harmonics(vec, self.lmax_edge, self.sh_normalize)
        onehot = torch.nn.functional.one_hot(types, self.nsp).to(dt)
        x = (onehot @ self.t('onehot_to_feature_x.linear.weight').reshape(self.nsp, -1)) \
            / math.sqrt(self.nsp)
        x = add_bias(x, self.irreps[0], self.p.get('onehot_to_feature_x.linear.bias'))
        for t in range(self.nlayer):
            irr_x, irr_out = self.irreps[t], self.irreps[t + 1]
            gin = gate_irreps(irr_out)[0]
            if self.sc_type == 'nequip':
                sc = fctp_scalar(x, irr_x, onehot, gin,
                                 self.p[f'{t}_self_connection_intro.fc_tensor_product.weight'])
            else:
                sc = e3nn_linear(x, irr_x, gin, self.p[f'{t}_self_connection_intro.linear.weight'])
            h = self.lin(x, irr_x, irr_x, f'{t}_self_interaction_1')
            # edge_index[1] is the gathered source, [0] the target (convolution.py:111-113)
            # the convolution's output irreps (model_build.py:303-315); without
            # the key (sevenn < 0.9 deployments) the block's irreps_manual
            agg, mid = self.convolution(t, h, emb, sh, dst, src, irr_x, self.conv_out[t])
            y = self.lin(agg, mid, gin, f'{t}_self_interaction_2') + sc
            x = self.gate(y, irr_out)
        if self.man.get('readout', {}).get('type', 'linear') == 'fcn':
            e_s = self.readout_fcn(x)
        else:
            hid = self.lin(x, self.irreps[-1], [(self.hidden, 0, 1)], 'reduce_input_to_hidden')
            e_s = self.lin(hid, [(self.hidden, 0, 1)], [(1, 0, 1)], 'reduce_hidden_to_energy')
        atomic = e_s[:, 0] * self.t('rescale_atomic_energy.scale')[types] + \
            self.t('rescale_atomic_energy.shift')[types]
        return {'energy': atomic.sum(), 'atomic_energy': atomic, 'strain': strain}

    def __call__(self, pos, types, edge_index, shift, cell, with_stress=True):
        pos = pos.detach().to(self.dtype).requires_grad_(True)
        out = self.energy(pos, types, edge_index, shift, cell, with_stress)
        wrt = [pos, out['strain']] if with_stress else [pos]
        grads = torch.autograd.grad(out['energy'], wrt, allow_unused=True)
        res = {'energy': out['energy'].detach(), 'atomic_energy': out['atomic_energy'].detach(),
               'forces': -grads[0]}
        if with_stress:
            vol = torch.abs(torch.det(cell.to(self.dtype)))
            s = -grads[1] / vol
            res['stress'] = torch.stack([s[0, 0], s[1, 1], s[2, 2], s[0, 1], s[1, 2], s[0, 2]])
        return res
