"""Trainable SevenNet-0 on the HIP convolution op -- the model the fine-tune
step differentiates (BASELINE config 5).

Mirrors the reference's training-mode ``AtomGraphSequential``
(sevenn/model_build.py:186-445 with ``set_is_batch_data(True)``,
trainer.py:18-27):

  EdgeEmbedding        edge_embedding.py:220-230  (BesselBasis :85-116 with
                       trainable coeffs, XPLORCutoff :163-173, SphericalEncoding
                       :177-198)  -- on a precomputed, grad-requiring edge_vec
                       (dataset.py:177-185, collate.py:49)
  OnehotEmbedding      node_embedding.py:39-48, linear.py:37-44
  5 x interaction      interaction_blocks.py:22-86: SelfConnectionLinearIntro,
                       IrrepsLinear si1, IrrepsConvolution (radial MLP + uvu TP +
                       neighbour sum / denominator, convolution.py:104-123),
                       IrrepsLinear si2, SelfConnectionOutro, EquivariantGate
  readout              model_build.py:374-408, SpeciesWiseRescale scale.py:67-73,
                       AtomReduce linear.py:76-90 (per graph)
  ForceStressOutputFromEdge  force_output.py:158-215 (create_graph while training)

The tensor product + neighbour sum runs in libe3gnn_hip.so through
``conv_ops.conv`` (double-backward capable); the dense e3nn linears and the
radial MLP are plain GEMMs (hipBLASLt through torch) and the element-wise
pieces are torch plumbing.  Parameter names, shapes and order are the
reference's ``named_parameters()`` (so the reference's ``state_dict``,
``fisher_sevenn.pt`` and ``opt_params_sevenn.pt`` load by name), and every
parameter is a view of ONE contiguous fp32 buffer whose gradients also live in
one buffer: the data-parallel gradient all-reduce is a single collective with
no packing copy (``flat_grad``).
"""
import json
import math
import os

import numpy as np
import torch

from . import _keys as KEY
from . import conv_ops

ASSETS = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'assets')


def parse_irreps(s):
    """'4x0o+4x1e' -> [(4, 0, -1), (4, 1, 1)] (mul, l, parity)"""
    out = []
    for term in s.split('+'):
        mul, ir = term.strip().split('x')
        out.append((int(mul), int(ir[:-1]), 1 if ir[-1] == 'e' else -1))
    return out


def _offsets(irreps):
    return np.cumsum([0] + [t[0] * (2 * t[1] + 1) for t in irreps]).tolist()


def _ir(t):
    """(l, p) of an irreps entry (mul, l[, p]); parity defaults to even"""
    return (t[1], t[2] if len(t) > 2 else 1)


class _Linear:
    """e3nn o3.Linear without bias (sevenn/nn/linear.py:46-49): one block per
    (i_in, i_out) pair of equal l, i_in-major, each (mul_in, mul_out)
    row-major in the flat weight, path weight 1/sqrt(fan-in of i_out).

    Launch-lean form (the fine-tune step is launch-bound at its batch sizes):
    inputs of one l that are adjacent in x (the sorted mid irreps are) form one
    (n, sum mul, 2l+1) block and their weight blocks one stacked matrix, so each
    output irrep is ONE GEMM, W^T x_l, written straight into the mul-major
    layout; x and the weight are split (backward: one cat) rather than sliced
    (backward: zero-fill + copy per slice)."""

    def __init__(self, irreps_in, irreps_out):
        self.irreps_in, self.irreps_out = irreps_in, irreps_out
        self.ins = [(i, j) for i, a in enumerate(irreps_in)
                    for j, b in enumerate(irreps_out) if _ir(a) == _ir(b)]
        fan = {j: sum(irreps_in[i][0] for i, jj in self.ins if jj == j) for _, j in self.ins}
        self.alpha = {j: 1.0 / math.sqrt(f) for j, f in fan.items()}
        self.in_off, self.out_off = _offsets(irreps_in), _offsets(irreps_out)
        self.numel = sum(irreps_in[i][0] * irreps_out[j][0] for i, j in self.ins)
        self.w_sizes = [irreps_in[i][0] * irreps_out[j][0] for i, j in self.ins]
        # per output j: runs of consecutive input irreps feeding it
        self.groups = {}
        for k, (i, j) in enumerate(self.ins):
            runs = self.groups.setdefault(j, [])
            if runs and runs[-1][-1][0] == i - 1:
                runs[-1].append((i, k))
            else:
                runs.append([(i, k)])
        # x split points: every input irrep boundary
        self.x_sizes = [t[0] * (2 * t[1] + 1) for t in irreps_in]

    # Dense form (the fine-tune step's default): the block-sparse e3nn weight
    # scattered ONCE per call into a (dim_in, dim_out) matrix -- W[u, v] * alpha_j
    # on the (u m, v m) diagonals of each (i, j) block, 0 elsewhere -- so the
    # linear is ONE GEMM forward and one per derivative product, instead of a
    # GEMM per output irrep plus the splits, cats and scalings around them and
    # their backward / double-backward copies.  At the fine-tune batch sizes
    # (hundreds of atoms) the step is launch-bound, so the FLOPs of the zeros
    # (~7x on 128x0e+64x1e+32x2e) are free.  Only the nonzeros move: a gather of
    # the flat weight (each element repeated 2l+1 times) and a scatter to unique
    # positions -- no index with millions of duplicates (a gather from a zero pad
    # slot that way faulted inside a captured graph's backward on the GPU).
    dense = os.environ.get('E3GNN_TRAIN_DENSE_LINEAR', '1') != '0'

    def _dense_maps(self, device, dtype):
        key = (str(device), dtype)
        if getattr(self, '_dkey', None) != key:
            dout = self.out_off[-1]
            pos, src, scl = [], [], []
            woff = 0
            for i, j in self.ins:
                mi = self.irreps_in[i][0]
                mo, d = self.irreps_out[j][0], 2 * self.irreps_in[i][1] + 1
                u, v, m = np.meshgrid(np.arange(mi), np.arange(mo), np.arange(d), indexing='ij')
                pos.append(((self.in_off[i] + u * d + m) * dout + self.out_off[j] + v * d + m).ravel())
                src.append((woff + u * mo + v).ravel())
                scl.append(np.full(u.size, self.alpha[j]))
                woff += mi * mo
            self._dpos = torch.as_tensor(np.concatenate(pos), device=device)
            self._dsrc = torch.as_tensor(np.concatenate(src), device=device)
            self._dscl = torch.as_tensor(np.concatenate(scl), device=device, dtype=dtype)
            self._dkey = key
        return self._dpos, self._dsrc, self._dscl

    def _dense_weight(self, w_flat):
        pos, src, scl = self._dense_maps(w_flat.device, w_flat.dtype)
        wd = w_flat.new_zeros(self.in_off[-1] * self.out_off[-1])
        wd = wd.index_put((pos,), w_flat[src] * scl)
        return wd.view(self.in_off[-1], self.out_off[-1])

    def __call__(self, x, w_flat):
        n = x.shape[0]
        # (dense only where the expanded matrix stays small: <= 4M entries, and
        # while the zeros' extra FLOPs are cheap against the launches saved)
        if self.dense and len(self.x_sizes) > 1 and \
                self.in_off[-1] * self.out_off[-1] <= (1 << 22) and n <= 65536:
            return x @ self._dense_weight(w_flat)
        xs = x.split(self.x_sizes, dim=1) if len(self.x_sizes) > 1 else (x,)
        ws = w_flat.split(self.w_sizes) if len(self.w_sizes) > 1 else (w_flat,)
        parts = []
        for j, to in enumerate(self.irreps_out):
            mo, d = to[0], 2 * to[1] + 1
            acc = None
            for run in self.groups.get(j, []):
                mul = sum(self.irreps_in[i][0] for i, _ in run)
                xr = xs[run[0][0]] if len(run) == 1 else torch.cat([xs[i] for i, _ in run], 1)
                wr = ws[run[0][1]].view(-1, mo) if len(run) == 1 else \
                    torch.cat([ws[k].view(-1, mo) for _, k in run], 0)
                if d == 1:
                    y = torch.mm(xr, wr)
                else:
                    y = torch.matmul(wr.t(), xr.view(n, mul, d)).reshape(n, mo * d)
                acc = y if acc is None else acc + y
            if acc is None:
                acc = x.new_zeros(n, mo * d)
            parts.append(acc)
        out = torch.cat(parts, dim=1) if len(parts) > 1 else parts[0]
        return out * self.alpha[0] if self._uniform_alpha() else self._scale(out)

    def _uniform_alpha(self):
        if not hasattr(self, '_ua'):
            vals = {self.alpha.get(j) for j in range(len(self.irreps_out))}
            self._ua = len(vals) == 1 and None not in vals
        return self._ua

    def _scale(self, out):
        if not hasattr(self, '_alpha_cols'):
            cols = []
            for j, to in enumerate(self.irreps_out):
                cols += [self.alpha.get(j, 0.0)] * (to[0] * (2 * to[1] + 1))
            self._alpha64 = torch.tensor(cols, dtype=torch.float64)
            self._alpha_cols = self._alpha64
        if self._alpha_cols.device != out.device or self._alpha_cols.dtype != out.dtype:
            self._alpha_cols = self._alpha64.to(out.device, out.dtype)
        return out * self._alpha_cols


def _gate_irreps(irreps_out):
    """e3nn Gate.irreps_in for EquivariantGate (equivariant_gate.py:30-51):
    scalars = the l = 0 output irreps, gated = the rest (both in order), one
    gate scalar per gated channel of parity +1 when '0e' is among the scalars,
    else -1 (:41); e3nn's Gate stable-sorts [scalars | gates | gated] by
    (l, p) (odd first) and merges equal neighbours.  Returns (irreps_in,
    scalars, gated, layout) with layout = (gate parity, the offset of every
    piece -- each scalar irrep, the gate block, each gated irrep -- in the
    sorted row, and whether that is the unsorted order)."""
    scal = [t for t in irreps_out if t[1] == 0]
    gated = [t for t in irreps_out if t[1] > 0]
    ng = sum(t[0] for t in gated)
    gate_p = 1 if any(_ir(t) == (0, 1) for t in scal) else -1
    pieces = scal + ([(ng, 0, gate_p)] if ng else []) + gated
    order = sorted(range(len(pieces)), key=lambda i: _ir(pieces[i]))   # stable
    offs, off = [0] * len(pieces), 0
    for i in order:
        offs[i] = off
        off += pieces[i][0] * (2 * pieces[i][1] + 1)
    simp = []
    for i in order:
        m, (l, p) = pieces[i][0], _ir(pieces[i])
        if simp and _ir(simp[-1]) == (l, p):
            simp[-1] = (simp[-1][0] + m, l, p)
        else:
            simp.append((m, l, p))
    return simp, scal, gated, (gate_p, offs, order == list(range(len(pieces))))


def conv_instructions(irreps_x, lmax_filter, filter_parity, irreps_out):
    """IrrepsConvolution instructions (convolution.py:72-95): every (x irrep,
    filter irrep l2 of parity filter_parity^l2, output) whose output irrep is
    in the block's output irreps, as (i_x, l2, l3, p3, mul) in weight order;
    the mid irreps are the outputs stable-sorted by (l, p) (odd first), perm[k]
    the slot of instruction k."""
    allowed = {_ir(t) for t in irreps_out}
    ins = []
    for i, t in enumerate(irreps_x):
        mul, (l1, p1) = t[0], _ir(t)
        for l2 in range(lmax_filter + 1):
            p3 = p1 * filter_parity ** l2
            for l3 in range(abs(l1 - l2), l1 + l2 + 1):
                if (l3, p3) in allowed:
                    ins.append((i, l2, l3, p3, mul))
    order = sorted(range(len(ins)), key=lambda k: (ins[k][2], ins[k][3], k))
    perm = [0] * len(ins)
    for slot, k in enumerate(order):
        perm[k] = slot
    mid = [(ins[k][4], ins[k][2], ins[k][3]) for k in order]
    return ins, mid, perm


def path_table(irreps_x, lmax_filter, filter_parity, irreps_out):
    """Runtime path table of e3gnn_gtp_create: per instruction (l1, l2, l3,
    mul, x offset, Y offset, w offset, agg offset), plus (dx, dy, dw, dm)."""
    ins, mid, perm = conv_instructions(irreps_x, lmax_filter, filter_parity, irreps_out)
    xo, mo = _offsets(irreps_x), _offsets(mid)
    rows, woff = [], 0
    for k, (i, l2, l3, _, mul) in enumerate(ins):
        rows.append((irreps_x[i][1], l2, l3, mul, xo[i], l2 * l2, woff, mo[perm[k]]))
        woff += mul
    return (np.asarray(rows, dtype=np.int32).reshape(-1, 8), xo[-1], (lmax_filter + 1) ** 2,
            woff, mo[-1]), mid


def spherical_harmonics(vec, lmax=2, normalize=True):
    """e3nn SphericalHarmonics(0e+1p+2e, 'component') (edge_embedding.py:177-198);
    ``normalize`` False (sevenn < 0.9 checkpoints, util.py:143-144) evaluates
    the same homogeneous polynomials on the raw edge vector."""
    if normalize:
        u = vec / torch.linalg.norm(vec, dim=-1, keepdim=True)
    else:
        u = vec
    # one constant map from the monomials [1, u, u (x) u] (as a GEMM: the
    # fine-tune step is launch-bound and this keeps the SH and its first and
    # second derivatives to a handful of launches instead of ~25 element-wise
    # nodes per derivative order)
    feats = [torch.ones_like(u[:, :1]), u]
    if lmax >= 2:
        feats.append((u.unsqueeze(-1) * u.unsqueeze(-2)).reshape(-1, 9))
    return torch.cat(feats, dim=-1) @ _sh_map(lmax, u.device, u.dtype)


_SH_MAPS = {}


def _sh_map(lmax, device, dtype):
    """(1 + 3 + 9, (lmax+1)^2) coefficients of the component-normalised real
    SH (edge_embedding.py:177-198) on the monomials 1, x, y, z, u_a u_b."""
    key = (lmax, str(device), dtype)
    if key not in _SH_MAPS:
        s3, s5, s15 = math.sqrt(3.0), math.sqrt(5.0), math.sqrt(15.0)
        nf = 4 if lmax < 2 else 13
        m = np.zeros((nf, (lmax + 1) ** 2))
        m[0, 0] = 1.0
        if lmax >= 1:
            m[1, 1] = m[2, 2] = m[3, 3] = s3
        if lmax >= 2:
            q = lambda a, b: 4 + 3 * a + b   # row of u_a u_b (x, y, z = 0, 1, 2)
            m[q(0, 2), 4] = s15
            m[q(0, 1), 5] = s15
            m[q(1, 1), 6] = s5
            m[q(0, 0), 6] = m[q(2, 2), 6] = -0.5 * s5
            m[q(1, 2), 7] = s15
            m[q(2, 2), 8] = 0.5 * s15
            m[q(0, 0), 8] = -0.5 * s15
        _SH_MAPS[key] = torch.as_tensor(m[:, :(lmax + 1) ** 2], device=device, dtype=dtype)
    return _SH_MAPS[key]


def sevennet0_kinds(manifest, conv_only=False):
    """THE test for SevenNet-0's architecture, shared by every router
    (model.load_model and model_build's family label; e3gnn_load checks the
    same knobs): even-parity lmax-2 filters (SH of the unit vector, or of the
    raw vector for pre-0.9 checkpoints: one flag of the edge kernels), the
    XPLOR cutoff, a linear self-connection and exactly
    128x0e -> 4 x (128x0e+64x1e+32x2e) -> 128x0e.  Returns the kernel kind of
    every block (0 first, 1 middle, 2 last; csrc/tp.h) or None.
    ``conv_only``: only what the convolution kernels depend on (filter parity,
    lmax_edge, irreps) -- the trainable model computes the edge basis, SH and
    self-connection itself and needs no more for its kernel choice."""
    man = manifest
    if man.get('is_parity', False) or int(man.get('lmax_edge', man.get('lmax', 2))) != 2:
        return None
    cf = man.get('cutoff_function', {}) or {}
    if not conv_only and (man.get('self_connection_type', 'linear') != 'linear' or
                          cf.get('name', 'XPLOR') != 'XPLOR' or bool(man.get('use_bias_in_linear')) or
                          (man.get('readout') or {}).get('type', 'linear') != 'linear'):
        return None
    irreps = [parse_irreps(s) for s in man['irreps_manual']]
    L = int(man['num_convolution_layer'])
    if len(irreps) != L + 1 or L < 2:
        return None
    kinds = [0 if t == 0 else (2 if t == L - 1 else 1) for t in range(L)]
    want = {0: ([(128, 0, 1)], [(128, 0, 1), (64, 1, 1), (32, 2, 1)]),
            1: ([(128, 0, 1), (64, 1, 1), (32, 2, 1)],) * 2,
            2: ([(128, 0, 1), (64, 1, 1), (32, 2, 1)], [(128, 0, 1)])}
    for t, k in enumerate(kinds):
        if (irreps[t], irreps[t + 1]) != want[k]:
            return None
    return kinds


class SevenNetTrainable(torch.nn.Module):
    """Training-mode SevenNet-0 (batched graphs) with reference parameter names.

    ``train_shift_scale`` / ``train_denominator`` / ``train_radial_coeffs``
    set ``requires_grad`` as the reference's config keys do
    (scale.py:58-61, convolution.py:60, edge_embedding.py:107-110).
    ``conv_backend`` defaults to the HIP kernels; tests may pass another
    object with the same three methods to check host logic on the CPU."""

    def __init__(self, model_dir=os.path.join(ASSETS, 'sevennet0'), device='cuda',
                 train_shift_scale=False, train_denominator=False, train_radial_coeffs=True,
                 conv_backend=None, dtype=torch.float32, manifest=None, weights=None):
        """Parameters from a deployment directory (manifest.json +
        weights.bin), or from ``manifest`` (dict) + ``weights`` (flat fp32
        array in manifest tensor order) -- what model_build produces."""
        super().__init__()
        self.dtype = dtype
        if manifest is None:
            with open(os.path.join(model_dir, 'manifest.json')) as f:
                manifest = json.load(f)
        man = manifest
        self.manifest = man
        self.chemical_symbols = list(man['chemical_symbols'])
        self.nsp = int(man['num_species'])
        self.cutoff = float(man['cutoff'])
        self.cut = dict(man['cutoff_function'])
        self.r_on = float(self.cut.get('cutoff_on', self.cutoff))
        self.silu_norm = float(man['silu_norm'])
        self.tanh_norm = float(man.get('act_norm', {}).get('tanh', 1.0))
        self.irreps = [parse_irreps(s) for s in man['irreps_manual']]
        self.nlayer = int(man['num_convolution_layer'])
        # the nequip family's other knobs (sevenn 0.8.6 HfO2 example:
        # odd parity, raw-vector SH, FCTP self-connection, tanh odd scalars)
        self.lmax_edge = int(man.get('lmax_edge', man.get('lmax', 2)))
        self.filter_parity = -1 if man.get('is_parity', False) else 1
        self.sh_normalize = bool(man.get('sh_normalize', True))
        self.sc_type = man.get('self_connection_type', 'linear')
        self.readout_hidden = int(man.get('readout_hidden', self.irreps[-1][0][0] // 2))
        # use_bias_in_linear (e3nn Linear biases on 0e outputs) and the
        # readout_as_fcn readout (FCN_e3nn): model_build.py:194-240, :396-408
        self.use_bias = bool(man.get('use_bias_in_linear', False))
        self.readout_cfg = dict(man.get('readout') or {'type': 'linear'})
        self.conv_backend = conv_backend
        flat_host = np.fromfile(os.path.join(model_dir, 'weights.bin'), dtype='<f4') \
            if weights is None else np.ascontiguousarray(weights, dtype='<f4').reshape(-1)
        total = sum(t['numel'] for t in man['tensors'])
        self.flat = torch.empty(total, dtype=dtype, device=device)
        self.flat_grad = torch.zeros(total, dtype=dtype, device=device)
        self.slices = {}
        off = 0
        for t in man['tensors']:
            name, n = t['name'], int(t['numel'])
            self.flat[off:off + n].copy_(
                torch.from_numpy(flat_host[t['offset']:t['offset'] + n].copy()))
            p = torch.nn.Parameter(self.flat[off:off + n].view(t['shape']))
            self._register_nested(name, p)
            self.slices[name] = (off, n, tuple(t['shape']))
            off += n
        self._build_layers()
        for name, p in self.named_parameters():
            if name.startswith('rescale_atomic_energy.'):
                p.requires_grad_(train_shift_scale)
            elif name.endswith('.denominator'):
                p.requires_grad_(train_denominator)
            elif name == 'edge_embedding.basis_function.coeffs':
                p.requires_grad_(train_radial_coeffs)
        self.attach_flat_grad()
        self.is_batch_data = True
        self._gate_dims = {}

    # ------------------------------------------------------------ parameters
    def _register_nested(self, name, p):
        parts = name.split('.')
        mod = self
        for part in parts[:-1]:
            if part not in mod._modules:
                mod.add_module(part, torch.nn.Module())
            mod = mod._modules[part]
        mod.register_parameter(parts[-1], p)

    def param(self, name):
        mod = self
        for part in name.split('.'):
            mod = getattr(mod, part)
        return mod

    def attach_flat_grad(self):
        """Point every parameter's .grad at its slice of ``flat_grad`` so that
        backward accumulates in place into one contiguous buffer."""
        for name, p in self.named_parameters():
            off, n, shape = self.slices[name]
            p.grad = self.flat_grad[off:off + n].view(shape)

    def zero_grad(self, set_to_none=False):
        self.flat_grad.zero_()
        self.attach_flat_grad()

    def grads_in_flat_buffer(self):
        base = self.flat_grad.data_ptr()
        end = base + self.flat_grad.numel() * self.flat_grad.element_size()
        return all(p.grad is not None and base <= p.grad.data_ptr() < end
                   for p in self.parameters())

    def set_is_batch_data(self, flag: bool):
        self.is_batch_data = bool(flag)

    # ------------------------------------------------------------ structure
    def _sevennet0_kinds(self):
        """The SevenNet-0 kernel kinds (csrc/tp.h) of the blocks, or None when
        the architecture is another member of the family."""
        return sevennet0_kinds(self.manifest, conv_only=True)

    def _build_layers(self):
        irr = self.irreps
        # the convolution's output irreps per block (model_build: the
        # reference's irreps_out_tp); deployments without the key (SevenNet-0,
        # the 0.8.6 HfO2 example) built it on irreps_manual
        conv_out = [parse_irreps(s) for s in self.manifest['conv_irreps_out']] \
            if 'conv_irreps_out' in self.manifest else irr[1:]
        self.blocks = []
        tables = []
        for t in range(self.nlayer):
            x_ir, out_ir = irr[t], irr[t + 1]
            gate_irreps = _gate_irreps(out_ir)
            gin = gate_irreps[0]
            table, mid = path_table(x_ir, self.lmax_edge, self.filter_parity, conv_out[t])
            tables.append(table)
            self.blocks.append({
                'kind': t, 'gate': gate_irreps, 'sc_irreps': (x_ir, gin),
                'sc': _Linear(x_ir, gin), 'si1': _Linear(x_ir, x_ir), 'si2': _Linear(mid, gin)})
        kinds = self._sevennet0_kinds()
        be = self.conv_backend
        if be is None:
            # SevenNet-0: the specialised kernels (compile-time path tables);
            # any other member of the family: the runtime path tables (gtp.hip)
            be = conv_ops.HipConvBackend() if kinds is not None \
                else conv_ops.GenericHipConvBackend(tables)
        elif getattr(be, 'generic', False):
            be.configure(tables)
        self.conv_backend = be
        if not getattr(be, 'generic', False):
            if kinds is None:
                raise ValueError('this architecture has no SevenNet-0 kernel path table; use the '
                                 'generic (runtime path table) backend')
            for blk, k in zip(self.blocks, kinds):
                blk['kind'] = k
        for blk, table in zip(self.blocks, tables):
            _, dx, _, dw, dm = table
            if tuple(be.dims[blk['kind']]) != (dx, dw, dm):
                raise ValueError(f'block {blk["kind"]}: backend dims {be.dims[blk["kind"]]} != '
                                 f'{(dx, dw, dm)}')
        hid = self.readout_hidden
        if self.readout_cfg.get('type', 'linear') == 'fcn' and any(l != 0 for _, l, _ in irr[-1]):
            raise ValueError('readout_as_fcn needs a scalar-only last block')
        self.readout1 = _Linear(irr[-1], [(hid, 0, 1)])
        self.readout2 = _Linear([(hid, 0, 1)], [(1, 0, 1)])

    def bias(self, y, irreps_out, name):
        """+ the IrrepsLinear's bias (its 0e output channels) when the model
        has biases (use_bias_in_linear)"""
        if f'{name}.linear.bias' not in self.slices:
            return y
        b = self.param(f'{name}.linear.bias')
        parts, off, k = [], 0, 0
        for m, l, p in irreps_out:
            d = m * (2 * l + 1)
            blk = y[:, off:off + d]
            if (l, p) == (0, 1):
                blk = blk + b[k:k + m]
                k += m
            parts.append(blk)
            off += d
        return torch.cat(parts, dim=1) if len(parts) > 1 else parts[0]

    def readout_fcn(self, x):
        """FCN_e3nn (nn/linear.py:94-129): e3nn FullyConnectedNet on the
        last block's scalars, c act(h W / sqrt(fan_in)) between layers"""
        ro = self.readout_cfg
        f = {'relu': torch.relu, 'silu': torch.nn.functional.silu, 'tanh': torch.tanh,
             'sigmoid': torch.sigmoid, 'abs': torch.abs,
             'elu': torch.nn.functional.elu}[ro['act']]
        c = float(ro['act_norm'])
        nh = len(ro['hidden'])
        h = x
        for k in range(nh + 1):
            w = self.param(f'readout_FCN.fcn.layer{k}.weight')
            h = h @ (w / math.sqrt(w.shape[0]))
            if k < nh:
                h = f(h) * c
        return h[:, 0]

    def act(self, x):
        # HIP kernels on the GPU (one launch per derivative order); the CPU
        # runs of this model are the tests' float64 double
        if x.is_cuda and x.dtype == torch.float32:
            return conv_ops.scaled_silu(x, self.silu_norm, self._act_lib())
        return torch.nn.functional.silu(x) * self.silu_norm

    def _act_lib(self):
        if getattr(self, '_lib_handle', None) is None:
            from . import _lib
            self._lib_handle = _lib.load()
        return self._lib_handle

    def gate(self, x, gate_irreps):
        # e3nn nn.Gate (equivariant_gate.py:59-61); split, not sliced (one cat
        # in the backward instead of a zero-fill + copy per slice).  Odd
        # scalars and odd gates take tanh (act 'o'), the rest scaled SiLU.
        _, scal, gated, (gate_p, offs, natural) = gate_irreps
        n = x.shape[0]
        ns = sum(t[0] for t in scal)
        ng = sum(t[0] for t in gated)
        odd = any(_ir(t)[1] == -1 for t in scal) or gate_p == -1
        if natural and ng > 0 and not odd and x.is_cuda and x.dtype == torch.float32 and \
                len(gated) <= 2:
            key = id(gate_irreps)
            if key not in self._gate_dims:
                self._gate_dims[key] = conv_ops.gate_dims([t[:2] for t in scal],
                                                          [t[:2] for t in gated])
            return conv_ops.gate(x, self._gate_dims[key], self.silu_norm, self._act_lib())
        sizes = [t[0] for t in scal] + ([ng] if ng else []) + \
            [t[0] * (2 * t[1] + 1) for t in gated]
        if natural:
            pieces = x.split(sizes, dim=1) if len(sizes) > 1 else (x[:, :sizes[0]],)
        else:   # the row is e3nn's (l, p)-sorted layout: each piece at its offset
            pieces = [x[:, o:o + w] for o, w in zip(offs, sizes)]
        act_o = lambda v: torch.tanh(v) * self.tanh_norm   # noqa: E731
        outs = []
        for k, t in enumerate(scal):
            outs.append(self.act(pieces[k]) if _ir(t)[1] == 1 else act_o(pieces[k]))
        if ng:
            g = pieces[len(scal)]
            gs = (self.act(g) if gate_p == 1 else act_o(g)).split([t[0] for t in gated], dim=1)
            for k, t in enumerate(gated):
                blk = pieces[len(scal) + 1 + k].reshape(n, t[0], 2 * t[1] + 1)
                outs.append((gs[k].unsqueeze(-1) * blk).reshape(n, -1))
        return torch.cat(outs, dim=1) if len(outs) > 1 else outs[0]

    def _edge_basis(self, r):
        # BesselBasis (edge_embedding.py:114-116) * XPLORCutoff (:163-173) or
        # PolynomialCutoff (:131-145)
        rc = self.cutoff
        coeffs = self.param('edge_embedding.basis_function.coeffs')
        ur = r.unsqueeze(-1)
        bessel = (2.0 / rc) * torch.sin(coeffs * ur) / ur
        if self.cut.get('name', 'XPLOR') == 'poly_cut':
            p = float(self.cut['p'])
            x = r / rc
            env = 1.0 - (p + 1.0) * (p + 2.0) / 2.0 * x ** p + p * (p + 2.0) * x ** (p + 1) \
                - p * (p + 1.0) / 2.0 * x ** (p + 2)
            return bessel * env.unsqueeze(-1)
        # XPLOR switch as ONE polynomial in s = max(r^2, r_on^2): it equals 1 at
        # s = r_on^2, so the clamp is the r < r_on branch (value and derivatives)
        # without a where/ones_like pair per derivative order
        ron, rc2 = self.r_on, rc * rc
        s = torch.clamp(r * r, min=ron * ron)
        env = (rc2 - s) ** 2 * (2.0 * s + (rc2 - 3.0 * ron * ron)) * (1.0 / (rc2 - ron * ron) ** 3)
        return bessel * env.unsqueeze(-1)

    def self_connection(self, t, blk, x, types):
        """SelfConnectionLinearIntro (self_connection.py:42-62) or, for the
        'nequip' type, SelfConnectionIntro = FullyConnectedTensorProduct(x,
        one-hot) (:11-38): per (i_x, i_out) of equal irrep a (mul_x, nsp,
        mul_out) weight block, path weight 1/sqrt(sum of mul_x nsp into i_out)
        -- with a one-hot operand, row n uses the block of its species."""
        if self.sc_type != 'nequip':
            return blk['sc'](x, self.param(f'{t}_self_connection_intro.linear.weight'))
        x_ir, gin = blk['sc_irreps']
        w = self.param(f'{t}_self_connection_intro.fc_tensor_product.weight')
        n, nsp = x.shape[0], self.nsp
        xo = _offsets(x_ir)
        ins = [(i, j) for i, a in enumerate(x_ir) for j, b in enumerate(gin) if _ir(a) == _ir(b)]
        fan = {}
        for i, j in ins:
            fan[j] = fan.get(j, 0) + x_ir[i][0] * nsp
        outs = [None] * len(gin)
        woff = 0
        for i, j in ins:
            mi, l, mo = x_ir[i][0], x_ir[i][1], gin[j][0]
            wb = w[woff:woff + mi * nsp * mo].view(mi, nsp, mo)
            woff += mi * nsp * mo
            xi = x[:, xo[i]:xo[i + 1]].reshape(n, mi, 2 * l + 1)
            # (n, mo, 2l+1): the species' (mi, mo) block per row
            y = torch.einsum('nui,unw->nwi', xi, wb[:, types, :]) / math.sqrt(fan[j])
            outs[j] = y if outs[j] is None else outs[j] + y
        parts = [o.reshape(n, -1) if o is not None else x.new_zeros(n, t_[0] * (2 * t_[1] + 1))
                 for o, t_ in zip(outs, gin)]
        return torch.cat(parts, dim=1)

    # ------------------------------------------------------------ forward
    def forward(self, data, graph=None):
        """AtomGraphSequential.forward on a batched AtomGraphData dict:
        ``x`` (type index), ``edge_index``, ``edge_vec``, ``batch``,
        ``num_atoms``, ``cell_volume`` -> adds ``atomic_energy``,
        ``inferred_total_energy`` [B], ``inferred_force`` [N,3],
        ``inferred_stress`` [B,6] (eV/A^3, order xx,yy,zz,xy,yz,zx)."""
        dev = self.flat.device
        types = data[KEY.NODE_FEATURE].to(dev).long()
        n = int(types.shape[0])
        ei = data[KEY.EDGE_IDX].to(dev).long()
        vec = data[KEY.EDGE_VEC].to(dev, self.dtype)
        if not vec.requires_grad:
            vec = vec.detach().requires_grad_(True)
        batch = data[KEY.BATCH].to(dev).long() if KEY.BATCH in data else \
            torch.zeros(n, dtype=torch.long, device=dev)
        center, nbr = ei[0], ei[1]
        vec_k = vec
        if graph is None:
            if center.numel() > 1 and bool((center[1:] < center[:-1]).any()):
                perm = torch.argsort(center, stable=True)
                center, nbr, vec_k = center[perm], nbr[perm], vec[perm]
            graph = conv_ops.ConvGraph(n, center, nbr, self.conv_backend)

        r = torch.linalg.norm(vec_k, dim=-1)
        emb = self._edge_basis(r)
        Y = spherical_harmonics(vec_k, self.lmax_edge, self.sh_normalize)
        P = self.param
        x = P('onehot_to_feature_x.linear.weight').view(self.nsp, -1)[types] / math.sqrt(self.nsp)
        x = self.bias(x, self.irreps[0], 'onehot_to_feature_x')
        for t, blk in enumerate(self.blocks):
            sc = self.self_connection(t, blk, x, types)
            h = self.bias(blk['si1'](x, P(f'{t}_self_interaction_1.linear.weight')), self.irreps[t],
                          f'{t}_self_interaction_1')
            pre = f'{t}_convolution'
            w0 = P(f'{pre}.weight_nn.layer0.weight')
            hid = self.act(emb @ (w0 / math.sqrt(w0.shape[0])))
            w1 = P(f'{pre}.weight_nn.layer1.weight')
            hid = self.act(hid @ (w1 / math.sqrt(w1.shape[0])))
            w2 = P(f'{pre}.weight_nn.layer2.weight')
            w = hid @ (w2 / math.sqrt(w2.shape[0]))
            agg = conv_ops.conv(h, Y, w, blk['kind'], graph) / P(f'{pre}.denominator')
            y = self.bias(blk['si2'](agg, P(f'{t}_self_interaction_2.linear.weight')),
                          blk['sc_irreps'][1], f'{t}_self_interaction_2') + sc
            x = self.gate(y, blk['gate'])
        if self.readout_cfg.get('type', 'linear') == 'fcn':
            e_s = self.readout_fcn(x)
        else:
            hid = self.readout_hidden
            hidden = self.bias(self.readout1(x, P('reduce_input_to_hidden.linear.weight')),
                               [(hid, 0, 1)], 'reduce_input_to_hidden')
            e_s = self.bias(self.readout2(hidden, P('reduce_hidden_to_energy.linear.weight')),
                            [(1, 0, 1)], 'reduce_hidden_to_energy')[:, 0]
        atomic = e_s * P('rescale_atomic_energy.scale')[types] + \
            P('rescale_atomic_energy.shift')[types]
        nb = int(data[KEY.NUM_ATOMS].numel()) if KEY.NUM_ATOMS in data else 1
        energy = torch.zeros(nb, device=dev, dtype=atomic.dtype).index_add(0, batch, atomic)

        out = dict(data)
        out[KEY.EDGE_VEC] = vec
        out[KEY.ATOMIC_ENERGY] = atomic.unsqueeze(-1)
        out[KEY.PRED_TOTAL_ENERGY] = energy
        # ForceStressOutputFromEdge (force_output.py:158-215)
        fij, = torch.autograd.grad([energy.sum()], [vec], create_graph=self.training,
                                   allow_unused=False)
        # (few launches per derivative order: the fine-tune step is launch-bound)
        src, dst = ei[0], ei[1]
        force = torch.zeros(n, 3, device=dev, dtype=fij.dtype).index_add(
            0, torch.cat([src, dst]), torch.cat([fij, -fij]))
        out[KEY.PRED_FORCE] = force
        # virial terms xx yy zz xy yz zx = r_a f_b for (a, b) = (x,x) .. (z,x),
        # summed per graph straight from the edges (graph of the edge's dst atom)
        voigt = vec.repeat(1, 2) * torch.cat([fij, fij.roll(-1, dims=1)], dim=1)
        s_graph = torch.zeros(nb, 6, device=dev, dtype=fij.dtype).index_add(0, batch[dst], voigt)
        if KEY.CELL_VOLUME in data:
            vol = data[KEY.CELL_VOLUME].to(dev, self.dtype).view(-1)
            out[KEY.PRED_STRESS] = torch.neg(s_graph) / vol.unsqueeze(-1)
        return out
