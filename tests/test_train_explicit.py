"""The hand-scheduled fine-tune derivatives (train_explicit.py) against
autograd of the trainable model, float64 on the CPU (conv op: the oracle's
tensor product, _conv_cpu.py).

The explicit step computes forces / stress by a first reverse and the
parameter gradient of the loss (energy + force + stress terms, the
second-order derivative of force_output.py:158-215 under trainer.py:155-222)
by a tangent forward along dL/df and one reverse sweep; autograd of
nn.SevenNetTrainable (itself pinned against the fp64 oracle in
test_train.py) differentiates the same loss with create_graph.  Every
trainable parameter (incl. shift/scale, denominators, Bessel coefficients)
must agree to float64 round-off."""
import numpy as np
import pytest
import torch

from _conv_cpu import CpuConvBackend
from _systems import load_manifest_symbols
from sevennet_finetuning_amd import _keys as KEY
from sevennet_finetuning_amd import train
from sevennet_finetuning_amd.nn import SevenNetTrainable
from sevennet_finetuning_amd.structures import diamond_primitive, mixed_symbols

SYMS = load_manifest_symbols()


@pytest.fixture(scope='module')
def model():
    return SevenNetTrainable(device='cpu', conv_backend=CpuConvBackend(), dtype=torch.float64,
                             train_shift_scale=True, train_denominator=True)


def _batch(seeds=(0, 1), cells=(2, 2, 1)):
    gs = []
    for s in seeds:
        pos, cell = diamond_primitive(cells, sigma=0.08, seed=s)
        types = np.array([SYMS.index(x) for x in mixed_symbols(len(pos), seed=s + 1)])
        rng = np.random.default_rng(50 + s)
        gs.append(train.labeled_graph(pos, cell, types, 5.0, energy=-4.0 * len(pos),
                                      force=rng.normal(size=(len(pos), 3)),
                                      stress=rng.normal(size=6) * 1e-2))
    return train.collate(gs, dtype=torch.float64)


def _losses(kind):
    cfg = {'loss': kind, 'force_loss_weight': 0.7, 'stress_loss_weight': 0.05,
           'is_train_stress': True, 'continue': {'fisher_information': False, 'opt_params': False}}
    if kind == 'huber':
        cfg['loss_param'] = {'delta': 0.05}
    return train.get_loss_functions_from_config(cfg)


def _autograd(model, batch, fns):
    model.train(True)
    model.zero_grad()
    out = model(batch)
    loss = sum(f.get_loss(out, model) * w for f, w in fns)
    loss.backward()
    model.train(False)
    return out, float(loss), model.flat_grad.clone()


def _explicit(model, batch, fns):
    from sevennet_finetuning_amd.train_explicit import ExplicitStep
    step = ExplicitStep(model)
    model.zero_grad()
    out = step.forward(batch)
    loss = sum(f.get_loss(out, model) * w for f, w in fns)
    leaves = [out[KEY.PRED_TOTAL_ENERGY], out[KEY.PRED_FORCE], out[KEY.PRED_STRESS]]
    cE, cF, cS = torch.autograd.grad(loss, leaves, allow_unused=True)
    step.backward(cE, cF, cS)
    return out, float(loss), model.flat_grad.clone()


@pytest.mark.parametrize('kind', ['mse', 'huber'])
def test_explicit_gradient_equals_autograd(model, kind):
    batch = _batch()
    fns = _losses(kind)
    oa, la, ga = _autograd(model, batch, fns)
    oe, le, ge = _explicit(model, batch, fns)
    for k in (KEY.PRED_TOTAL_ENERGY, KEY.PRED_FORCE, KEY.PRED_STRESS):
        assert torch.allclose(oe[k].detach(), oa[k].detach(), rtol=1e-11, atol=1e-12), k
    assert abs(le - la) <= 1e-11 * abs(la)
    scale = ga.abs().max()
    bad = {}
    for name, (off, n, _) in model.slices.items():
        d = (ge[off:off + n] - ga[off:off + n]).abs().max()
        if d > 1e-9 * scale:
            bad[name] = (float(d), float(ga[off:off + n].abs().max()))
    assert not bad, bad
    assert float(ga.abs().sum()) > 0


def test_explicit_gradient_unsorted_edges_and_frozen_parameters():
    """Edges not centre-sorted (the step sorts them as the model does) and the
    default trainability (shift/scale and denominators frozen)."""
    m = SevenNetTrainable(device='cpu', conv_backend=CpuConvBackend(), dtype=torch.float64)
    batch = _batch(seeds=(3,))
    perm = torch.randperm(batch[KEY.EDGE_IDX].shape[1], generator=torch.Generator().manual_seed(0))
    for k in (KEY.EDGE_IDX,):
        batch[k] = batch[k][:, perm]
    for k in (KEY.EDGE_VEC, KEY.CELL_SHIFT):
        if k in batch:
            batch[k] = batch[k][perm]
    fns = _losses('mse')
    _, _, ga = _autograd(m, batch, fns)
    _, _, ge = _explicit(m, batch, fns)
    assert torch.allclose(ge, ga, rtol=1e-9, atol=1e-9 * float(ga.abs().max()))
    off, n, _ = m.slices['rescale_atomic_energy.scale']
    assert float(ge[off:off + n].abs().max()) == 0.0


@pytest.mark.parametrize('frozen', ['2_self_interaction_1.linear.weight',
                                    '3_self_interaction_2.linear.weight',
                                    'reduce_hidden_to_energy.linear.weight'])
def test_explicit_gradient_frozen_linear(frozen):
    """A frozen e3nn Linear gets no gradient in the flat buffer (autograd
    leaves its slice at zero), and every other parameter's gradient is
    unchanged: the dense-bank flush skips it (si2 with its denominator fold
    included)."""
    m = SevenNetTrainable(device='cpu', conv_backend=CpuConvBackend(), dtype=torch.float64)
    batch = _batch(seeds=(4,))
    fns = _losses('mse')
    _, _, g_all = _explicit(m, batch, fns)
    m.param(frozen).requires_grad_(False)
    _, _, ga = _autograd(m, batch, fns)
    _, _, ge = _explicit(m, batch, fns)
    off, n, _ = m.slices[frozen]
    assert float(ga[off:off + n].abs().max()) == 0.0
    assert float(ge[off:off + n].abs().max()) == 0.0
    assert float(g_all[off:off + n].abs().max()) > 0
    assert torch.allclose(ge, ga, rtol=1e-9, atol=1e-9 * float(ga.abs().max()))
    keep = torch.ones_like(ge, dtype=torch.bool)
    keep[off:off + n] = False
    assert torch.allclose(ge[keep], g_all[keep], rtol=1e-12, atol=1e-14)


def test_split_k_weight_gradient():
    """_wgrad's chunked batched GEMM + sum equals A^T B (K = 24,192 rows, the
    fine-tune step's stacked edge count)."""
    from sevennet_finetuning_amd.train_explicit import _wgrad
    g = torch.Generator().manual_seed(0)
    A = torch.randn(24192, 64, generator=g, dtype=torch.float64)
    B = torch.randn(24192, 64, generator=g, dtype=torch.float64)
    G = torch.randn(64, 64, generator=g, dtype=torch.float64)
    ref = G + 0.5 * A.t() @ B
    _wgrad(G, A, B, 0.5)
    assert torch.allclose(G, ref, rtol=1e-12, atol=1e-10)


def test_block_sparsity_tables_cover_every_nonzero(model):
    """The per-tile k ranges the fine-tune GEMMs skip by (e3gnn_gemm_desc::
    krange, ExplicitStep._kr) cover every nonzero of the dense linear matrices
    (built from random weights, so no weight is zero by chance): C = A D and
    C = A D^T read each output tile's nonzero rows only inside its range, the
    gradient tables mark every tile that holds a nonzero."""
    from sevennet_finetuning_amd.train_explicit import ExplicitStep
    step = ExplicitStep(model)
    D = step.bank.build()
    T = 64
    for key in [k for k in D if k[:2] in ('sc', 'si')]:
        nz = (D[key] != 0).numpy()
        for trans in (False, True):
            m = nz.T if trans else nz              # op(D): k rows x output columns
            tab = step._kr((key, trans))[0].cpu().numpy().reshape(-1, 4)
            for b in range(tab.shape[0]):
                rows = np.nonzero(m[:, b * T:(b + 1) * T].any(1))[0]
                if rows.size:
                    assert tab[b, 0] <= rows.min() and rows.max() < tab[b, 1], (key, trans, b)
        tab, stride = step._kr(None, grad=key)
        tab = tab.cpu().numpy().reshape(-1, stride, 4)
        for a in range(tab.shape[0]):
            for b in range(stride):
                if nz[a * T:(a + 1) * T, b * T:(b + 1) * T].any():
                    assert tab[a, b, 1] > 0, (key, a, b)


def test_gemm_layout_torch_fallback_matches_dense():
    """_Gemms' torch form of a general-layout problem (used when an operand
    is beyond the library's 32-bit buffer offsets): the linear weight
    gradient's layout -- K summed over (m, node) segments of the irreps rows
    -- equals the dense product, and a 2 GB+ layout is detected"""
    from sevennet_finetuning_amd import _lib
    from sevennet_finetuning_amd.train_explicit import _Gemms
    g = torch.Generator().manual_seed(0)
    rows, d, mi, mo = 7, 3, 4, 5
    X = torch.randn(rows, 2 + mi * d, generator=g, dtype=torch.float64)
    Y = torch.randn(rows, 1 + mo * d, generator=g, dtype=torch.float64)
    G = torch.randn(mi * 10, generator=g, dtype=torch.float64)
    lay = _lib.GemmLayouts()
    lay.a.ld, lay.a.rep, lay.a.rs, lay.a.kst, lay.a.ks, lay.a.sst = d, 1, 0, X.stride(0), rows, 1
    lay.b.ld, lay.b.rep, lay.b.rs, lay.b.kst, lay.b.ks, lay.b.sst = d, 1, 0, Y.stride(0), rows, 1
    lay.ldc, lay.crep, lay.crs, lay.cns = 10, 1, 0, 2
    gm = _Gemms.__new__(_Gemms)
    G0 = G.clone()
    gm._lay_torch(mi, mo, d * rows, (G, 0), (X, 2), (Y, 1), lay, None, None, 0, 0.5, 1)
    Xs = X[:, 2:].reshape(rows, mi, d)
    Ys = Y[:, 1:].reshape(rows, mo, d)
    ref = 0.5 * torch.einsum('num,nvm->uv', Xs, Ys)
    Gv = G0.view(mi, 10)[:, 0:2 * mo:2] + ref
    assert torch.allclose(G.view(mi, 10)[:, 0:2 * mo:2], Gv)
    assert torch.equal(G.view(mi, 10)[:, 1::2], G0.view(mi, 10)[:, 1::2])
    assert _Gemms._lay_fits(X, 2, lay.a, mi, d * rows)
    lay.a.sst = 1 << 29
    assert not _Gemms._lay_fits(X, 2, lay.a, mi, d * rows)
    big = torch.empty((1 << 30) + 4, device='meta').as_strided((1 << 20, 4), (1 << 10, 1))
    assert not _Gemms._fits(big) and _Gemms._fits(torch.empty(64, 64))
