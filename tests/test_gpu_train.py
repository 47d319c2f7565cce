"""Fine-tune step on the HIP kernels (conv_ops -> libe3gnn_hip.so training
ops) against the float64 CPU double of the same op (_conv_cpu.py, the
oracle's uvu tensor product).  Needs an MI355X: ``pytest -m gpu``.

Tolerances (fp32 kernels vs float64): convolution outputs and their first and
second derivatives 2e-5 relative to the output's max magnitude; model forces
1e-4 eV/A (north_star), energies 2e-6 relative; parameter gradients of the
force loss (double backward, create_graph=True) 1e-4 relative in norm.
"""
import ctypes

import numpy as np
import pytest
import torch

from _conv_cpu import CpuConvBackend
from _systems import load_manifest_symbols
from sevennet_finetuning_amd import _keys as KEY
from sevennet_finetuning_amd import conv_ops, train
from sevennet_finetuning_amd.structures import diamond_primitive, mixed_symbols

pytestmark = pytest.mark.gpu
SYMS = load_manifest_symbols()
DEV = 'cuda:0'


def ft_structure(seed, cells=(3, 3, 3)):
    pos, cell = diamond_primitive(cells, sigma=0.05, seed=seed)
    types = np.array([SYMS.index(s) for s in mixed_symbols(len(pos), seed=seed + 1)])
    return pos, cell, types


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.fixture(scope='module')
def hip_backend():
    assert torch.cuda.is_available(), 'GPU tests need a HIP device'
    return conv_ops.HipConvBackend()


def _problem(kind, dims, n=61, seed=0):
    """Ragged random graph: some nodes without edges, some with many,
    sorted centres, random neighbours (repeats allowed)."""
    rng = np.random.default_rng(seed)
    deg = rng.integers(0, 12, n)
    deg[::7] = 0
    deg[3] = 40
    center = np.repeat(np.arange(n), deg)
    e = len(center)
    nbr = rng.integers(0, n, e)
    dx, dw, dm = dims[kind]
    h = rng.normal(size=(n, dx))
    Y = rng.normal(size=(e, 9))
    w = rng.normal(size=(e, dw))
    g = rng.normal(size=(n, dm))
    probe = [rng.normal(size=(n, dx)), rng.normal(size=(e, 9)), rng.normal(size=(e, dw))]
    return center, nbr, (h, Y, w), g, probe


def _derivs(conv, graph, ops, g, probe, dtype, device):
    t = [torch.tensor(a, dtype=dtype, device=device, requires_grad=True) for a in ops]
    gt = torch.tensor(g, dtype=dtype, device=device)
    pt = [torch.tensor(a, dtype=dtype, device=device) for a in probe]
    agg = conv(*t, graph)
    d1 = torch.autograd.grad((agg * gt).sum(), t, create_graph=True)
    s = sum((di * pi).sum() for di, pi in zip(d1, pt))
    d2 = torch.autograd.grad(s, t)
    return agg, d1, d2


@pytest.mark.parametrize('kind', [0, 1, 2])
def test_conv_op_first_and_second_derivatives(hip_backend, kind):
    center, nbr, ops, g, probe = _problem(kind, hip_backend.dims, seed=kind)
    cpu = CpuConvBackend()
    gc = conv_ops.ConvGraph(len(g), torch.tensor(center), torch.tensor(nbr), cpu)
    gh = conv_ops.ConvGraph(len(g), torch.tensor(center, device=DEV),
                            torch.tensor(nbr, device=DEV), hip_backend)
    fwd = lambda h, Y, w, gr: conv_ops.conv(h, Y, w, kind, gr)  # noqa: E731
    ref = _derivs(fwd, gc, ops, g, probe, torch.float64, 'cpu')
    got = _derivs(fwd, gh, ops, g, probe, torch.float32, DEV)
    assert _rel(got[0], ref[0]) < 2e-5
    for a, b in zip(got[1], ref[1]):
        assert _rel(a, b) < 2e-5
    for a, b in zip(got[2], ref[2]):
        assert _rel(a, b) < 2e-5


@pytest.mark.parametrize('kind', [0, 1, 2])
@pytest.mark.parametrize('with_hd', [True, False])
def test_fused_tangent_forward_and_dual_backward(hip_backend, kind, with_hd):
    """e3gnn_conv_tangent_forward / e3gnn_conv_dual_backward (one launch each)
    against their definition -- three forward / four backward products --
    on the fp64 CPU double, over a ragged graph (isolated centres, a 40-edge
    centre, repeated neighbours); plus the accumulating forward / backward."""
    center, nbr, (h, Y, w), g, (hd, Yd, wd) = _problem(kind, hip_backend.dims, seed=10 + kind)
    gd = np.random.default_rng(99).normal(size=g.shape)
    cpu = CpuConvBackend()
    n, E = len(g), len(center)
    dx, dwd, dm = hip_backend.dims[kind]
    gc = conv_ops.ConvGraph(n, torch.tensor(center), torch.tensor(nbr), cpu)
    gh = conv_ops.ConvGraph(n, torch.tensor(center, device=DEV), torch.tensor(nbr, device=DEV),
                            hip_backend)
    T64 = lambda a: torch.tensor(a, dtype=torch.float64)                     # noqa: E731
    T32 = lambda a: torch.tensor(a, dtype=torch.float32, device=DEV)         # noqa: E731
    hd_c = T64(hd) if with_hd else None
    hd_h = T32(hd) if with_hd else None
    ref = cpu.tangent_forward(kind, gc, T64(h), hd_c, T64(Y), T64(Yd), T64(w), T64(wd),
                              out=torch.empty(n, dm, dtype=torch.float64))
    got = hip_backend.tangent_forward(kind, gh, T32(h), hd_h, T32(Y), T32(Yd), T32(w), T32(wd),
                                      out=torch.empty(n, dm, device=DEV))
    assert _rel(got, ref) < 2e-5
    base = T32(g)
    hip_backend.tangent_forward(kind, gh, T32(h), hd_h, T32(Y), T32(Yd), T32(w), T32(wd),
                                out=base, acc=True)
    assert _rel(base, ref + T64(g)) < 2e-5
    z = lambda *sh: torch.empty(*sh, dtype=torch.float64)                    # noqa: E731
    r = cpu.dual_backward(kind, gc, T64(h), hd_c, T64(Y), T64(Yd), T64(w), T64(wd), T64(g),
                          T64(gd), z(n, dx), z(n, dx) if with_hd else None, z(E, dwd), z(E, dwd))
    e = lambda *sh: torch.empty(*sh, device=DEV)                             # noqa: E731
    o = hip_backend.dual_backward(kind, gh, T32(h), hd_h, T32(Y), T32(Yd), T32(w), T32(wd),
                                  T32(g), T32(gd), e(n, dx), e(n, dx) if with_hd else None,
                                  e(E, dwd), e(E, dwd))
    for a, b in zip(o, r):
        assert (a is None) == (b is None)
        if a is not None:
            assert _rel(a, b) < 2e-5
    # accumulating single products: dh += , dY += , dw +=
    dh0, dY0, dw0 = T32(hd), T32(Yd), T32(wd)
    hip_backend.backward(kind, gh, T32(h), T32(Y), T32(w), T32(g), dh_out=dh0, dY_out=dY0,
                         dw_out=dw0, acc=conv_ops.ACC_DH | conv_ops.ACC_DY | conv_ops.ACC_DW)
    rh, rY, rw = cpu.backward(kind, gc, T64(h), T64(Y), T64(w), T64(g))
    for a, b in ((dh0, rh + T64(hd)), (dY0, rY + T64(Yd)), (dw0, rw + T64(wd))):
        assert _rel(a, b) < 2e-5


@pytest.mark.parametrize('normalize', [True, False])
def test_edge_geometry_kernels_vs_fp64(hip_backend, normalize):
    """The explicit step's edge-geometry kernels (e3gnn_edge_geometry*: Y /
    emb, dE/dr from (dE/dY, dE/demb), the tangent along the loss cotangent of
    the edge forces incl. the stress term, the Bessel-coefficient gradient,
    the per-atom force sum) against the float64 torch formulas of
    train_explicit._Geometry; unit-vector and raw-vector SH."""
    from sevennet_finetuning_amd import _lib
    from sevennet_finetuning_amd.train_explicit import _Geometry

    class M:
        cutoff, r_on, sh_normalize = 5.0, 4.5, normalize

    class P:
        lib = None

    class PH:
        lib = _lib.load()

    rng = np.random.default_rng(7)
    n, E, nb = 40, 300, 2
    center = np.sort(rng.integers(0, n, E))
    nbr = rng.integers(0, n, E)
    d = rng.normal(size=(E, 3))
    vec = d / np.linalg.norm(d, axis=1, keepdims=True) * rng.uniform(0.8, 4.99, (E, 1))
    batch = (np.arange(n) >= n // 2).astype(np.int64)
    coeffs = np.pi * np.arange(1, 9) / 5.0 * rng.uniform(0.9, 1.1, 8)
    cF, cS, vol = rng.normal(size=(n, 3)), rng.normal(size=(nb, 6)), rng.uniform(50, 80, nb)
    Yb, embb, embdb = rng.normal(size=(E, 9)), rng.normal(size=(E, 8)), rng.normal(size=(E, 8))
    T64 = lambda a: torch.tensor(a, dtype=torch.float64)                        # noqa: E731
    T32 = lambda a: torch.tensor(a, dtype=torch.float32, device=DEV)            # noqa: E731
    Tl = lambda a, dev: torch.tensor(a, dtype=torch.long, device=dev)           # noqa: E731
    gc, gh = _Geometry(M, P), _Geometry(M, PH)
    rc_ = gc.forward(T64(vec), T64(coeffs))
    rh = gh.forward(T32(vec), T32(coeffs))
    assert _rel(rh['Y'], rc_['Y']) < 1e-5 and _rel(rh['emb'], rc_['emb']) < 1e-5
    assert _rel(gh.vjp(rh, T32(Yb), T32(embb)), gc.vjp(rc_, T64(Yb), T64(embb))) < 1e-5
    graph = conv_ops.ConvGraph(n, Tl(center, DEV), Tl(nbr, DEV), hip_backend)
    Sc = {'center': Tl(center, 'cpu'), 'nbr': Tl(nbr, 'cpu'), 'batch': Tl(batch, 'cpu'),
          'vec': T64(vec), 'vol': T64(vol)}
    Sh = {'center': Tl(center, DEV), 'nbr': Tl(nbr, DEV), 'batch': Tl(batch, DEV),
          'vec': T32(vec), 'vol': T32(vol), 'graph': graph}
    for with_stress in (True, False):
        ec, eh = torch.empty(E, 8, dtype=torch.float64), torch.empty(E, 8, device=DEV)
        Ydc, rdc = gc.tangent(rc_, Sc, T64(cF), T64(cS) if with_stress else None, ec)
        Ydh, rdh = gh.tangent(rh, Sh, T32(cF), T32(cS) if with_stress else None, eh)
        for a, b in ((Ydh, Ydc), (eh, ec), (rdh, rdc)):
            assert _rel(a, b) < 1e-5
    cc = gc.coeff_grad(rc_, T64(embb), T64(embdb), rdc, T64(coeffs))
    ch = gh.coeff_grad(rh, T32(embb), T32(embdb), rdh, T32(coeffs))
    assert _rel(ch, cc) < 1e-5
    # per-atom force sum over the graph's CSR
    fij = rng.normal(size=(E, 3))
    F = torch.empty(n, 3, device=DEV)
    aux = graph.aux
    _lib.check(PH.lib.e3gnn_edge_forces_to_atoms(
        n, aux['row_ptr'].data_ptr(), aux['src_ptr'].data_ptr(), aux['src_perm'].data_ptr(),
        T32(fij).data_ptr(), F.data_ptr(), torch.cuda.current_stream().cuda_stream))
    ref = torch.zeros(n, 3, dtype=torch.float64).index_add(
        0, torch.cat([Tl(center, 'cpu'), Tl(nbr, 'cpu')]), torch.cat([T64(fij), -T64(fij)]))
    assert _rel(F, ref) < 1e-5


@pytest.mark.parametrize('pieces', [False, True])
@pytest.mark.parametrize('width', [384, 960, 224])
def test_radial_mlp_chain_kernels_vs_fp64(width, pieces):
    """e3gnn_radial_mlp_forward / _backward (whole chains per 16-row tile) vs
    the same chains as float64 GEMMs + element-wise steps (train_explicit's
    torch path): forward, tangent, first reverse and dual reverse; a row
    count that is not a multiple of 16; the three block widths; pieces: layer
    2 of the forward / tangent chains on bf16x6 (e3gnn_radial_mlp_forward_p
    with e3gnn_radial_mlp_w2_pieces' image) -- the same f32-grade bound."""
    from sevennet_finetuning_amd import _lib
    from sevennet_finetuning_amd.train_explicit import ExplicitStep, _Prims

    class FM:
        silu_norm = 1.679177
        def __init__(self, dev):
            self.flat = torch.empty(1, device=dev)
        def _act_lib(self):
            return _lib.load()

    def host(dev):
        h = type('Host', (), {k: getattr(ExplicitStep, k) for k in
                              ('_mlp_hip', '_mlp_fwd', '_mlp_rev', '_mlp_dual')})()
        h._stream = ExplicitStep._stream
        h.p = _Prims(FM(dev))
        return h

    rng = np.random.default_rng(width)
    E = 301
    Wn = [rng.normal(size=(8, 64)) / np.sqrt(8), rng.normal(size=(64, 64)) / 8,
          rng.normal(size=(64, width)) / 8]
    emb, embd = rng.normal(size=(E, 8)), rng.normal(size=(E, 8))
    WB = rng.normal(size=(2 * E, width))
    embb0 = rng.normal(size=(2 * E, 8))
    out = {}
    for dev, dt in (('cpu', torch.float64), (DEV, torch.float32)):
        T = lambda a: torch.tensor(a, dtype=dt, device=dev)           # noqa: E731
        z = lambda *sh: torch.zeros(*sh, dtype=dt, device=dev)        # noqa: E731
        h = host(dev)
        Ws = tuple(T(w) for w in Wn)
        h._w2p_of = {}
        if pieces and dev != 'cpu':
            lib = _lib.load()
            img = torch.empty(int(lib.e3gnn_radial_mlp_w2_piece_bytes(width)), dtype=torch.uint8, device=dev)
            _lib.check(lib.e3gnn_radial_mlp_w2_pieces(
                1, (ctypes.c_void_p * 1)(Ws[2].data_ptr()), (ctypes.c_int32 * 1)(width),
                (ctypes.c_void_p * 1)(img.data_ptr()), torch.cuda.current_stream().cuda_stream))
            h._w2p_of = {Ws[2].data_ptr(): img.data_ptr()}
        A1, H1, A2, H2, WT = z(2 * E, 64), z(2 * E, 64), z(2 * E, 64), z(2 * E, 64), z(2 * E, width)
        h._mlp_fwd(T(emb), Ws, None, None, A1[:E], H1[:E], A2[:E], H2[:E], WT[:E])
        h._mlp_fwd(T(embd), Ws, A1[:E], A2[:E], A1[E:], H1[E:], A2[E:], H2[E:], WT[E:])
        eb1 = T(embb0[:E])
        h._mlp_rev(T(WB[:E]), Ws, A1[:E], A2[:E], eb1)
        A2B, A1B, EBB = z(2 * E, 64), z(2 * E, 64), T(embb0)
        h._mlp_dual(T(WB), Ws, A1, A2, A2B, A1B, EBB)
        out[dev] = (A1, H1, A2, H2, WT, eb1, A2B, A1B, EBB)
    names = ('A1', 'H1', 'A2', 'H2', 'WT', 'embb', 'A2B', 'A1B', 'EMBB')
    for nm, a, b in zip(names, out[DEV], out['cpu']):
        assert _rel(a, b) < 2e-5, nm


@pytest.mark.parametrize('n,mean_deg,hub', [(5, 2, 0), (3000, 0.0005, 0), (1000, 6, 150), (3000, 6, 150),
                                             (20000, 28, 90)])
def test_conv_graph_csr_matches_numpy(hip_backend, n, mean_deg, hub):
    """row_ptr / src_ptr / src_perm of e3gnn_conv_graph against numpy: the
    transposed CSR lists each neighbour's edges in ascending edge id.  Sizes
    span one and several 1,024-count scan blocks, nodes without edges, and a
    hub neighbour with more than 64 incoming edges (the long-segment sort);
    the one-workgroup build (<= 3,072 nodes, <= 16,384 edges: n = 5, 1,000 and
    the sparse 3,000) and the multi-launch one (the rest)."""
    rng = np.random.default_rng(n)
    deg = rng.poisson(mean_deg, n)
    deg[::11] = 0
    center = np.repeat(np.arange(n), deg)
    nbr = rng.integers(0, n, len(center))
    if hub:
        nbr[rng.choice(len(center), hub, replace=False)] = n // 2
    g = conv_ops.ConvGraph(n, torch.tensor(center, device=DEV), torch.tensor(nbr, device=DEV),
                           hip_backend)
    aux = g.aux
    row_ptr = np.concatenate([[0], np.cumsum(deg)])
    cnt = np.bincount(nbr, minlength=n)
    src_ptr = np.concatenate([[0], np.cumsum(cnt)])
    src_perm = np.argsort(nbr, kind='stable')
    assert np.array_equal(aux['row_ptr'].cpu().numpy(), row_ptr)
    assert np.array_equal(aux['src_ptr'].cpu().numpy(), src_ptr)
    assert np.array_equal(aux['src_perm'].cpu().numpy()[:len(center)], src_perm)
    # the in-place rebuild of a captured step from int64 edge_index rows (one
    # launch up to e3gnn_conv_graph_small_max_nodes(), the int32 copies +
    # multi-launch build beyond): new neighbours, same edge count
    nbr2 = rng.permutation(nbr)
    ei = torch.tensor(np.stack([center, nbr2]), device=DEV, dtype=torch.int64)
    g.rebuild(ei[0], ei[1])
    cnt2 = np.bincount(nbr2, minlength=n)
    assert np.array_equal(aux['center'].cpu().numpy(), center)
    assert np.array_equal(aux['nbr'].cpu().numpy(), nbr2)
    assert np.array_equal(aux['row_ptr'].cpu().numpy(), row_ptr)
    assert np.array_equal(aux['src_ptr'].cpu().numpy(), np.concatenate([[0], np.cumsum(cnt2)]))
    assert np.array_equal(aux['src_perm'].cpu().numpy()[:len(center)], np.argsort(nbr2, kind='stable'))


def test_conv_graph_rejects_unsorted(hip_backend):
    from sevennet_finetuning_amd._lib import E3GNNError
    with pytest.raises(E3GNNError, match='not sorted'):
        conv_ops.ConvGraph(4, torch.tensor([0, 2, 1], device=DEV),
                           torch.tensor([1, 1, 1], device=DEV), hip_backend)
    with pytest.raises(E3GNNError, match='out of'):
        conv_ops.ConvGraph(4, torch.tensor([0, 1, 2], device=DEV),
                           torch.tensor([1, 9, 1], device=DEV), hip_backend)
    g = conv_ops.ConvGraph(4, torch.tensor([0, 1, 2], device=DEV), torch.tensor([1, 2, 1], device=DEV),
                           hip_backend)
    with pytest.raises(E3GNNError, match='not sorted'):   # the int64 one-launch rebuild validates too
        g.rebuild(torch.tensor([0, 2, 1], device=DEV), torch.tensor([1, 1, 1], device=DEV))
    with pytest.raises(E3GNNError, match='out of'):
        g.rebuild(torch.tensor([0, 1, 2], device=DEV), torch.tensor([1, -1, 1], device=DEV))
    # int64 indices are range-checked before narrowing: 2^32 + 1 is not 1
    with pytest.raises(E3GNNError, match='out of'):
        g.rebuild(torch.tensor([0, 1, 2], device=DEV), torch.tensor([1, (1 << 32) + 1, 1], device=DEV))
    with pytest.raises(E3GNNError, match='edge_center out of'):
        g.rebuild(torch.tensor([0, (1 << 32) + 1, 2], device=DEV), torch.tensor([1, 2, 1], device=DEV))
    # a negative centre before a valid one: reported, and the row_ptr fill of
    # the next edge stays inside the buffer (the graph still rebuilds after)
    with pytest.raises(E3GNNError, match='edge_center out of'):
        g.rebuild(torch.tensor([-7, 1, 2], device=DEV), torch.tensor([1, 2, 1], device=DEV))
    g.rebuild(torch.tensor([0, 1, 2], device=DEV), torch.tensor([1, 2, 1], device=DEV))
    assert g.aux['row_ptr'].cpu().tolist() == [0, 1, 2, 3, 3]


@pytest.fixture(scope='module')
def models(hip_backend):
    from sevennet_finetuning_amd.nn import SevenNetTrainable
    m32 = SevenNetTrainable(device=DEV)
    m64 = SevenNetTrainable(device='cpu', conv_backend=CpuConvBackend(), dtype=torch.float64)
    return m32, m64


def _batch(seeds, cells=(3, 3, 3), labels=True):
    gs = []
    for s in seeds:
        pos, cell, types = ft_structure(s, cells)
        rng = np.random.default_rng(1000 + s)
        lab = dict(energy=-4.0 * len(pos), force=rng.normal(0, 0.3, (len(pos), 3)),
                   stress=rng.normal(0, 2e-3, 6)) if labels else {}
        gs.append(train.labeled_graph(pos, cell, types, 5.0, **lab))
    return gs


def test_trainable_energy_force_stress_vs_fp64(models):
    m32, m64 = models
    gs = _batch([0, 1, 2])
    m32.train(False)
    m64.train(False)
    a = m32(train.collate(gs, device=DEV, dtype=torch.float32))
    b = m64(train.collate(gs, dtype=torch.float64))
    e32, e64 = a[KEY.PRED_TOTAL_ENERGY].detach().cpu().double(), b[KEY.PRED_TOTAL_ENERGY].detach()
    assert float(((e32 - e64).abs() / e64.abs()).max()) < 2e-6
    assert float((a[KEY.PRED_FORCE].detach().cpu().double() - b[KEY.PRED_FORCE]).abs().max()) \
        < 1e-4
    assert float((a[KEY.PRED_STRESS].detach().cpu().double() - b[KEY.PRED_STRESS]).abs().max()) \
        < 2e-6


def test_force_loss_parameter_gradients_vs_fp64(models):
    """The double-backward gradient every fine-tune step takes (force loss,
    create_graph=True) through the HIP kernels, against float64."""
    m32, m64 = models
    cfg = {'loss': 'mse', 'force_loss_weight': 1.0, 'stress_loss_weight': 1e-2,
           'is_train_stress': True, 'continue': {'fisher_information': False,
                                                 'opt_params': False}}
    fns = train.get_loss_functions_from_config(cfg)
    gs = _batch([3, 4])
    grads = []
    for m, kw in ((m32, dict(device=DEV, dtype=torch.float32)), (m64, dict(dtype=torch.float64))):
        m.train(True)
        m.zero_grad()
        out = m(train.collate(gs, **kw))
        loss = sum(f.get_loss(out, m) * w for f, w in fns)
        loss.backward()
        grads.append(m.flat_grad.detach().cpu().double().clone())
        m.train(False)
    g32, g64 = grads
    assert float(g64.abs().max()) > 0
    assert float((g32 - g64).norm() / g64.norm()) < 1e-4
    # per tensor, relative to each tensor's own scale
    worst = []
    for name, (off, n, _) in m64.slices.items():
        ref = g64[off:off + n]
        if float(ref.abs().max()) == 0.0:
            assert float(g32[off:off + n].abs().max()) == 0.0, name
            continue
        worst.append((float((g32[off:off + n] - ref).norm() / ref.norm()), name))
    worst.sort(reverse=True)
    print('autograd-path per-tensor relative gradient errors, worst five:', worst[:5])
    for err, name in worst:
        assert err < 2e-4, name


def test_explicit_step_gradients_vs_fp64(models):
    """The hand-scheduled derivatives (train_explicit.py: first reverse for
    the forces, tangent forward along dL/dF, one reverse sweep) on the HIP
    kernels -- the Trainer's default path -- against float64 autograd of the
    same loss; plus the dual act / gate kernels against their torch forms."""
    from sevennet_finetuning_amd.train_explicit import ExplicitStep, _Gate, _Prims
    m32, m64 = models
    cfg = {'loss': 'huber', 'loss_param': {'delta': 0.01}, 'force_loss_weight': 1.0,
           'stress_loss_weight': 1e-2, 'is_train_stress': True,
           'continue': {'fisher_information': False, 'opt_params': False}}
    fns = train.get_loss_functions_from_config(cfg)
    gs = _batch([8, 9])
    step = ExplicitStep(m32)
    m32.zero_grad()
    out = step.forward(train.collate(gs, device=DEV, dtype=torch.float32))
    loss = sum(f.get_loss(out, m32) * w for f, w in fns)
    loss.backward()
    step.backward(out[KEY.PRED_TOTAL_ENERGY].grad, out[KEY.PRED_FORCE].grad,
                  out[KEY.PRED_STRESS].grad)
    g32 = m32.flat_grad.detach().cpu().double().clone()
    m64.train(True)
    m64.zero_grad()
    o64 = m64(train.collate(gs, dtype=torch.float64))
    sum(f.get_loss(o64, m64) * w for f, w in fns).backward()
    m64.train(False)
    g64 = m64.flat_grad.detach().clone()
    assert float((out[KEY.PRED_FORCE].detach().cpu().double() - o64[KEY.PRED_FORCE]).abs().max()) < 1e-4
    assert float((g32 - g64).norm() / g64.norm()) < 1e-4
    worst = []
    for name, (off, n, _) in m64.slices.items():
        ref = g64[off:off + n]
        if float(ref.abs().max()) == 0.0:
            assert float(g32[off:off + n].abs().max()) == 0.0, name
            continue
        worst.append((float((g32[off:off + n] - ref).norm() / ref.norm()), name))
    worst.sort(reverse=True)
    print('explicit-step per-tensor relative gradient errors, worst five:', worst[:5])
    for err, name in worst:   # measured ~2e-6 at worst (round 5)
        assert err < 2e-4, name
    # the dual kernels against the torch forms of the same module
    torch.manual_seed(0)
    p = _Prims(m32)
    x, xd, g, gd = (torch.randn(1000, device=DEV) for _ in range(4))
    a0, a1 = p.act_dual(x, xd, g, gd)
    d1, d2 = p._d(x)
    assert torch.allclose(a0, g * d1 + gd * d2 * xd, atol=1e-5) and torch.allclose(a1, gd * d1, atol=1e-5)
    gate = _Gate(m32.blocks[1]['gate'], p)
    y, yd = torch.randn(50, 576, device=DEV), torch.randn(50, 576, device=DEV)
    xb, xdb = torch.randn(50, 480, device=DEV), torch.randn(50, 480, device=DEV)
    lib, gate.p.lib = gate.p.lib, None          # torch forms
    ref_jvp, ref_dual = gate.jvp(y, yd), gate.dual_vjp(y, yd, xb, xdb)
    gate.p.lib = lib
    assert torch.allclose(gate.jvp(y, yd), ref_jvp, atol=1e-5)
    got = gate.dual_vjp(y, yd, xb, xdb)
    assert torch.allclose(got[0], ref_dual[0], atol=1e-4) and torch.allclose(got[1], ref_dual[1], atol=1e-5)


def test_explicit_and_autograd_trainers_take_the_same_step(models):
    """Trainer with explicit_grad (default) and with autograd: one rehearsal
    step (SGD: the update is the gradient) from the same parameters makes the
    same parameter change."""
    from sevennet_finetuning_amd.nn import SevenNetTrainable
    cfg = {'loss': 'mse', 'force_loss_weight': 0.5, 'stress_loss_weight': 1e-3,
           'is_train_stress': True, 'optimizer': 'sgd', 'optim_param': {'lr': 1e-3},
           'scheduler': 'exponentiallr', 'scheduler_param': {'gamma': 0.99},
           'continue': {'fisher_information': False, 'opt_params': False}}
    b = train.collate(_batch([11, 12]), device=DEV, dtype=torch.float32)
    mem = train.collate(_batch([13]), device=DEV, dtype=torch.float32)
    deltas = []
    for explicit in (True, False):
        m = SevenNetTrainable(device=DEV)
        before = m.flat.detach().clone()
        tr = train.Trainer(m, dict(cfg, explicit_grad=explicit))
        assert (tr.explicit is not None) == explicit
        tr.rehearsal_step(b, mem)
        deltas.append((m.flat.detach() - before).double())
    assert float(deltas[1].norm()) > 0
    assert float((deltas[0] - deltas[1]).norm() / deltas[1].norm()) < 1e-4


def test_trainer_on_the_runtime_table_backend_uses_autograd(models):
    """SevenNet-0 on GenericHipConvBackend: the Trainer must not pick the
    explicit step (it drives the specialised kernels only), and its SGD step
    equals the specialised backend's explicit step."""
    from sevennet_finetuning_amd import conv_ops
    from sevennet_finetuning_amd.nn import SevenNetTrainable
    cfg = {'loss': 'mse', 'force_loss_weight': 0.5, 'stress_loss_weight': 1e-3,
           'is_train_stress': True, 'optimizer': 'sgd', 'optim_param': {'lr': 1e-3},
           'scheduler': 'exponentiallr', 'scheduler_param': {'gamma': 0.99},
           'continue': {'fisher_information': False, 'opt_params': False}}
    b = train.collate(_batch([11, 12]), device=DEV, dtype=torch.float32)
    mem = train.collate(_batch([13]), device=DEV, dtype=torch.float32)
    deltas = []
    for generic in (False, True):
        kw = {'conv_backend': conv_ops.GenericHipConvBackend()} if generic else {}
        m = SevenNetTrainable(device=DEV, **kw)
        before = m.flat.detach().clone()
        tr = train.Trainer(m, cfg)
        assert (tr.explicit is None) == generic
        tr.rehearsal_step(b, mem)
        deltas.append((m.flat.detach() - before).double())
    with pytest.raises(Exception, match='no fused tangent forward'):
        conv_ops.GenericHipConvBackend().tangent_forward(0, None, None, None, None, None,
                                                         None, None, None)
    assert float(deltas[0].norm()) > 0
    assert float((deltas[0] - deltas[1]).norm() / deltas[0].norm()) < 1e-4


def test_rehearsal_ewc_steps_reduce_loss(models):
    """A few rehearsal+EWC Adam steps (the reference's FT_w_reEWC recipe,
    Huber delta 0.01) on fixed batches lower the data loss of both batches,
    and the EWC term grows from exactly zero at the optimum."""
    from sevennet_finetuning_amd.nn import SevenNetTrainable
    m = SevenNetTrainable(device=DEV)
    fisher = {n: torch.full_like(p, 1e-3) for n, p in m.named_parameters()}
    opt = {n: p.detach().clone() for n, p in m.named_parameters()}
    cfg = {'loss': 'huber', 'loss_param': {'delta': 0.01}, 'force_loss_weight': 1.0,
           'stress_loss_weight': 0.01, 'is_train_stress': True, 'optimizer': 'adam',
           'optim_param': {'lr': 1e-5}, 'scheduler': 'exponentiallr',
           'scheduler_param': {'gamma': 0.99},
           'continue': {'fisher_information': fisher, 'opt_params': opt, 'ewc_lambda': 1e2},
           'device': DEV}
    tr = train.Trainer(m, cfg)
    data_fns = [(f, w) for f, w in tr.loss_functions if not isinstance(f, train.EWCLoss)]
    ewc = [f for f, _ in tr.loss_functions if isinstance(f, train.EWCLoss)][0]
    b = train.collate(_batch([5, 6]), device=DEV, dtype=torch.float32)
    mem = train.collate(_batch([7]), device=DEV, dtype=torch.float32)

    def data_loss():
        m.train(True)
        return sum(float(sum(f.get_loss(m(x), m) * w for f, w in data_fns).detach())
                   for x in (b, mem))

    before = data_loss()
    assert float(ewc.get_loss({}, m)) == 0.0
    for _ in range(5):
        loss, mloss = tr.rehearsal_step(b, mem)
        assert torch.isfinite(loss).all() and torch.isfinite(mloss).all()
    after = data_loss()
    m.train(False)
    assert after < before
    assert float(ewc.get_loss({}, m)) > 0.0


def test_graphed_rehearsal_step_equals_eager():
    """The HIP-graph-captured rehearsal step (train.GraphedRehearsalStep)
    reproduces the eager step: same losses and parameters after steps on
    changing batches of one shape (one with its edges in a random order: the
    graphed step sorts them by centre like the eager model), a new shape is
    captured separately, and once hip_graph_max shapes are cached a further
    shape runs eagerly with the same result as the eager trainer."""
    from sevennet_finetuning_amd.nn import SevenNetTrainable

    def run(graph, batches, third):
        m = SevenNetTrainable(device=DEV)
        fisher = {n: torch.full_like(p, 1e-3) for n, p in m.named_parameters()}
        opt = {n: p.detach().clone() for n, p in m.named_parameters()}
        cfg = {'loss': 'huber', 'loss_param': {'delta': 0.01}, 'force_loss_weight': 1.0,
               'stress_loss_weight': 0.01, 'is_train_stress': True, 'optimizer': 'adam',
               'optim_param': {'lr': 1e-4}, 'scheduler': 'exponentiallr',
               'scheduler_param': {'gamma': 0.99}, 'device': DEV, 'hip_graph': graph,
               'hip_graph_max': 2, 'continue': {'fisher_information': fisher,
                                                'opt_params': opt, 'ewc_lambda': 1e2}}
        tr = train.Trainer(m, cfg)
        m.train(True)
        losses = [tuple(float(x) for x in tr.rehearsal_step(b, mm)) for b, mm in batches]
        cached = len(tr._graphed.cache) if graph else 0
        losses.append(tuple(float(x) for x in tr.rehearsal_step(*third)))
        if graph:   # the third shape ran eagerly: nothing new captured
            assert len(tr._graphed.cache) == cached == 2
        return m.flat.detach().double().cpu(), losses

    def coll(seeds, cells=(3, 3, 3)):
        return train.collate(_batch(seeds, cells), device=DEV, dtype=torch.float32)
    batches = [(coll([1, 2]), coll([3])), (coll([4, 5]), coll([6])), (coll([7, 8]), coll([9])),
               (coll([10], (2, 2, 2)), coll([11]))]
    # one label NaN: the static (masked) loss drops it like the eager one
    batches[1][0][KEY.FORCE][3, 1] = float('nan')
    # edges of one batch in a random order
    b2 = batches[2][0]
    perm = torch.as_tensor(np.random.default_rng(0).permutation(b2[KEY.EDGE_IDX].shape[1]),
                           device=DEV)
    for k in (KEY.EDGE_IDX, KEY.EDGE_VEC):
        b2[k] = b2[k][:, perm] if k == KEY.EDGE_IDX else b2[k][perm]
    # collate's EDGE_SORTED flag is left in place: it names the old edge_index
    # storage, so it is stale by itself and the steps sort the edges again
    assert not train.edges_marked_sorted(b2)
    third = (coll([12], (2, 2, 1)), coll([13], (2, 2, 1)))
    theta0 = SevenNetTrainable(device=DEV).flat.detach().double().cpu()
    fe, le = run(False, batches, third)
    fg, lg = run(True, batches, third)
    assert len(le) == len(lg) == 5
    for a, b in zip(le, lg):
        assert abs(a[0] - b[0]) <= 1e-5 * abs(a[0]) and abs(a[1] - b[1]) <= 1e-5 * abs(a[1])
    # Adam normalises every component: where a gradient is ~0, fp32 rounding
    # differences between the capturable and the eager update flip its sign,
    # so the parameter MOVES are compared in norm, not element by element
    de, dg = fe - theta0, fg - theta0
    assert float((de - dg).norm() / de.norm()) < 1e-2


def test_graphed_step_replays_of_equal_shapes_equal_eager():
    """Many replays of ONE captured graph whose new and memory batches have
    the same shapes (bench_train's case: the graph's memory plan then reuses
    the first pass's buffers in the second): every step's losses and the
    parameters equal the eager trainer's.  (A captured hipMemsetAsync node did
    not re-zero the convolution backward's accumulators on replay; the ops now
    zero them with a kernel.)"""
    from sevennet_finetuning_amd.nn import SevenNetTrainable

    def make(graph):
        m = SevenNetTrainable(device=DEV)
        fisher = {n: torch.full_like(p, 1e-3) for n, p in m.named_parameters()}
        opt = {n: p.detach().clone() for n, p in m.named_parameters()}
        cfg = {'loss': 'huber', 'loss_param': {'delta': 0.01}, 'force_loss_weight': 1.0,
               'stress_loss_weight': 0.01, 'is_train_stress': True, 'optimizer': 'adam',
               'optim_param': {'lr': 1e-5}, 'scheduler': 'exponentiallr',
               'scheduler_param': {'gamma': 0.99}, 'device': DEV, 'hip_graph': graph,
               'continue': {'fisher_information': fisher, 'opt_params': opt,
                            'ewc_lambda': 1e5}}
        tr = train.Trainer(m, cfg)
        m.train(True)
        return m, tr

    def coll(seeds):
        return train.collate(_batch(seeds), device=DEV, dtype=torch.float32)
    pairs = [(coll([1, 2]), coll([3, 4])), (coll([5, 6]), coll([7, 8]))]
    assert all(a[KEY.EDGE_IDX].shape == b[KEY.EDGE_IDX].shape for a, b in pairs)
    me, te = make(False)
    le = [[float(x) for x in te.rehearsal_step(*pairs[i % 2])] for i in range(5)]
    mg, tg = make(True)
    lg = [[float(x) for x in tg.rehearsal_step(*pairs[i % 2])] for i in range(5)]
    for i in range(5):
        for a, c in zip(le[i], lg[i]):
            assert abs(a - c) <= 1e-5 * abs(a), (i, le[i], lg[i])
    assert len(tg._graphed.cache) == 1
    # Adam normalises each gradient entry: one whose gradient is ~0 moves by up
    # to lr per step in the direction of its rounding noise (torch's atomic
    # scatter-adds differ run to run), so the bound on any entry is 2 lr x steps;
    # all but a handful agree to fp32 rounding
    d = (me.flat - mg.flat).abs()
    assert float(d.max()) <= 2 * 1e-5 * 5
    assert float((d > 1e-6).float().mean()) < 1e-3


def test_graphed_small_shape_replayed_after_workspace_growth():
    """A graph captured on a small batch shape, then a larger shape whose
    grouped-GEMM workspaces outgrow the first ones (the old buffers are
    replaced), then the small graph replayed: its captured workspace
    addresses must still be owned by the trainer, so the replays equal the
    eager trainer's steps."""
    from sevennet_finetuning_amd.nn import SevenNetTrainable

    def make(graph):
        m = SevenNetTrainable(device=DEV)
        cfg = {'loss': 'mse', 'force_loss_weight': 1.0, 'stress_loss_weight': 0.01,
               'is_train_stress': True, 'optimizer': 'adam', 'optim_param': {'lr': 1e-5},
               'scheduler': 'exponentiallr', 'scheduler_param': {'gamma': 0.99}, 'device': DEV,
               'hip_graph': graph}
        tr = train.Trainer(m, cfg)
        m.train(True)
        return m, tr

    def coll(seeds, cells):
        return train.collate(_batch(seeds, cells), device=DEV, dtype=torch.float32)
    small = (coll([1], (2, 2, 1)), coll([2], (2, 2, 1)))
    large = (coll([3, 4, 5], (3, 3, 3)), coll([6, 7], (3, 3, 3)))
    seq = [small, large, small, large, small]
    me, te = make(False)
    le = [[float(x) for x in te.rehearsal_step(*b)] for b in seq]
    mg, tg = make(True)
    gm = tg.explicit.gm
    lg = [[float(x) for x in tg.rehearsal_step(*b)] for b in seq]
    assert len(tg._graphed.cache) == 2
    for i in range(len(seq)):
        for a, c in zip(le[i], lg[i]):
            assert abs(a - c) <= 1e-5 * abs(a) + 1e-12, (i, le[i], lg[i])
    assert gm.lib is not None   # the library's grouped GEMM ran (its workspaces are what is tested)
    d = (me.flat - mg.flat).abs()
    assert float(d.max()) <= 2 * 1e-5 * len(seq)


def test_graphed_ewc_step_interleaved_with_eager_trainer():
    """An eager and a graphed EWC trainer stepped alternately in one process
    (round 3 diagnostic, git history): every step's losses and the final
    parameters equal.  Round 2 shipped this broken: the graphed trainer's
    REPORTED loss came back ~800 (parameters right) once other work ran
    between its replays -- the EWC term's torch.sum over the 842k-entry flat
    buffer is a multi-block reduction that did not survive graph replay here;
    train._sum_two_level keeps every reduction inside one block."""
    from sevennet_finetuning_amd.nn import SevenNetTrainable

    def make(graph):
        m = SevenNetTrainable(device=DEV)
        fisher = {n: torch.full_like(p, 1e-3) for n, p in m.named_parameters()}
        opt = {n: p.detach().clone() for n, p in m.named_parameters()}
        cfg = {'loss': 'huber', 'loss_param': {'delta': 0.01}, 'force_loss_weight': 1.0,
               'stress_loss_weight': 0.01, 'is_train_stress': True, 'optimizer': 'adam',
               'optim_param': {'lr': 1e-5}, 'scheduler': 'exponentiallr',
               'scheduler_param': {'gamma': 0.99}, 'device': DEV, 'hip_graph': graph,
               'continue': {'fisher_information': fisher, 'opt_params': opt,
                            'ewc_lambda': 1e5}}
        tr = train.Trainer(m, cfg)
        m.train(True)
        return m, tr

    def coll(seeds):
        return train.collate(_batch(seeds), device=DEV, dtype=torch.float32)
    pairs = [(coll([1, 2]), coll([3, 4])), (coll([5, 6]), coll([7, 8]))]
    me, te = make(False)
    mg, tg = make(True)
    for i in range(5):
        le = [float(x) for x in te.rehearsal_step(*pairs[i % 2])]
        torch.cuda.synchronize()
        lg = [float(x) for x in tg.rehearsal_step(*pairs[i % 2])]
        torch.cuda.synchronize()
        for a, c in zip(le, lg):
            assert abs(a - c) <= 1e-5 * abs(a), (i, le, lg)
    d = (me.flat - mg.flat).abs()
    assert float(d.max()) <= 2 * 1e-5 * 5
    assert float((d > 1e-6).float().mean()) < 1e-3


def test_two_level_sum_in_a_replayed_graph():
    """The reduction form of the EWC loss reproduces the eager sum on every
    replay of a captured graph, with other reductions run between replays."""
    N = 842623
    x = torch.randn(N, device=DEV)
    y = torch.randn(N, device=DEV)
    fn = lambda v: train._sum_two_level(v * v)   # noqa: E731
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn(x)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = fn(x)
    for _ in range(4):
        x.mul_(1.01)
        g.replay()
        got = out.clone()
        _ = (y * y).sum()
        torch.cuda.synchronize()
        ref = (x.double() ** 2).sum()
        assert abs(float(got) - float(ref)) <= 1e-5 * float(ref)


def test_scaled_silu_op_derivatives():
    """e3gnn_act (fused scale * silu) against torch's composite in float64:
    value, first and second derivatives."""
    from sevennet_finetuning_amd import _lib
    lib = _lib.load()
    rng = np.random.default_rng(3)
    xv, gv, pv = (rng.normal(0, 3, (257, 33)) for _ in range(3))

    def run(fn, dtype, dev):
        x = torch.tensor(xv, dtype=dtype, device=dev, requires_grad=True)
        g = torch.tensor(gv, dtype=dtype, device=dev)
        pr = torch.tensor(pv, dtype=dtype, device=dev)
        y = fn(x)
        d1, = torch.autograd.grad((y * g).sum(), [x], create_graph=True)
        d2, = torch.autograd.grad((d1 * pr).sum(), [x])
        return y, d1, d2
    c = 1.679177
    got = run(lambda x: conv_ops.scaled_silu(x, c, lib), torch.float32, DEV)
    ref = run(lambda x: torch.nn.functional.silu(x) * c, torch.float64, 'cpu')
    for a, b in zip(got, ref):
        assert _rel(a, b) < 2e-6


def test_scaled_silu_op_noncontiguous_input_second_order():
    """The gate feeds column slices (non-contiguous views) to the activation;
    the second-order chain must still reach the sliced tensor."""
    from sevennet_finetuning_amd import _lib
    lib = _lib.load()
    rng = np.random.default_rng(4)
    base_v, gv, pv = rng.normal(0, 2, (64, 40)), rng.normal(size=(64, 16)), rng.normal(size=(64, 40))

    def run(fn, dtype, dev):
        base = torch.tensor(base_v, dtype=dtype, device=dev, requires_grad=True)
        x = base.split([16, 24], dim=1)[0]          # non-contiguous
        y = fn(x)
        g = torch.tensor(gv, dtype=dtype, device=dev)
        d1, = torch.autograd.grad((y * g).sum(), [base], create_graph=True)
        d2, = torch.autograd.grad((d1 * torch.tensor(pv, dtype=dtype, device=dev)).sum(), [base])
        return d1, d2
    c = 1.679177
    got = run(lambda x: conv_ops.scaled_silu(x, c, lib), torch.float32, DEV)
    ref = run(lambda x: torch.nn.functional.silu(x) * c, torch.float64, 'cpu')
    for a, b in zip(got, ref):
        assert _rel(a, b) < 2e-6


def test_fused_gate_op_derivatives():
    """e3gnn_gate (fused e3nn Gate of the trainable model) against the torch
    composite in float64: value, first and second derivatives, through a
    column slice of a wider tensor (the gate input is a view in the model)."""
    from sevennet_finetuning_amd import _lib
    lib = _lib.load()
    scal, gated = [(128, 0)], [(64, 1), (32, 2)]
    dims = conv_ops.gate_dims(scal, gated)
    c = 1.679177
    rng = np.random.default_rng(5)
    din, dout = int(dims[2]), int(dims[3])
    base_v = rng.normal(0, 1.5, (37, din + 7))
    gv, pv = rng.normal(size=(37, dout)), rng.normal(size=(37, din + 7))

    def composite(x):
        act = lambda t: torch.nn.functional.silu(t) * c  # noqa: E731
        s, g = act(x[:, :128]), act(x[:, 128:224])
        b1 = x[:, 224:416].reshape(-1, 64, 3) * g[:, :64].unsqueeze(-1)
        b2 = x[:, 416:576].reshape(-1, 32, 5) * g[:, 64:96].unsqueeze(-1)
        return torch.cat([s, b1.reshape(len(x), -1), b2.reshape(len(x), -1)], 1)

    def run(fn, dtype, dev):
        base = torch.tensor(base_v, dtype=dtype, device=dev, requires_grad=True)
        x = base[:, 3:3 + din]
        y = fn(x)
        d1, = torch.autograd.grad((y * torch.tensor(gv, dtype=dtype, device=dev)).sum(), [base],
                                  create_graph=True)
        d2, = torch.autograd.grad((d1 * torch.tensor(pv, dtype=dtype, device=dev)).sum(), [base])
        return y, d1, d2
    got = run(lambda x: conv_ops.gate(x, dims, c, lib), torch.float32, DEV)
    ref = run(composite, torch.float64, 'cpu')
    for a, b in zip(got, ref):
        assert _rel(a, b) < 2e-6


def test_multi_rank_graphed_step_equals_eager(tmp_path):
    """is_ddp + hip_graph: the rehearsal step as three captured segments
    replayed around the two gradient all-reduces (train.GraphedRehearsalStep),
    two gloo ranks on the GPU, equals the eager multi-rank step: same losses
    on every rank and step, ranks hold identical parameters, and the
    parameters equal the eager run's up to Adam's per-step sign-flip bound."""
    import socket
    import torch.multiprocessing as mp
    from _train_workers import ddp_rehearsal_worker
    res = {}
    for graph in (False, True):
        with socket.socket() as sk:
            sk.bind(('127.0.0.1', 0))
            port = sk.getsockname()[1]
        out = str(tmp_path / f'ddp_{int(graph)}')
        mp.spawn(ddp_rehearsal_worker, args=(2, port, graph, out), nprocs=2, join=True)
        res[graph] = [np.load(out + f'.{r}.npz') for r in range(2)]
    for r in range(2):
        le, lg = res[False][r]['losses'], res[True][r]['losses']
        assert np.all(np.abs(le - lg) <= 1e-5 * np.abs(le)), (r, le, lg)
        assert int(res[True][r]['n_graphs']) == 1
    for graph in (False, True):   # DDP: every rank holds the same parameters
        assert np.array_equal(res[graph][0]['flat'], res[graph][1]['flat'])
    d = np.abs(res[False][0]['flat'] - res[True][0]['flat'])
    assert d.max() <= 2 * 1e-5 * 4
    assert (d > 1e-6).mean() < 1e-3


def test_grouped_gemm_matches_fp64():
    """e3gnn_gemm_grouped (csrc/tgemm.hip), the fine-tune step's dense products:
    op(A) op(B) [+ op(A2) op(B2)] with every transpose combination, alpha /
    beta, ragged tails, a split-K weight gradient (K = 24,192 rows, the
    stacked edge count) and a K-concatenated pair, several problems in one
    launch, both tile shapes (64 x 64 for the 1100 x 1000 and the split-K
    products, 32 x 32 with the waves over k for the small ones) -- against float64 torch (f32 MFMA accumulation: 2e-6 relative to
    the output's scale); deterministic bitwise on repetition."""
    from sevennet_finetuning_amd.train_explicit import _Gemms

    class _M:   # the helper takes the library from the model's accessor
        flat = torch.empty(1, device=DEV)

        @staticmethod
        def _act_lib():
            from sevennet_finetuning_amd import _lib
            return _lib.load()
    gm = _Gemms(_M())
    g = torch.Generator(device='cpu').manual_seed(0)
    rnd = lambda *s: torch.randn(*s, generator=g).to(DEV)   # noqa: E731
    cases = []
    for (m, n, k, ta, tb) in [(432, 480, 576, 0, 0), (433, 97, 61, 1, 0), (64, 960, 24192, 1, 0),
                              (221, 64, 130, 0, 1), (37, 29, 17, 1, 1), (1, 64, 128, 0, 0),
                              (864, 1, 64, 0, 0), (1100, 1000, 96, 0, 1)]:
        A = rnd(k, m).t() if ta else rnd(m, k)
        B = rnd(n, k).t() if tb else rnd(k, n)
        cases.append((A, B))
    outs = [[]]
    for i, (A, B) in enumerate(cases):
        C = rnd(A.shape[0], B.shape[1])
        outs[0].append((C.clone(), C))
        gm.add(C, A, B, alpha=0.5 if i % 2 else 1.0, beta=i % 2)
    gm.flush()
    for i, ((C0, C), (A, B)) in enumerate(zip(outs[0], cases)):
        ref = A.double() @ B.double() * (0.5 if i % 2 else 1.0) + (C0.double() if i % 2 else 0)
        scale = float(ref.abs().max())
        assert float((C.double() - ref).abs().max()) <= 2e-6 * scale * max(1.0, A.shape[1] / 4096) ** 0.5, i
    # K-concatenated pair with transposed operands (x W1^T + y W2^T)
    x, W1, y, W2 = rnd(300, 480), rnd(480, 480), rnd(300, 576), rnd(480, 576)
    C = torch.empty(300, 480, device=DEV)
    gm.add(C, x, W1.t(), A2=y, B2=W2.t())
    gm.flush()
    ref = x.double() @ W1.double().t() + y.double() @ W2.double().t()
    assert float((C.double() - ref).abs().max()) <= 2e-6 * float(ref.abs().max())
    # bitwise determinism of the split-K path
    A, B = cases[2]
    r1, r2 = torch.empty(64, 960, device=DEV), torch.empty(64, 960, device=DEV)
    gm.add(r1, A, B)
    gm.flush()
    gm.add(r2, A, B)
    gm.flush()
    assert torch.equal(r1, r2)
    # deferred split-K reductions (E3GNN_GEMM_DEFER_REDUCE + e3gnn_gemm_reduce,
    # the fine-tune sweep's weight gradients): bitwise the immediate result,
    # over several launches, beta 0 / 1, split and unsplit problems mixed
    outs = []
    for defer in (False, True):
        Cs = [torch.ones(64, 960, device=DEV), torch.ones(433, 97, device=DEV), torch.ones(64, 960, device=DEV)]
        if defer:
            gm.begin_defer()
        gm.add(Cs[0], A, B, alpha=0.5, beta=1, wgrad=True)
        gm.add(Cs[1], *cases[1], wgrad=True)
        gm.flush()
        gm.add(Cs[2], A, B, beta=0, wgrad=True)
        gm.flush()
        if defer:
            assert gm.defer and len(gm.defer) == 2    # the two split problems wait
            gm.finish_defer()
        outs.append(Cs)
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize('loss', ['mse', 'huber'])
def test_fused_loss_and_ewc_match_autograd(loss):
    """e3gnn_loss_efs / e3gnn_ewc_flat (the explicit step's loss in one launch)
    against autograd through the reference's loss classes (train.py
    LossDefinition: loss.py:8-252) on the same predictions: the loss value and
    the cotangents of E, F, S, with NaN labels (dropped from the means) and the
    flat EWC gradient."""
    from sevennet_finetuning_amd.nn import SevenNetTrainable
    m = SevenNetTrainable(device=DEV)
    fisher = {n: torch.rand_like(p) * 1e-3 for n, p in m.named_parameters()}
    opt = {n: p.detach() + 1e-2 * torch.randn_like(p) for n, p in m.named_parameters()}
    cfg = {'loss': loss, 'loss_param': {'delta': 0.05} if loss == 'huber' else {},
           'force_loss_weight': 0.7, 'stress_loss_weight': 0.05, 'is_train_stress': True,
           'optimizer': 'sgd', 'optim_param': {'lr': 0.0}, 'scheduler': 'exponentiallr',
           'scheduler_param': {'gamma': 1.0},
           'continue': {'fisher_information': fisher, 'opt_params': opt, 'ewc_lambda': 1e3},
           'device': DEV}
    tr = train.Trainer(m, cfg)
    assert tr._fused_loss is not None
    b = train.collate(_batch([21, 22, 23]), device=DEV, dtype=torch.float32)
    b[KEY.ENERGY][1] = float('nan')
    b[KEY.FORCE][5, 1] = float('nan')
    b[KEY.STRESS][0, 2] = float('nan')
    out = tr.explicit.forward(b)
    # reference: autograd through the loss classes
    ref = tr.total_loss(out)
    m.zero_grad()
    ref.backward()
    leaves = [out[k] for k in (KEY.PRED_TOTAL_ENERGY, KEY.PRED_FORCE, KEY.PRED_STRESS)]
    rc = [x.grad.clone() for x in leaves]
    g_ref = m.flat_grad.clone()          # the EWC term's gradient (the data terms' go through cE, cF, cS)
    # fused
    m.zero_grad()
    calls = {}
    orig = tr.explicit.backward
    tr.explicit.backward = lambda cE, cF, cS: calls.update(c=(cE, cF, cS))
    try:
        got = tr._fused_loss_backward(out, b)
    finally:
        tr.explicit.backward = orig
    assert abs(float(got) - float(ref)) <= 2e-6 * abs(float(ref))
    for a, r in zip(calls['c'], rc):
        assert float((a - r).abs().max()) <= 1e-6 * float(r.abs().max()) + 1e-12
    assert float(calls['c'][0][1]) == 0.0 and float(calls['c'][1][5, 1]) == 0.0
    assert float((m.flat_grad - g_ref).abs().max()) <= 1e-6 * float(g_ref.abs().max())


def test_irreps_layout_linears_match_dense():
    """The fine-tune step's linears in the irreps layout (one grouped-GEMM
    problem per l-block, e3gnn_gemm_layouts: rows (node, m), the m = 0
    diagonal of the dense matrix; weight gradients over K = (m, node)
    segments) against the dense float64 products: C = A D, C = A D^T with two
    operand pairs, and the gradient's diagonal sums."""
    from sevennet_finetuning_amd.nn import SevenNetTrainable
    from sevennet_finetuning_amd.train_explicit import ExplicitStep
    torch.manual_seed(0)
    m = SevenNetTrainable(device=DEV)
    st = ExplicitStep(m)
    D = st.bank.build()
    st.S = {'D': D}
    rows = 77                                            # not a multiple of any tile
    for t in range(len(m.blocks)):
        for key, key2 in ((f'si1{t}', None), (f'sc{t}', f'si2{t}')):
            din, dout = D[key].shape
            A = torch.randn(rows, din, device=DEV)
            A2 = torch.randn(rows, D[key2].shape[0], device=DEV) if key2 else None
            C = torch.empty(rows, dout, device=DEV)
            st._lin(C, A, key, A2=A2, key2=key2)
            ref = A.double() @ D[key].double()
            if key2:
                ref += A2.double() @ D[key2].double()
            assert (C.double() - ref).abs().max() <= 2e-5 * (1 + ref.abs().max()), (key, key2)
            # transposed: C = A D^T (+ A2 D2^T) into the input space
            if key2 is None or D[key2].shape[1] == dout:
                At = torch.randn(rows, dout, device=DEV)
                Ct = torch.empty(rows, din, device=DEV)
                if key == f'si1{t}':
                    st._lin(Ct, At, key, trans=True)
                    reft = At.double() @ D[key].double().t()
                    assert (Ct.double() - reft).abs().max() <= 2e-5 * (1 + reft.abs().max()), key
        for key in (f'si1{t}', f'sc{t}', f'si2{t}'):
            din, dout = D[key].shape
            X, Y = torch.randn(rows, din, device=DEV), torch.randn(rows, dout, device=DEV)
            G = torch.zeros(din, dout, device=DEV)
            st._lin_grad(G, X, Y, key)
            st.gm.flush()
            full = X.double().t() @ Y.double()
            for (l, d, in_lo, mi, out_lo, mo) in st._lblocks(key):
                u = torch.arange(mi, device=DEV)[:, None]
                v = torch.arange(mo, device=DEV)[None, :]
                want = sum(full[in_lo + u * d + k, out_lo + v * d + k] for k in range(d))
                got = G[in_lo + u * d, out_lo + v * d].double()
                assert (got - want).abs().max() <= 2e-5 * (1 + want.abs().max()), (key, l)
