"""Fine-tune step host logic (nn.py / train.py / conv_ops.py) on the CPU.

The trainable model runs here with the CPU test double of the convolution op
(_conv_cpu.py: the oracle's uvu tensor product, float64), so these tests pin
everything AROUND the HIP kernels against the oracle and the reference's
files: energies/forces/stress of the training-mode model, PyG-style batching,
parameter names (fisher_sevenn.pt / opt_params_sevenn.pt), the loss
definitions, the warmup-cosine schedule (golden LR column of the reference's
fine-tuning log), the second-order derivative chain of conv_ops, and the
data-parallel gradient averaging (gloo, world_size 2).  The HIP kernels are
compared with the same double in tests/test_gpu_train.py.
"""
import json
import math
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from _conv_cpu import CpuConvBackend
from _systems import GOLD, load_manifest_symbols, oracle_eval, system
from sevennet_finetuning_amd import _keys as KEY
from sevennet_finetuning_amd import conv_ops, train
from sevennet_finetuning_amd.nn import SevenNetTrainable
from sevennet_finetuning_amd.structures import diamond_primitive, mixed_symbols

SYMS = load_manifest_symbols()
REF_FT = '/root/reference/example_inputs/fine_tuning/estimate_Fisher'


@pytest.fixture(scope='module')
def model64():
    return SevenNetTrainable(device='cpu', conv_backend=CpuConvBackend(), dtype=torch.float64)


def graph_of(name):
    pos, cell, types = system(name, SYMS)
    return train.labeled_graph(pos, cell, types, 5.0), (pos, cell, types)


def ft_structure(seed, cells=(3, 3, 3)):
    """SURVEY 8d config 5 cell: 54-atom primitive diamond, mixed species."""
    pos, cell = diamond_primitive(cells, sigma=0.05, seed=seed)
    types = np.array([SYMS.index(s) for s in mixed_symbols(len(pos), seed=seed + 1)])
    return pos, cell, types


def test_diamond_primitive_geometry():
    pos, cell = diamond_primitive((3, 3, 3), sigma=0.0)
    assert pos.shape == (54, 3)
    assert abs(abs(np.linalg.det(cell)) - 54 / 8 * 5.43 ** 3) < 1e-9
    d = np.linalg.norm(pos[1] - pos[0])
    assert abs(d - 5.43 * math.sqrt(3) / 4) < 1e-12   # Si-Si bond


@pytest.mark.parametrize('name', ['si_rng0_2x2x1', 'hfo2_resdat'])
def test_trainable_matches_oracle(model64, name):
    g, (pos, cell, types) = graph_of(name)
    ref = oracle_eval(pos, cell, types)
    model64.train(False)
    out = model64(train.collate([g], dtype=torch.float64))
    assert abs(float(out[KEY.PRED_TOTAL_ENERGY][0]) - ref['energy']) < 1e-9 * abs(ref['energy'])
    assert np.abs(out[KEY.PRED_FORCE].detach().numpy() - ref['forces']).max() < 1e-10
    assert np.abs(out[KEY.PRED_STRESS].detach().numpy()[0] - ref['stress']).max() < 2e-9
    assert np.allclose(out[KEY.ATOMIC_ENERGY].detach().numpy()[:, 0], ref['atomic_energy'],
                       atol=1e-10)


def test_batched_graphs_equal_single(model64):
    """PyG collate: per-graph energies/stress and per-atom forces of a batch of
    three graphs (different sizes and species) equal the single-graph runs."""
    model64.train(False)
    gs = [train.labeled_graph(*ft_structure(s), 5.0) for s in (0, 1)]
    gs.append(graph_of('si_rng0_2x2x1')[0])
    batch = train.collate(gs, dtype=torch.float64)
    assert batch[KEY.EDGE_IDX].shape[1] == sum(g[KEY.EDGE_IDX].shape[1] for g in gs)
    assert batch[KEY.BATCH].tolist() == sum(([b] * int(g[KEY.NUM_ATOMS]) for b, g in
                                             enumerate(gs)), [])
    out = model64(batch)
    off = 0
    for b, g in enumerate(gs):
        one = model64(train.collate([g], dtype=torch.float64))
        n = int(g[KEY.NUM_ATOMS])
        assert abs(float(out[KEY.PRED_TOTAL_ENERGY][b] - one[KEY.PRED_TOTAL_ENERGY][0])) < 1e-9
        assert torch.allclose(out[KEY.PRED_FORCE][off:off + n], one[KEY.PRED_FORCE], atol=1e-11)
        assert torch.allclose(out[KEY.PRED_STRESS][b], one[KEY.PRED_STRESS][0], atol=1e-13)
        off += n


def test_unsorted_edges_are_accepted(model64):
    """A collated batch with edges not sorted by centre gives the same result
    (the model sorts a copy; the caller's edge order is kept for the forces)."""
    model64.train(False)
    g = graph_of('si_rng0_2x2x1')[0]
    perm = torch.from_numpy(np.random.default_rng(5).permutation(g[KEY.EDGE_IDX].shape[1]))
    h = dict(g)
    h[KEY.EDGE_IDX] = g[KEY.EDGE_IDX][:, perm]
    h[KEY.EDGE_VEC] = g[KEY.EDGE_VEC][perm]
    a = model64(train.collate([g], dtype=torch.float64))
    b = model64(train.collate([h], dtype=torch.float64))
    assert abs(float(a[KEY.PRED_TOTAL_ENERGY] - b[KEY.PRED_TOTAL_ENERGY])) < 1e-9
    assert torch.allclose(a[KEY.PRED_FORCE], b[KEY.PRED_FORCE], atol=1e-11)


def test_parameters_live_in_one_buffer(model64):
    n = sum(p.numel() for p in model64.parameters())
    assert n == 842623 == model64.flat.numel()   # "Total number of weight" (log.sevenn)
    for p in model64.parameters():
        assert model64.flat.data_ptr() <= p.data_ptr() < model64.flat.data_ptr() + 8 * n
    assert model64.grads_in_flat_buffer()


@pytest.mark.skipif(not os.path.isdir(REF_FT), reason='reference fixtures absent')
def test_parameter_names_match_reference_fisher(model64):
    fisher = torch.load(os.path.join(REF_FT, 'fisher_sevenn.pt'), weights_only=True,
                        map_location='cpu')
    opt = torch.load(os.path.join(REF_FT, 'opt_params_sevenn.pt'), weights_only=True,
                     map_location='cpu')
    names = dict(model64.named_parameters())
    assert set(fisher) == set(opt) == set(names)
    for k, p in names.items():
        assert tuple(fisher[k].shape) == tuple(p.shape) == tuple(opt[k].shape)
        # the converted weights are the reference's optimum bit for bit
        assert torch.equal(p.detach().to(torch.float32), opt[k])
    ewc = train.EWCLoss({k: v.double() for k, v in fisher.items()},
                        {k: v.double() for k, v in opt.items()})
    assert float(ewc.get_loss({}, model64)) == 0.0


def test_ewc_loss_value_and_gradient():
    torch.manual_seed(0)
    lin = torch.nn.Linear(3, 2)
    fisher = {k: torch.rand_like(v) for k, v in lin.named_parameters()}
    opt = {k: v.detach() + 0.1 * torch.randn_like(v) for k, v in lin.named_parameters()}
    opt.pop('bias')   # parameters missing from either dict are skipped (loss.py:262)
    loss = train.EWCLoss(fisher, opt).get_loss({}, lin)
    want = torch.sum(fisher['weight'] * (lin.weight - opt['weight']) ** 2)
    assert torch.allclose(loss, want)
    loss.sum().backward()
    assert torch.allclose(lin.weight.grad, 2 * fisher['weight'] * (lin.weight - opt['weight']))
    assert lin.bias.grad is None
    with pytest.raises(ValueError):
        train.EWCLoss(fisher, opt).get_loss({}, None)


def test_loss_definitions_from_config():
    cfg = {'loss': 'huber', 'loss_param': {'delta': 0.01}, 'force_loss_weight': 1.0,
           'stress_loss_weight': 0.01, 'is_train_stress': True,
           'continue': {'fisher_information': False, 'opt_params': False}}
    fns = train.get_loss_functions_from_config(cfg)
    assert [type(f).__name__ for f, _ in fns] == ['PerAtomEnergyLoss', 'ForceLoss', 'StressLoss']
    assert [w for _, w in fns] == [1.0, 1.0, 0.01]
    rng = np.random.default_rng(0)
    out = {KEY.PRED_TOTAL_ENERGY: torch.tensor([-10.0, -20.0]),
           KEY.ENERGY: torch.tensor([-10.5, float('nan')]),
           KEY.NUM_ATOMS: torch.tensor([2, 4]),
           KEY.PRED_FORCE: torch.tensor(rng.normal(size=(6, 3))),
           KEY.FORCE: torch.tensor(rng.normal(size=(6, 3))),
           KEY.PRED_STRESS: torch.tensor(rng.normal(size=(2, 6)) * 1e-3),
           KEY.STRESS: torch.tensor(rng.normal(size=(2, 6)) * 1e-3)}
    hub = torch.nn.HuberLoss(delta=0.01)
    e = fns[0][0].get_loss(out)
    assert torch.allclose(e, hub(torch.tensor([-5.0]), torch.tensor([-5.25])))  # NaN dropped
    f = fns[1][0].get_loss(out)
    assert torch.allclose(f, hub(out[KEY.PRED_FORCE].reshape(-1), out[KEY.FORCE].reshape(-1)))
    s = fns[2][0].get_loss(out)
    kb = train.StressLoss.TO_KB
    assert torch.allclose(s, hub(out[KEY.PRED_STRESS].reshape(-1) * kb,
                                 out[KEY.STRESS].reshape(-1) * kb))
    out[KEY.ENERGY][0] = float('nan')
    assert float(fns[0][0].get_loss(out)) == 0.0
    cfg['load_dataset_with_weights'] = True
    fns = train.get_loss_functions_from_config(cfg)
    out[train.DATA_WEIGHT] = {KEY.FORCE: torch.tensor([1.0, 3.0])}
    out[KEY.BATCH] = torch.tensor([0, 0, 1, 1, 1, 1])
    f = fns[1][0].get_loss(out)
    w = torch.tensor([1.0, 3.0])[out[KEY.BATCH]].repeat_interleave(3)
    raw = torch.nn.HuberLoss(delta=0.01, reduction='none')(
        out[KEY.PRED_FORCE].reshape(-1), out[KEY.FORCE].reshape(-1))
    assert torch.allclose(f, torch.mean(raw * w))


def test_lr_schedule_matches_reference_log():
    """Warmup-cosine LR of the reference's FT_w_reEWC run (Epoch 601..610 lr
    column of log.sevenn, fresh scheduler after reset_scheduler)."""
    gold = json.load(open(os.path.join(GOLD, 'ft_lr_schedule.json')))
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.Adam([p], **gold['optim_param'])
    sch = train.scheduler_dict[gold['scheduler']](opt, **gold['scheduler_param'])
    got = []
    for _ in gold['lr']:
        got.append(round(opt.param_groups[0]['lr'], gold['printed_decimals']))
        sch.step()
    assert got == gold['lr']


def test_warmup_cosine_full_cycle():
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.SGD([p], lr=0.0)
    sch = train.CosineAnnealingWarmupRestarts(opt, first_cycle_steps=20, max_lr=1.0, min_lr=0.1,
                                              warmup_steps=5, gamma=0.5)
    lrs = []
    for _ in range(45):
        lrs.append(opt.param_groups[0]['lr'])
        sch.step()
    assert lrs[0] == pytest.approx(0.1) and lrs[5] == pytest.approx(1.0)
    assert lrs[5 + 15 // 2] < 1.0 and lrs[19] > 0.1
    assert lrs[20] == pytest.approx(0.1) and lrs[25] == pytest.approx(0.5)  # gamma per cycle


def _small_conv_problem(kind, n=7, seed=0, dtype=torch.float64):
    rng = np.random.default_rng(seed)
    be = CpuConvBackend()
    dx, dw, dm = be.dims[kind]
    e = 23
    center = np.sort(rng.integers(0, n, e))
    nbr = rng.integers(0, n, e)
    g = conv_ops.ConvGraph(n, torch.tensor(center), torch.tensor(nbr), be)
    h = torch.tensor(rng.normal(size=(n, dx)), dtype=dtype, requires_grad=True)
    Y = torch.tensor(rng.normal(size=(e, 9)), dtype=dtype, requires_grad=True)
    w = torch.tensor(rng.normal(size=(e, dw)), dtype=dtype, requires_grad=True)
    return g, h, Y, w


@pytest.mark.parametrize('kind', [0, 1, 2])
def test_conv_op_double_backward_chain(kind):
    """conv_ops' custom second-order rules (trilinearity) equal plain autograd
    through the same forward -- the rules the HIP path relies on."""
    g, h, Y, w = _small_conv_problem(kind)
    be = g.backend
    rng = np.random.default_rng(1)
    gout = torch.tensor(rng.normal(size=(g.n_nodes, be.dims[kind][2])))
    probe = [torch.tensor(rng.normal(size=t.shape)) for t in (h, Y, w)]

    def second(fwd):
        agg = fwd(h, Y, w)
        d = torch.autograd.grad((agg * gout).sum(), [h, Y, w], create_graph=True)
        s = sum((di * pi).sum() for di, pi in zip(d, probe))
        return torch.autograd.grad(s, [h, Y, w])

    want = second(lambda a, b, c: be.forward(kind, g, a, b, c))
    got = second(lambda a, b, c: conv_ops.conv(a, b, c, kind, g))
    for x, y in zip(got, want):
        assert torch.allclose(x, y, rtol=1e-10, atol=1e-10)


def test_force_loss_parameter_gradient_finite_difference(model64):
    """d(force loss)/d(theta) through create_graph (force_output.py:168) against
    a central finite difference on a few parameters, float64."""
    model64.train(True)
    g = train.labeled_graph(*ft_structure(3, cells=(2, 2, 1)), 5.0)
    batch = train.collate([g], dtype=torch.float64)
    rng = np.random.default_rng(4)
    target = torch.tensor(rng.normal(size=(int(g[KEY.NUM_ATOMS]), 3)))

    def loss_fn():
        out = model64(batch)
        return ((out[KEY.PRED_FORCE] - target) ** 2).sum() + out[KEY.PRED_TOTAL_ENERGY].sum()

    model64.zero_grad()
    loss_fn().backward()
    grad = model64.flat_grad.clone()
    picks = {'1_convolution.weight_nn.layer2.weight': 17,
             '2_self_interaction_1.linear.weight': 5,
             'edge_embedding.basis_function.coeffs': 3,
             '0_convolution.weight_nn.layer0.weight': 40,
             'reduce_hidden_to_energy.linear.weight': 7}
    eps = 1e-6
    with torch.no_grad():
        for name, k in picks.items():
            off = model64.slices[name][0] + k
            old = float(model64.flat[off])
            model64.flat[off] = old + eps
            with torch.enable_grad():
                lp = float(loss_fn())
            model64.flat[off] = old - eps
            with torch.enable_grad():
                lm = float(loss_fn())
            model64.flat[off] = old
            fd = (lp - lm) / (2 * eps)
            assert abs(fd - float(grad[off])) <= 1e-6 * max(1.0, abs(fd)), name
    model64.train(False)


def _sgd_config(ddp):
    return {'loss': 'mse', 'force_loss_weight': 0.1, 'stress_loss_weight': 1e-4,
            'is_train_stress': True, 'optimizer': 'sgd', 'optim_param': {'lr': 1e-3},
            'scheduler': 'exponentiallr', 'scheduler_param': {'gamma': 0.99},
            'continue': {'fisher_information': False, 'opt_params': False}, 'is_ddp': ddp}


def _ddp_batches():
    gs = []
    for s in range(4):
        pos, cell, types = ft_structure(10 + s, cells=(2, 2, 1))
        rng = np.random.default_rng(100 + s)
        gs.append(train.labeled_graph(pos, cell, types, 5.0, energy=-3.0 * len(pos),
                                      force=rng.normal(0, 0.3, (len(pos), 3)),
                                      stress=rng.normal(0, 1e-3, 6)))
    return gs


def _ddp_worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    torch.set_num_threads(2)
    model = SevenNetTrainable(device='cpu', conv_backend=CpuConvBackend(), dtype=torch.float64)
    tr = train.Trainer(model, _sgd_config(True))
    gs = _ddp_batches()
    model.train(True)
    b = train.collate(gs[2 * rank:2 * rank + 2], dtype=torch.float64)
    m = train.collate(gs[(2 * rank + 3) % 4:(2 * rank + 3) % 4 + 1], dtype=torch.float64)
    tr.rehearsal_step(b, m)
    if rank == 0:
        torch.save(model.flat.detach().clone(), out)
    else:
        flat0 = model.flat.detach().clone()
        dist.barrier()
        return_code = 0 if torch.equal(flat0, torch.load(out, weights_only=True)) else 1
        assert return_code == 0, 'ranks diverged'
        dist.destroy_process_group()
        return
    dist.barrier()
    dist.destroy_process_group()


def test_data_parallel_rehearsal_step_gloo(tmp_path):
    """world_size 2: after one rehearsal step (new batch + memory batch, SGD)
    both ranks hold identical parameters, equal to a single process applying
    the rank-averaged gradients (DDP semantics, trainer.py:174-206)."""
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    out = str(tmp_path / 'flat.pt')
    mp.spawn(_ddp_worker, args=(2, port, out), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)

    model = SevenNetTrainable(device='cpu', conv_backend=CpuConvBackend(), dtype=torch.float64)
    model.train(True)
    tr = train.Trainer(model, _sgd_config(False))
    gs = _ddp_batches()
    lr = 1e-3

    def grads(batch_sets):
        acc = []
        for bs in batch_sets:
            model.zero_grad()
            tr.total_loss(model(train.collate(bs, dtype=torch.float64))).backward()
            acc.append(model.flat_grad.clone())
        return sum(acc) / len(acc)

    with torch.no_grad():
        theta = model.flat.clone()
    g1 = grads([gs[0:2], gs[2:4]])
    mask = torch.zeros_like(g1)
    for name, p in model.named_parameters():
        if p.requires_grad:
            off, n, _ = model.slices[name]
            mask[off:off + n] = 1
    with torch.no_grad():
        model.flat.copy_(theta - lr * g1 * mask)
    g2 = grads([gs[3:4], gs[1:2]])
    with torch.no_grad():
        want = theta - lr * g1 * mask - lr * (g1 + g2) * mask
    assert torch.allclose(got, want, rtol=1e-12, atol=1e-14)


def test_flat_ewc_equals_per_tensor_loop(model64):
    """The fused flat-buffer EWC (one pass over model.flat, gradient straight
    into flat_grad) gives the per-parameter loop's value and gradients,
    skipping parameters missing from the dicts and frozen ones."""
    torch.manual_seed(3)
    names = [n for n, _ in model64.named_parameters()]
    fisher = {n: torch.rand_like(p, dtype=torch.float64) for n, p in model64.named_parameters()
              if n != names[2]}
    opt = {n: (p.detach() + 1e-2 * torch.randn_like(p)) for n, p in model64.named_parameters()}
    ewc = train.EWCLoss(fisher, opt)
    model64.zero_grad()
    fused = ewc.get_loss({}, model64)
    fused.backward()
    g_fused = model64.flat_grad.clone()
    model64.zero_grad()
    want = torch.zeros(1, dtype=torch.float64)
    for n, p in model64.named_parameters():
        if n in fisher:
            want = want + torch.sum(fisher[n] * (p - opt[n]) ** 2)
    want.backward()
    g_loop = model64.flat_grad.clone()
    model64.zero_grad()
    assert fused.shape == (1,)
    assert torch.allclose(fused, want, rtol=1e-13)
    assert torch.allclose(g_fused, g_loop, rtol=1e-12, atol=1e-15)
    frozen = model64.slices['rescale_atomic_energy.scale']
    assert float(g_loop[frozen[0]:frozen[0] + frozen[1]].abs().max()) == 0.0
