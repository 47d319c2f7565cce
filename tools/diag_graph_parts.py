"""Diagnostic: which part of the fine-tune step is not replay-idempotent under
HIP-graph capture.  Each stage is captured after a side-stream warm-up and
replayed three times on the same inputs; the outputs should repeat."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench_train as bt  # noqa: E402
from sevennet_finetuning_amd import _keys as KEY  # noqa: E402
from sevennet_finetuning_amd import conv_ops, train  # noqa: E402
from sevennet_finetuning_amd.nn import SevenNetTrainable  # noqa: E402

dev = torch.device('cuda', 0)
m = SevenNetTrainable(device=dev)
m.train(True)
batches = bt.make_batches(0, 2, 8, m.chemical_symbols)
b = train.collate(batches[0], device=dev, dtype=torch.float32)
ei = b[KEY.EDGE_IDX]
graph = conv_ops.ConvGraph(int(b[KEY.NODE_FEATURE].shape[0]), ei[0], ei[1], m.conv_backend)


def stage_fwd():
    out = m(b, graph=graph)
    return out[KEY.PRED_TOTAL_ENERGY].sum().detach() + 0.0


def stage_force():
    out = m(b, graph=graph)
    return out[KEY.PRED_FORCE].detach().abs().sum()


def stage_backward():
    m.zero_grad()
    out = m(b, graph=graph)
    loss = (out[KEY.PRED_FORCE] ** 2).sum() + out[KEY.PRED_TOTAL_ENERGY].sum()
    loss.backward()
    return m.flat_grad.abs().sum()


def stage_stress():
    out = m(b, graph=graph)
    return out[KEY.PRED_STRESS].detach().abs().sum()


def stage_stress_backward():
    m.zero_grad()
    out = m(b, graph=graph)
    loss = (out[KEY.PRED_STRESS] ** 2).sum() * 1e4
    loss.backward()
    return m.flat_grad.abs().sum()


def stage_stress_loss():
    m.zero_grad()
    out = m(b, graph=graph)
    sl = train.StressLoss(criterion=torch.nn.HuberLoss(delta=0.01))
    sl.static = True
    loss = sl.get_loss(out)
    loss.backward()
    return m.flat_grad.abs().sum() + 0 * loss.detach().sum()


b2 = train.collate(batches[1], device=dev, dtype=torch.float32)
ei2 = b2[KEY.EDGE_IDX]
graph2 = conv_ops.ConvGraph(int(b2[KEY.NODE_FEATURE].shape[0]), ei2[0], ei2[1], m.conv_backend)
lossdefs = train.get_loss_functions_from_config(
    {'loss': 'huber', 'loss_param': {'delta': 0.01}, 'force_loss_weight': 1.0,
     'stress_loss_weight': 0.01, 'is_train_stress': True})
for ld, _ in lossdefs:
    ld.static = True


def total(out):
    t = torch.zeros(1, device=dev)
    for ld, w in lossdefs:
        t = t + ld.get_loss(out, m) * w
    return t


def stage_two_pass():
    m.zero_grad()
    l1 = total(m(b, graph=graph))
    l1.backward()
    l2 = total(m(b2, graph=graph2))
    l2.backward()
    return m.flat_grad.abs().sum() + 0 * (l1 + l2).detach().sum()


def stage_two_pass_step():
    m.zero_grad()
    l1 = total(m(b, graph=graph))
    l1.backward()
    with torch.no_grad():
        m.flat.sub_(1e-9 * m.flat_grad)
    l2 = total(m(b2, graph=graph2))
    l2.backward()
    with torch.no_grad():
        m.flat.add_(1e-9 * m.flat_grad)
    return m.flat_grad.abs().sum() + 0 * (l1 + l2).detach().sum()


STAGES = [('fwd', stage_fwd), ('force', stage_force), ('backward', stage_backward),
          ('stress', stage_stress), ('stress_backward', stage_stress_backward),
          ('stress_loss', stage_stress_loss), ('two_pass', stage_two_pass),
          ('two_pass_step', stage_two_pass_step)]
for name, fn in STAGES[int(sys.argv[1]) if len(sys.argv) > 1 else 6:]:
    eager = [float(fn()) for _ in range(2)]
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            fn()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = fn()
    reps = []
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        reps.append(float(out))
    print(f'{name}: eager {eager} replays {reps}', flush=True)
