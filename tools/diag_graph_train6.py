"""Diagnostic: what, run eagerly between two replays of the graphed
rehearsal step, breaks the replay (reference: the same steps with nothing in
between)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
from sevennet_finetuning_amd import train  # noqa: E402
from sevennet_finetuning_amd.nn import SevenNetTrainable  # noqa: E402
import test_gpu_train as T  # noqa: E402

dev = torch.device('cuda', 0)


def make(graph):
    m = SevenNetTrainable(device=dev)
    cfg = {'loss': 'huber', 'loss_param': {'delta': 0.01}, 'force_loss_weight': 1.0,
           'stress_loss_weight': 0.01, 'is_train_stress': True, 'optimizer': 'adam',
           'optim_param': {'lr': 1e-5}, 'scheduler': 'exponentiallr',
           'scheduler_param': {'gamma': 0.99}, 'device': dev, 'hip_graph': graph}
    tr = train.Trainer(m, cfg)
    m.train(True)
    return m, tr


def coll(seeds):
    return train.collate(T._batch(seeds), device=dev, dtype=torch.float32)


pairs = [(coll([1, 2]), coll([3, 4])), (coll([5, 6]), coll([7, 8]))]
other = SevenNetTrainable(device=dev)
other.train(True)


def between(kind):
    if kind == 'mm':
        a = torch.randn(4096, 4096, device=dev)
        (a @ a).sum().item()
    elif kind == 'mm_small':
        a = torch.randn(12096, 64, device=dev)
        (a @ torch.randn(64, 960, device=dev)).sum().item()
    elif kind == 'fwd':
        out = other(pairs[0][0])
        out['inferred_total_energy'].sum().item()
    elif kind == 'eager_step':
        ref_tr.rehearsal_step(*pairs[1])
        torch.cuda.synchronize()
    elif kind == 'alloc':
        x = [torch.randn(1 << 20, device=dev) for _ in range(64)]
        del x


import gc
ref_m, ref_tr = make(False)
KINDS = sys.argv[1:] or ['none', 'fwd', 'eager_step']
for kind in KINDS:
    gc.collect()
    torch.cuda.synchronize()
    m, tr = make(True)
    res = []
    for i in range(4):
        res.append([round(float(x), 6) for x in tr.rehearsal_step(*pairs[i % 2])])
        between(kind)
    print(kind, res, flush=True)
