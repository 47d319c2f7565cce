"""Diagnostic: tests/test_gpu_train.py's same-shape replay check with the
eager and graphed trainers interleaved step by step, with and without EWC."""
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


def make(graph, ewc):
    m = SevenNetTrainable(device=dev)
    cfg = {'loss': 'huber', 'loss_param': {'delta': 0.01}, 'force_loss_weight': 1.0,
           'stress_loss_weight': 0.01, 'is_train_stress': True, 'optimizer': 'adam',
           'optim_param': {'lr': 1e-5}, 'scheduler': 'exponentiallr',
           'scheduler_param': {'gamma': 0.99}, 'device': dev, 'hip_graph': graph}
    if ewc:
        fisher = {n: torch.full_like(p, 1e-3) for n, p in m.named_parameters()}
        opt = {n: p.detach().clone() for n, p in m.named_parameters()}
        cfg['continue'] = {'fisher_information': fisher, 'opt_params': opt, 'ewc_lambda': 1e5}
    tr = train.Trainer(m, cfg)
    m.train(True)
    return m, tr


def coll(seeds):
    return train.collate(T._batch(seeds), device=dev, dtype=torch.float32)


pairs = [(coll([1, 2]), coll([3, 4])), (coll([5, 6]), coll([7, 8]))]
for ewc in (True, False):
    me, te = make(False, ewc)
    mg, tg = make(True, ewc)
    for i in range(4):
        b, mm = pairs[i % 2]
        le = [round(float(x), 6) for x in te.rehearsal_step(b, mm)]
        lg = [round(float(x), 6) for x in tg.rehearsal_step(b, mm)]
        print(f'ewc {ewc} step {i}: eager {le} graphed {lg}', flush=True)
    del me, te, mg, tg
    import gc
    gc.collect()
    torch.cuda.synchronize()
