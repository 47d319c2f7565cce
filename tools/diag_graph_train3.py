"""Diagnostic: repeated replays of the graphed rehearsal step (same batch
pair), for several loss configurations, against the eager step."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench_train as bt  # noqa: E402
from sevennet_finetuning_amd import train  # noqa: E402
from sevennet_finetuning_amd.nn import SevenNetTrainable  # noqa: E402

dev = torch.device('cuda', 0)


def make(hip_graph, variant):
    m = SevenNetTrainable(device=dev)
    cfg = {'loss': 'huber', 'loss_param': {'delta': 0.01}, 'force_loss_weight': 1.0,
           'stress_loss_weight': 0.01, 'is_train_stress': True, 'optimizer': 'adam',
           'optim_param': {'lr': 1e-5}, 'scheduler': 'exponentiallr',
           'scheduler_param': {'gamma': 0.99}, 'device': dev, 'hip_graph': hip_graph}
    if variant == 'ewc':
        fisher = {n: torch.full_like(p, 1e-3) for n, p in m.named_parameters()}
        opt = {n: p.detach().clone() for n, p in m.named_parameters()}
        cfg['continue'] = {'fisher_information': fisher, 'opt_params': opt, 'ewc_lambda': 1e5}
    if variant == 'energy':
        cfg['force_loss_weight'] = 0.0
        cfg['is_train_stress'] = False
    tr = train.Trainer(m, cfg)
    m.train(True)
    return m, tr


for variant in ['plain', 'energy', 'ewc']:
    ma, ta = make(False, variant)
    mb, tb = make(True, variant)
    batches = bt.make_batches(0, 2, 8, ma.chemical_symbols)
    db = [train.collate(b, device=dev, dtype=torch.float32) for b in batches]
    print(f'{variant}: loss terms {[type(l).__name__ for l, _ in tb.loss_functions]}', flush=True)
    for i in range(3):
        lb = tb.rehearsal_step(db[0], db[1])
        la = ta.rehearsal_step(db[0], db[1])
        torch.cuda.synchronize()
        print(f'  step {i}: eager {float(la[0]):.6g} {float(la[1]):.6g} graphed '
              f'{float(lb[0]):.6g} {float(lb[1]):.6g} max|dtheta| '
              f'{float((ma.flat - mb.flat).abs().max()):.3g}', flush=True)
