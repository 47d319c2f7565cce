"""Diagnostic: the graphed rehearsal step against the eager one on bench_train's
batch sequence (4 batch pairs of different edge counts, 13 steps); prints the
losses of both and the parameter difference after every step."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench_train as bt  # noqa: E402
from sevennet_finetuning_amd import train  # noqa: E402
from sevennet_finetuning_amd.nn import SevenNetTrainable  # noqa: E402

dev = torch.device('cuda', 0)


def make(hip_graph):
    m = SevenNetTrainable(device=dev)
    fisher = {n: torch.full_like(p, 1e-3) for n, p in m.named_parameters()}
    opt = {n: p.detach().clone() for n, p in m.named_parameters()}
    cfg = {'loss': 'huber', 'loss_param': {'delta': 0.01}, 'force_loss_weight': 1.0,
           'stress_loss_weight': 0.01, 'is_train_stress': True, 'optimizer': 'adam',
           'optim_param': {'lr': 1e-5}, 'scheduler': 'exponentiallr',
           'scheduler_param': {'gamma': 0.99}, 'device': dev, 'hip_graph': hip_graph,
           'continue': {'fisher_information': fisher, 'opt_params': opt, 'ewc_lambda': 1e5}}
    tr = train.Trainer(m, cfg)
    m.train(True)
    return m, tr


ma, ta = make(False)
mb, tb = make(True)
batches = bt.make_batches(0, 8, 8, ma.chemical_symbols)
db = [train.collate(b, device=dev, dtype=torch.float32) for b in batches]
for i in range(13):
    b, m = db[(2 * i) % 8], db[(2 * i + 1) % 8]
    la = ta.rehearsal_step(b, m)
    lb = tb.rehearsal_step(b, m)
    torch.cuda.synchronize()
    d = float((ma.flat - mb.flat).abs().max())
    print(f'step {i}: eager {float(la[0]):.6g} {float(la[1]):.6g}  graphed {float(lb[0]):.6g} '
          f'{float(lb[1]):.6g}  max|dtheta| {d:.3g}', flush=True)
