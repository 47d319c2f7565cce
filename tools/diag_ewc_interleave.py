"""Diagnostic (round 3): the graphed-EWC interleaving report of DESIGN.md.
Runs an eager and a graphed rehearsal trainer alone and interleaved step by
step, EWC on/off per trainer, and prints the losses of each run so the one
that deviates can be told apart."""
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
STEPS = 4


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


def fmt(x):
    return [round(float(v), 7) for v in x]


def alone(graph, ewc):
    m, tr = make(graph, ewc)
    out = [fmt(tr.rehearsal_step(*pairs[i % 2])) for i in range(STEPS)]
    return out, m.flat.detach().clone()


def interleaved(ewc_e, ewc_g, sync=False):
    me, te = make(False, ewc_e)
    mg, tg = make(True, ewc_g)
    le, lg = [], []
    for i in range(STEPS):
        le.append(fmt(te.rehearsal_step(*pairs[i % 2])))
        if sync:
            torch.cuda.synchronize()
        lg.append(fmt(tg.rehearsal_step(*pairs[i % 2])))
        if sync:
            torch.cuda.synchronize()
    return le, lg, me.flat.detach().clone(), mg.flat.detach().clone()


for ewc in (True, False):
    E, fe = alone(False, ewc)
    G, fg = alone(True, ewc)
    print(f'ewc={ewc} eager alone   {E}', flush=True)
    print(f'ewc={ewc} graphed alone {G}  |dflat| {float((fe - fg).abs().max()):.3g}', flush=True)
    for ee, eg, sync in ((ewc, ewc, False), (ewc, ewc, True), (False, ewc, False),
                         (ewc, False, False)):
        le, lg, f1, f2 = interleaved(ee, eg, sync)
        print(f'  interleaved ewc_e={ee} ewc_g={eg} sync={sync}: eager {le}', flush=True)
        print(f'  {"":44s}graphed {lg}  |de-fe| {float((f1 - (fe if ee == ewc else f1)).abs().max()):.3g}'
              f' |dg-fg| {float((f2 - (fg if eg == ewc else f2)).abs().max()):.3g}', flush=True)
