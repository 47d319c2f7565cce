"""Diagnostic: state of the graphed rehearsal step's static inputs between
replays (which static tensor, if any, changes under a replay)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench_train as bt  # noqa: E402
from sevennet_finetuning_amd import train  # noqa: E402
from sevennet_finetuning_amd.nn import SevenNetTrainable  # noqa: E402

dev = torch.device('cuda', 0)
m = SevenNetTrainable(device=dev)
cfg = {'loss': 'huber', 'loss_param': {'delta': 0.01}, 'force_loss_weight': 1.0,
       'stress_loss_weight': 0.01, 'is_train_stress': True, 'optimizer': 'adam',
       'optim_param': {'lr': 1e-5}, 'scheduler': 'exponentiallr',
       'scheduler_param': {'gamma': 0.99}, 'device': dev, 'hip_graph': True}
tr = train.Trainer(m, cfg)
m.train(True)
batches = bt.make_batches(0, 2, 8, m.chemical_symbols)
db = [train.collate(b, device=dev, dtype=torch.float32) for b in batches]
print('step0', [float(x) for x in tr.rehearsal_step(db[0], db[1])], flush=True)
ent = next(iter(tr._graphed.cache.values()))
for i in range(8):
    ent['g'].replay()
    torch.cuda.synchronize()
    print(f'  pure replay {i}: {float(ent["out"][0]):.6g} {float(ent["out"][1]):.6g}', flush=True)
snap = {w: {k: v.clone() for k, v in ent[w].items()} for w in ('b', 'm')}
aux = [{k: v.clone() for k, v in g.aux.items()} for g in ent['graphs']]
ent['g'].replay()
torch.cuda.synchronize()
print('bare replay', float(ent['out'][0]), float(ent['out'][1]), flush=True)
for w in ('b', 'm'):
    for k, v in ent[w].items():
        if not torch.equal(v, snap[w][k]):
            print(f'  static {w}[{k}] changed by the replay: max diff '
                  f'{float((v.double() - snap[w][k].double()).abs().max()):.3g}', flush=True)
for i, g in enumerate(ent['graphs']):
    for k, v in g.aux.items():
        if not torch.equal(v, aux[i][k]):
            print(f'  graph {i} aux[{k}] changed by the replay', flush=True)
G = tr._graphed
bs, ms = G._centre_sorted(db[0]), G._centre_sorted(db[1])
for w, src in (('b', bs), ('m', ms)):
    for k, v in src.items():
        if torch.is_tensor(v) and not torch.equal(v.to(ent[w][k].dtype), ent[w][k]):
            d = (v.double() - ent[w][k].double()).abs()
            print(f'  static {w}[{k}] differs from the batch: max diff {float(d.max()):.3g} at '
                  f'{int(d.argmax())}, batch {float(v.reshape(-1)[int(d.argmax())]):.6g} static '
                  f'{float(ent[w][k].reshape(-1)[int(d.argmax())]):.6g}', flush=True)
for dst, src in ((ent['b'], bs), (ent['m'], ms)):
    for k, v in src.items():
        if torch.is_tensor(v):
            if v.device != dst[k].device or v.dtype != dst[k].dtype or v.shape != dst[k].shape:
                print(f'  key {k}: src {v.device} {v.dtype} {tuple(v.shape)} dst {dst[k].device} '
                      f'{dst[k].dtype} {tuple(dst[k].shape)}', flush=True)
            dst[k].copy_(v)
torch.cuda.synchronize()
ent['g'].replay()
torch.cuda.synchronize()
print('after copy only', float(ent['out'][0]), float(ent['out'][1]), flush=True)
for gr, b in zip(ent['graphs'], (ent['b'], ent['m'])):
    gr.rebuild(b['edge_index'][0], b['edge_index'][1])
torch.cuda.synchronize()
for i, g in enumerate(ent['graphs']):
    for k, v in g.aux.items():
        if not torch.equal(v, aux[i][k]):
            print(f'  graph {i} aux[{k}] changed by the rebuild', flush=True)
ent['g'].replay()
torch.cuda.synchronize()
print('after rebuild', float(ent['out'][0]), float(ent['out'][1]), flush=True)
print('step1', [float(x) for x in tr.rehearsal_step(db[0], db[1])], flush=True)
