import sys, os, json, collections
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from torch.profiler import profile, ProfilerActivity
import bench_train as bt
from sevennet_finetuning_amd import train
from sevennet_finetuning_amd.nn import SevenNetTrainable
dev = torch.device('cuda', 0)
m = SevenNetTrainable(device=dev)
fisher = {n: torch.full_like(p, 1e-3) for n, p in m.named_parameters()}
opt = {n: p.detach().clone() for n, p in m.named_parameters()}
cfg = {'loss': 'huber', 'loss_param': {'delta': 0.01}, 'force_loss_weight': 1.0, 'stress_loss_weight': 0.01,
       'is_train_stress': True, 'optimizer': 'adam', 'optim_param': {'lr': 1e-5}, 'scheduler': 'exponentiallr',
       'scheduler_param': {'gamma': 0.99}, 'device': dev, 'hip_graph': False, 'explicit_grad': True,
       'continue': {'fisher_information': fisher, 'opt_params': opt, 'ewc_lambda': 1e5}}
tr = train.Trainer(m, cfg)
bs = bt.make_batches(0, 2, 8, m.chemical_symbols)
b = [train.collate(x, device=dev, dtype=torch.float32) for x in bs]
m.train(True)
tr.rehearsal_step(b[0], b[1]); torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    tr.rehearsal_step(b[0], b[1]); torch.cuda.synchronize()
print('explicit path:', tr.explicit is not None)
# where the element-wise launches come from (source line of the calling frame)
by_src = collections.Counter()
for e in prof.events():
    if e.name.startswith('aten::') and e.stack and e.device_time_total > 0:
        fr = [s for s in e.stack if 'sevennet_finetuning_amd' in s]
        by_src[(e.name, fr[0] if fr else '?')] += 1
# library kernels and runtime copies (no aten op of their own)
kern = collections.Counter()
for e in prof.events():
    if e.device_type == torch.autograd.DeviceType.CUDA:
        kern[e.name[:80]] += 1
print('device kernels:', sum(kern.values()))
for k, c in kern.most_common(60):
    print('  ', c, k)
for (name, src), c in by_src.most_common(60):
    print(c, name, src)
rows = []
for e in prof.key_averages():
    if e.key.startswith('aten::'):
        rows.append((e.count, e.key, round(e.device_time_total / 1e3, 3) if hasattr(e, 'device_time_total') else 0))
rows.sort(key=lambda r: -r[2])
for r in rows[:40]: print(r)
