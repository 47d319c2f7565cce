"""Diagnostic: the rehearsal body captured by hand, replayed repeatedly on
unchanged static inputs; prints the first pass's predictions and losses per
replay (an uninitialised read or a race shows as replay-to-replay garbage)."""
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
MODE = sys.argv[1] if len(sys.argv) > 1 else 'adam'
m = SevenNetTrainable(device=dev)
cfg = {'loss': 'huber', 'loss_param': {'delta': 0.01}, 'force_loss_weight': 1.0,
       'stress_loss_weight': 0.01, 'is_train_stress': True, 'optimizer': 'adam',
       'optim_param': {'lr': 0.0}, 'scheduler': 'exponentiallr',
       'scheduler_param': {'gamma': 0.99}, 'device': dev, 'hip_graph': True}
tr = train.Trainer(m, cfg)
m.train(True)
if MODE == 'sgd':
    class _Sgd:
        def step(self):
            with torch.no_grad():
                m.flat.sub_(0.0 * m.flat_grad)
    tr.optimizer = _Sgd()
elif MODE == 'adam_noforeach':
    params = [p for p in m.parameters() if p.requires_grad]
    tr.optimizer = torch.optim.Adam(params, lr=torch.tensor(0.0, device=dev), capturable=True,
                                    foreach=False)
elif MODE == 'adam_flat':
    tr.optimizer = torch.optim.Adam([m.flat], lr=torch.tensor(0.0, device=dev), capturable=True)
    m.flat.grad = m.flat_grad
print('mode', MODE, flush=True)
batches = bt.make_batches(0, 2, 8, m.chemical_symbols)
sb, sm = (train.collate(b, device=dev, dtype=torch.float32) for b in batches)
graphs = tuple(conv_ops.ConvGraph(int(b[KEY.NODE_FEATURE].shape[0]), b[KEY.EDGE_IDX][0],
                                  b[KEY.EDGE_IDX][1], m.conv_backend) for b in (sb, sm))
keep = {}


def body():
    tr.zero_grad()
    out = m(sb, graph=graphs[0])
    loss = tr.total_loss(out)
    tr.backward(loss)
    tr.optimizer.step()
    memout = m(sm, graph=graphs[1])
    mloss = tr.total_loss(memout)
    tr.backward(mloss)
    tr.optimizer.step()
    keep['e'] = out[KEY.PRED_TOTAL_ENERGY].detach()
    keep['f'] = out[KEY.PRED_FORCE].detach()
    keep['s'] = out[KEY.PRED_STRESS].detach()
    keep['s2'] = memout[KEY.PRED_STRESS].detach()
    return loss.detach(), mloss.detach()


print('eager', [float(x) for x in body()], float(keep['s'].abs().max()), flush=True)
side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    for _ in range(2):
        body()
torch.cuda.current_stream().wait_stream(side)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    out = body()
for i in range(6):
    g.replay()
    torch.cuda.synchronize()
    print(f'replay {i}: loss {float(out[0]):.6g} {float(out[1]):.6g} E {float(keep["e"].sum()):.6g} '
          f'|F| {float(keep["f"].abs().max()):.6g} |S| {float(keep["s"].abs().max()):.6g} '
          f'|S mem| {float(keep["s2"].abs().max()):.6g} finite {bool(torch.isfinite(m.flat).all())}',
          flush=True)
