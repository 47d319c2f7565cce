"""Compare the fused and v1 convolution kernels layer by layer on the box."""
import sys

import numpy as np
import torch

sys.path.insert(0, '.')
sys.path.insert(0, 'tests')
from _systems import load_manifest_symbols, system  # noqa: E402
from sevennet_finetuning_amd import _lib  # noqa: E402
from sevennet_finetuning_amd.model import E3GNNModel  # noqa: E402
from sevennet_finetuning_amd.neighbor import neighbor_list  # noqa: E402

syms = load_manifest_symbols()
pos, cell, types = system(sys.argv[1] if len(sys.argv) > 1 else 'si_rng0_2x2x1', syms)
m = E3GNNModel(device='cuda:0')
ei, sh = neighbor_list(pos, cell, m.cutoff)
vec = pos[ei[1]] + sh @ cell - pos[ei[0]]
dev = m.device
t32 = lambda a: torch.tensor(a, dtype=torch.int32, device=dev)
ty, c, nb = t32(types), t32(ei[0]), t32(ei[1])
v = torch.tensor(vec, dtype=torch.float32, device=dev)
n, E = len(types), ei.shape[1]
res = {}
for impl in ('v1', 'fused'):
    m.set_impl(impl)
    s = m.stream_handle()
    _lib.check(m.lib.e3gnn_graph_set(m._ctx, n, 0, E, ty.data_ptr(), c.data_ptr(), nb.data_ptr(),
                                     v.data_ptr(), s))
    out = {}
    for t in range(m.num_layers):
        _lib.check(m.lib.e3gnn_layer_forward(m._ctx, t, s))
        out[('h', t)] = m.debug_buffer('h', t)
        out[('agg', t)] = m.debug_buffer('agg', t)
        out[('x', t + 1)] = m.debug_buffer('x', t + 1)
    e = torch.zeros(1, device=dev)
    _lib.check(m.lib.e3gnn_readout(m._ctx, e.data_ptr(), None, s))
    for t in range(m.num_layers - 1, -1, -1):
        _lib.check(m.lib.e3gnn_layer_backward(m._ctx, t, s))
        out[('grad', t)] = m.debug_buffer('grad', t)
    for nm in ('dY', 'dgu', 'demb', 'dxc'):
        out[(nm, 0)] = m.debug_buffer(nm)
    out['E'] = float(e)
    res[impl] = out
a, b = res['v1'], res['fused']
print('energy v1', a['E'], 'fused', b['E'])
for k in a:
    if k == 'E':
        continue
    x, y = a[k], b[k]
    bad = ~np.isfinite(y)
    d = np.abs(x - y)
    print(k, 'n', x.size, 'nan', int(bad.sum()), 'maxdiff', float(np.nanmax(d)) if x.size else 0,
          'ref max', float(np.abs(x).max()) if x.size else 0,
          'first bad', int(np.argmax(bad)) if bad.any() else -1)
