"""Phase breakdown of the middle-block backward (k_conv_bwd_ls<LayerMid>) from a
DIAGNOSTIC build of the library (-DE3GNN_STAMPS: s_memtime stamps per phase,
per wave, written to a buffer of their own; the shipped library has none).

    python tools/stamps.py <variant.so> [cells] [fwd]

Builds nothing: the variant is made beforehand on the CPU with
``build_lib.build(out=..., defines=['E3GNN_STAMPS'])``.  Prints, over all
waves of the last middle launch of one step, the share of wave cycles in
each phase and the mean cycles per wave.  The stamps themselves cost ~10 %
(each s_memtime waits for outstanding scalar/LDS operations).
"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PHASES = ['tile start', 'setup+MLP chain', 'barriers+staging', 'w recompute', 'dH2',
          'TP (+dxc stores)', 'tile end', 'TOTAL']
# a variant built with E3GNN_STAMPS_FWD=1 stamps the middle FORWARD instead
PHASES_FWD = ['pass start', 'setup+MLP chain', 'w MFMAs', 'tensor product', 'path start (rows)',
              'row sums + LDS acc', 'copy-out', 'TOTAL']


def main():
    lib_path = os.path.abspath(sys.argv[1])
    cells = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 23
    names = PHASES_FWD if 'fwd' in sys.argv[2:] else PHASES
    os.environ['E3GNN_LIB'] = lib_path
    import bench
    from sevennet_finetuning_amd import _lib
    from sevennet_finetuning_amd.model import E3GNNModel
    dev = torch.device('cuda', 0)
    model = E3GNNModel(device=dev)
    box = bench.make_box(cells, dev)
    lib = ctypes.CDLL(lib_path)
    lib.e3gnn_debug_stamps.argtypes = [ctypes.c_void_p]
    n = box['n']
    buf = torch.zeros((n + 64) * 8, dtype=torch.int64, device=dev)
    step = lambda: model.energy_forces(box['types'], box['center'], box['nbr'], box['vec'])  # noqa: E731
    step()
    torch.cuda.synchronize()
    assert lib.e3gnn_debug_stamps(ctypes.c_void_p(buf.data_ptr())) == 0
    step()   # the three middle launches overwrite the same slots: the last one stays
    torch.cuda.synchronize()
    assert lib.e3gnn_debug_stamps(None) == 0
    a = buf.view(-1, 8)[:n].cpu().numpy().astype(np.float64)
    a = a[a[:, 7] > 0]
    tot = a[:, 7].sum()
    print(f'waves {len(a)}, mean cycles/wave {a[:, 7].mean():.0f}, '
          f'max {a[:, 7].max():.0f}')
    for k in range(7):
        print(f'  {names[k]:18s} {a[:, k].sum() / tot:6.3f}   {a[:, k].mean():10.0f} cyc/wave')
    print(f'  unaccounted        {1 - a[:, :7].sum() / tot:6.3f}')
    del _lib


if __name__ == '__main__':
    main()
