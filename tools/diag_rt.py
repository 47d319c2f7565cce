"""Diagnostic: HIP runtime sharing between torch and libe3gnn_hip.so."""
import ctypes
import sys

import torch

order = sys.argv[1] if len(sys.argv) > 1 else 'torch_first'
hip = ctypes.CDLL('libamdhip64.so.7')


def last(tag):
    e = hip.hipGetLastError()
    print(f'[{tag}] hipGetLastError={e}', flush=True)


if order == 'torch_first':
    x = torch.ones(4, device='cuda')
    print('torch init ok', float(x.sum()), flush=True)
last('after torch init')
sys.path.insert(0, '.')
from sevennet_finetuning_amd import _lib  # noqa: E402
lib = _lib.load()
print('abi', lib.e3gnn_abi_version(), flush=True)
last('after lib load')
try:
    y = torch.ones(4, device='cuda') * 2
    print('torch op after lib load ok', float(y.sum()), flush=True)
except Exception as e:
    print('torch op after lib load FAILED', e, flush=True)
last('x')
from sevennet_finetuning_amd.model import E3GNNModel  # noqa: E402
m = E3GNNModel(device='cuda:0')
print('model loaded', flush=True)
last('after e3gnn_load')
try:
    y = torch.ones(4, device='cuda') * 3
    print('torch op after model load ok', float(y.sum()), flush=True)
except Exception as e:
    print('torch op after model load FAILED', e, flush=True)
