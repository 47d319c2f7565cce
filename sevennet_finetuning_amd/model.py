"""Energy/force models on the HIP path -- the Python mirror of the reference's
model surface (SevenNet-0 and, through the generic engine of the same library,
any other deployment of the nequip family).

Reference surface mirrored here:
* ``AtomGraphSequential.forward(dict) -> dict`` (sevenn/nn/sequential.py:82-89)
  with the serial deployment's inputs/outputs (deploy.py:20-32,
  pair_e3gnn.cpp:205-256): ``x`` (type index), ``pos``, ``edge_index``,
  ``cell_lattice_vectors``, ``pbc_shift``, ``cell_volume``, ``num_atoms``
  (or a precomputed ``edge_vec``) -> ``inferred_total_energy``,
  ``atomic_energy``, ``inferred_force``, ``inferred_stress``.
* ``set_is_batch_data`` (sequential.py:38-46): batched graphs with a ``batch``
  vector give per-graph energies and stresses.
* ``build_E3_equivariant_model`` (model_build.py:186) and
  ``model_from_checkpoint`` (util.py:186-231) live in ``model_build.py``.

All arithmetic runs in libe3gnn_hip.so; torch is used for device memory and
host plumbing only.  There is no CPU fallback.
"""
import json
import os

import torch

from . import _keys as KEY
from . import _lib

ASSETS = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'assets')


class E3GNNModel:
    """A loaded deployment (weights.bin + manifest.json) on one HIP device."""

    def __init__(self, model_dir=os.path.join(ASSETS, 'sevennet0'), device=None):
        self.lib = _lib.load()
        if device is None:
            device = torch.device('cuda', torch.cuda.current_device())
        self.device = torch.device(device)
        if self.device.type != 'cuda':
            raise _lib.E3GNNError(f'the HIP path needs a GPU device, got {self.device}')
        self.model_dir = model_dir
        with open(os.path.join(model_dir, 'manifest.json')) as f:
            self.manifest = json.load(f)
        self.chemical_symbols = list(self.manifest['chemical_symbols'])
        self.cutoff = float(self.manifest['cutoff'])
        idx = self.device.index if self.device.index is not None else 0
        h = self.lib.e3gnn_load(os.path.join(model_dir, 'weights.bin').encode(),
                                os.path.join(model_dir, 'manifest.json').encode(), idx)
        if not h:
            raise _lib.E3GNNError(self.lib.e3gnn_last_error().decode())
        self._model = h
        self._ctx = self.lib.e3gnn_ctx_create(h)
        if not self._ctx:
            raise _lib.E3GNNError(self.lib.e3gnn_last_error().decode())
        ns, nl, cs = (_lib.ctypes.c_int(), _lib.ctypes.c_int(), _lib.ctypes.c_int())
        co = _lib.ctypes.c_float()
        _lib.check(self.lib.e3gnn_model_info(h, ns, co, nl, cs))
        self.num_species, self.num_layers, self.comm_size = ns.value, nl.value, cs.value
        # >= 0: the fused-kernel channel family serving it; -1: the generic engine
        self.family = int(self.lib.e3gnn_model_family(h))
        self.is_batch_data = False
        # outputs are device tensors on torch's current stream: return once the
        # evaluation is enqueued (stream order, like a torch module) rather than
        # synchronising; E3GNN_SYNC=1 restores the blocking call
        self.set_stream_ordered(os.environ.get('E3GNN_SYNC', '0') != '1')

    # --------------------------------------------------------------- metadata
    def type_map(self):
        """atomic number -> type index (chemical_symbols_to_index, deploy.py:34-51)."""
        from .structures import atomic_number
        return {atomic_number(s): i for i, s in enumerate(self.chemical_symbols)}

    def set_is_batch_data(self, flag: bool):
        self.is_batch_data = bool(flag)

    def close(self):
        if getattr(self, '_ctx', None):
            self.lib.e3gnn_ctx_free(self._ctx)
            self._ctx = None
        if getattr(self, '_model', None):
            self.lib.e3gnn_free(self._model)
            self._model = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # --------------------------------------------------------------- raw call
    def stream_handle(self):
        return torch.cuda.current_stream(self.device).cuda_stream

    def energy_forces(self, types, edge_center, edge_nbr, edge_vec, want_edge_grad=False):
        """One evaluation on device tensors (int32 types/centre/nbr, fp32 vec E x 3),
        edge_center sorted non-decreasing.  Returns dict of device tensors."""
        dev = self.device
        n = int(types.shape[0])
        E = int(edge_center.shape[0])
        types = types.to(dev, torch.int32).contiguous()
        edge_center = edge_center.to(dev, torch.int32).contiguous()
        edge_nbr = edge_nbr.to(dev, torch.int32).contiguous()
        edge_vec = edge_vec.to(dev, torch.float32).contiguous()
        energy = torch.empty(1, device=dev)
        eat = torch.empty(n, device=dev)
        forces = torch.empty(n, 3, device=dev)
        virial = torch.empty(6, device=dev)
        egrad = torch.empty(E, 3, device=dev) if want_edge_grad else None
        _lib.check(self.lib.e3gnn_energy_forces(
            self._ctx, n, E, types.data_ptr(), edge_center.data_ptr(), edge_nbr.data_ptr(),
            edge_vec.data_ptr(), energy.data_ptr(), eat.data_ptr(), forces.data_ptr(),
            virial.data_ptr(), egrad.data_ptr() if egrad is not None else None,
            self.stream_handle()))
        out = {'energy': energy[0], 'atomic_energy': eat, 'forces': forces, 'virial': virial}
        if egrad is not None:
            out['edge_grad'] = egrad
        return out

    def set_impl(self, impl):
        """'fused' (default) or 'v1' (unfused kernels, cross-check)."""
        _lib.check(self.lib.e3gnn_set_impl(self._ctx, {'fused': 0, 'v1': 1}[impl]))

    def set_stream_ordered(self, enable=True):
        _lib.check(self.lib.e3gnn_set_stream_ordered(self._ctx, int(enable)))

    def set_timing(self, enable=True):
        _lib.check(self.lib.e3gnn_set_timing(self._ctx, int(enable)))

    def kernel_stats(self):
        c = _lib.ctypes
        k = 32
        names = (c.c_char_p * k)()
        ms = (c.c_double * k)()
        la = (c.c_int64 * k)()
        fl = (c.c_double * k)()
        by = (c.c_double * k)()
        n = self.lib.e3gnn_kernel_stats(self._ctx, names, ms, la, fl, by, k)
        return {names[i].decode(): {'ms': ms[i], 'launches': la[i], 'flops': fl[i],
                                    'bytes': by[i]} for i in range(n)}

    def reset_stats(self):
        _lib.check(self.lib.e3gnn_reset_stats(self._ctx))

    def debug_buffer(self, name, layer=0):
        """Host copy (numpy fp32) of an internal workspace buffer (after a
        synchronising call)."""
        import ctypes
        import numpy as np
        n = ctypes.c_int64()
        ptr = self.lib.e3gnn_debug_ptr(self._ctx, name.encode(), layer, ctypes.byref(n))
        if not ptr:
            raise _lib.E3GNNError(f'no debug buffer {name}[{layer}]')
        out = np.empty(n.value, dtype=np.float32)
        torch.cuda.synchronize(self.device)
        hip = ctypes.CDLL('libamdhip64.so.7')  # torch's runtime (same SONAME)
        rc = hip.hipMemcpy(ctypes.c_void_p(out.ctypes.data), ctypes.c_void_p(ptr),
                           ctypes.c_size_t(out.nbytes), 2)
        if rc != 0:
            raise _lib.E3GNNError(f'hipMemcpy failed ({rc})')
        return out

    def workspace_bytes(self):
        return int(self.lib.e3gnn_workspace_bytes(self._ctx))

    # --------------------------------------------------------------- dict API
    def __call__(self, data):
        return self.forward(data)

    def forward(self, data):
        """AtomGraphSequential contract on an AtomGraphData-style dict."""
        dev = self.device
        types = torch.as_tensor(data[KEY.NODE_FEATURE]).to(dev).long()
        if types.dim() != 1:
            raise _lib.E3GNNError('x must hold one type index per atom')
        ei = torch.as_tensor(data[KEY.EDGE_IDX]).to(dev).long()
        if KEY.EDGE_VEC in data and data[KEY.EDGE_VEC] is not None:
            vec = torch.as_tensor(data[KEY.EDGE_VEC]).to(dev, torch.float32)
        else:  # EdgePreprocess (edge_embedding.py:62-76)
            pos = torch.as_tensor(data[KEY.POS]).to(dev, torch.float32)
            vec = pos[ei[1]] - pos[ei[0]]
            if KEY.CELL_SHIFT in data and data[KEY.CELL_SHIFT] is not None:
                shift = torch.as_tensor(data[KEY.CELL_SHIFT]).to(dev, torch.float32)
                cell = torch.as_tensor(data[KEY.CELL]).to(dev, torch.float32)
                if self.is_batch_data and cell.dim() == 3 or cell.numel() > 9:
                    batch = torch.as_tensor(data[KEY.BATCH]).to(dev).long()
                    cell = cell.view(-1, 3, 3)[batch[ei[0]]]
                    vec = vec + torch.bmm(shift.unsqueeze(1), cell).squeeze(1)
                else:
                    vec = vec + shift @ cell.view(3, 3)
        # the kernels require edges CSR-sorted by centre (edge_index[0])
        center = ei[0]
        perm = None
        if center.numel() > 1 and bool((center[1:] < center[:-1]).any()):
            perm = torch.argsort(center, stable=True)
            center, nbr, vec_s = center[perm], ei[1][perm], vec[perm]
        else:
            nbr, vec_s = ei[1], vec
        res = self.energy_forces(types, center, nbr, vec_s, want_edge_grad=True)
        egrad = res['edge_grad']
        if perm is not None:
            inv = torch.empty_like(perm)
            inv[perm] = torch.arange(perm.numel(), device=dev)
            egrad = egrad[inv]
        out = dict(data)
        n = types.shape[0]
        out[KEY.ATOMIC_ENERGY] = res['atomic_energy'].view(n, 1)
        out[KEY.PRED_FORCE] = res['forces']
        out[KEY.EDGE_GRAD] = egrad
        if self.is_batch_data and KEY.BATCH in data:
            batch = torch.as_tensor(data[KEY.BATCH]).to(dev).long()
            nb = int(batch.max().item()) + 1 if batch.numel() else 0
            e = torch.zeros(nb, device=dev).index_add_(0, batch, res['atomic_energy'])
            out[KEY.PRED_TOTAL_ENERGY] = e
            vol = torch.as_tensor(data[KEY.CELL_VOLUME]).to(dev, torch.float32).view(-1)
            r = vec
            f = egrad
            v6 = -torch.stack([r[:, 0] * f[:, 0], r[:, 1] * f[:, 1], r[:, 2] * f[:, 2],
                               0.5 * (r[:, 0] * f[:, 1] + r[:, 1] * f[:, 0]),
                               0.5 * (r[:, 1] * f[:, 2] + r[:, 2] * f[:, 1]),
                               0.5 * (r[:, 0] * f[:, 2] + r[:, 2] * f[:, 0])], dim=1)
            vir = torch.zeros(nb, 6, device=dev).index_add_(0, batch[ei[0]], v6)
            out[KEY.PRED_STRESS] = vir / vol.view(-1, 1)
        else:
            out[KEY.PRED_TOTAL_ENERGY] = res['energy']
            if KEY.CELL in data and data[KEY.CELL] is not None:
                cell = torch.as_tensor(data[KEY.CELL]).to(dev, torch.float64).view(3, 3)
                vol = torch.abs(torch.linalg.det(cell)).to(torch.float32)
                out[KEY.PRED_STRESS] = res['virial'] / vol
        return out


class GenericE3GNNModel:
    """Any other member of the nequip family (e.g. the reference's HfO2 example
    deployment: odd parity, lmax 1, FCTP self-connection, polynomial cutoff):
    the trainable model of nn.py in eval mode on the runtime-path-table HIP
    convolution (gtp.hip, e3gnn_gtp_*), with the E3GNNModel call surface
    (``energy_forces`` on device tensors, the ``AtomGraphSequential`` dict
    contract, ``type_map``, ``cutoff``).  Forces and virial are the edge-vector
    gradient scattered as ForceStressOutputFromEdge does (force_output.py:158-215);
    the SevenNet-0 architecture keeps the fully native E3GNNModel."""

    def __init__(self, model_dir, device=None):
        from .nn import SevenNetTrainable
        if device is None:
            device = torch.device('cuda', torch.cuda.current_device())
        self.device = torch.device(device)
        if self.device.type != 'cuda':
            raise _lib.E3GNNError(f'the HIP path needs a GPU device, got {self.device}')
        self.model_dir = model_dir
        self.net = SevenNetTrainable(model_dir=model_dir, device=self.device)
        self.net.eval()
        for p in self.net.parameters():
            p.requires_grad_(False)
        self.manifest = self.net.manifest
        self.chemical_symbols = self.net.chemical_symbols
        self.cutoff = self.net.cutoff
        self.num_species, self.num_layers = self.net.nsp, self.net.nlayer
        self.is_batch_data = False

    type_map = E3GNNModel.type_map

    def set_is_batch_data(self, flag: bool):
        self.is_batch_data = bool(flag)

    def energy_forces(self, types, edge_center, edge_nbr, edge_vec, want_edge_grad=False):
        dev = self.device
        n = int(types.shape[0])
        ei = torch.stack([edge_center.to(dev).long(), edge_nbr.to(dev).long()])
        data = {KEY.NODE_FEATURE: types.to(dev).long(), KEY.EDGE_IDX: ei,
                KEY.EDGE_VEC: edge_vec.to(dev, torch.float32),
                KEY.NUM_ATOMS: torch.tensor([n], device=dev),
                KEY.CELL_VOLUME: torch.ones(1, device=dev)}
        out = self.net(data)
        # with a unit volume the model's stress is the virial (xx,yy,zz,xy,yz,zx)
        res = {'energy': out[KEY.PRED_TOTAL_ENERGY].detach()[0],
               'atomic_energy': out[KEY.ATOMIC_ENERGY].detach().view(n),
               'forces': out[KEY.PRED_FORCE].detach(),
               'virial': out[KEY.PRED_STRESS].detach().view(6)}
        if want_edge_grad:
            raise _lib.E3GNNError('edge gradients are exposed by the SevenNet-0 engine only')
        return res

    def __call__(self, data):
        return self.forward(data)

    def forward(self, data):
        """AtomGraphSequential contract (sequential.py:82-89) on a dict."""
        dev = self.device
        d = dict(data)
        d[KEY.NODE_FEATURE] = torch.as_tensor(data[KEY.NODE_FEATURE]).to(dev).long()
        ei = torch.as_tensor(data[KEY.EDGE_IDX]).to(dev).long()
        d[KEY.EDGE_IDX] = ei
        if KEY.EDGE_VEC not in data or data[KEY.EDGE_VEC] is None:
            pos = torch.as_tensor(data[KEY.POS]).to(dev, torch.float32)
            vec = pos[ei[1]] - pos[ei[0]]
            if KEY.CELL_SHIFT in data and data[KEY.CELL_SHIFT] is not None:
                shift = torch.as_tensor(data[KEY.CELL_SHIFT]).to(dev, torch.float32)
                cell = torch.as_tensor(data[KEY.CELL]).to(dev, torch.float32).view(3, 3)
                vec = vec + shift @ cell
            d[KEY.EDGE_VEC] = vec
        if KEY.CELL_VOLUME not in d and KEY.CELL in data and data[KEY.CELL] is not None:
            cell = torch.as_tensor(data[KEY.CELL]).to(dev, torch.float64).view(3, 3)
            d[KEY.CELL_VOLUME] = torch.abs(torch.linalg.det(cell)).to(torch.float32).view(1)
        out = self.net(d)
        if not self.is_batch_data:
            out[KEY.PRED_TOTAL_ENERGY] = out[KEY.PRED_TOTAL_ENERGY][0]
            if KEY.PRED_STRESS in out:
                out[KEY.PRED_STRESS] = out[KEY.PRED_STRESS][0]
        return out


def load_model(model_dir=os.path.join(ASSETS, 'sevennet0'), device=None, engine='native'):
    """The engine for a deployment (pair_e3gnn.cpp:294-386 loads any deployed
    model): the native C-ABI engine (E3GNNModel -- SevenNet-0's specialised
    kernels, or the generic engine of libe3gnn_hip.so for the rest of the
    family); ``engine='torch'``: the trainable model in eval mode
    (GenericE3GNNModel, autograd backward) for the non-SevenNet-0 ones."""
    from .nn import sevennet0_kinds
    if engine not in ('native', 'torch'):
        raise ValueError(f"engine must be 'native' or 'torch', got {engine!r}")
    with open(os.path.join(model_dir, 'manifest.json')) as f:
        man = json.load(f)
    if engine == 'native' or sevennet0_kinds(man) is not None:
        return E3GNNModel(model_dir, device)
    return GenericE3GNNModel(model_dir, device)
