"""ASE calculator on the HIP path -- mirrors SevenNetCalculator
(sevenn/sevennet_calculator.py:17-157): same constructor arguments, same
``results`` keys (energy, free_energy, energies, forces, stress) and the same
ASE stress convention (-sigma in Voigt order xx yy zz yz xz xy, :151-156).

ASE is optional: when importable the class derives from
``ase.calculators.calculator.Calculator``; otherwise it duck-types the parts
of that interface the reference uses (``calculate(atoms)`` / ``results``).
"""
import numpy as np
import torch

from . import _keys as KEY
from .model import load_model
from .util import pretrained_name_to_path, unlabeled_atoms_to_graph

try:  # pragma: no cover - ase is not installed in this image
    from ase.calculators.calculator import Calculator, all_changes
except ImportError:  # minimal stand-in
    all_changes = ('positions', 'numbers', 'cell', 'pbc')

    class Calculator:
        implemented_properties = []

        def __init__(self, **kwargs):
            self.results = {}
            self.atoms = None

        def calculate(self, atoms=None, properties=None, system_changes=all_changes):
            self.atoms = atoms

        def get_property(self, name, atoms=None):
            self.calculate(atoms)
            return self.results[name]


class SevenNetCalculator(Calculator):
    def __init__(self, model='SevenNet-0', file_type='checkpoint', device='auto',
                 sevennet_config=None, **kwargs):
        super().__init__(**kwargs)
        file_type = file_type.lower()
        if file_type not in ('checkpoint', 'torchscript', 'deployed'):
            raise ValueError('file_type should be checkpoint or torchscript')
        if not isinstance(device, (str, torch.device)):
            raise ValueError('device must be an instance of torch.device or str.')
        if isinstance(device, str) and device == 'auto':
            # the reference falls back to 'cpu' here (sevennet_calculator.py:57-62);
            # this build has no CPU engine, so 'auto' means the first GPU
            device = torch.device('cuda', 0)
        self.device = torch.device(device)
        if self.device.type != 'cuda':
            # an explicit refusal, never a silent CPU fallback: the evaluation
            # runs only in libe3gnn_hip.so's HIP kernels
            raise ValueError(
                f"SevenNetCalculator(device='{self.device}'): this build evaluates the "
                "model only on an AMD GPU through its HIP library (libe3gnn_hip.so); "
                "there is no CPU path. Use device='cuda' / 'cuda:N' (ROCm) or 'auto'.")
        import os
        path = model if os.path.isdir(str(model)) else pretrained_name_to_path(model)
        # the native SevenNet-0 engine, or the generic one for other models of
        # the family (e.g. the HfO2 example deployment)
        self.model = load_model(path, device=self.device)
        self.type_map = self.model.type_map()
        self.cutoff = self.model.cutoff
        self.sevennet_config = sevennet_config
        self.implemented_properties = ['free_energy', 'energy', 'forces', 'stress', 'energies']
        self._nlist = None

    def _types(self, atoms):
        try:
            return np.array([self.type_map[int(z)] for z in atoms.get_atomic_numbers()])
        except KeyError as e:
            raise ValueError(f'atomic number {e} is not a species of this model') from None

    def _calculate_device_graph(self, atoms):
        """Graph built by the device neighbour list (periodic or isolated
        systems): positions go to the GPU once, nothing comes back until the
        results."""
        from .neighbor import DeviceNeighborList
        if self._nlist is None:
            self._nlist = DeviceNeighborList(self.device)
        pbc = bool(np.all(atoms.get_pbc()))
        cell = np.array(atoms.get_cell(), dtype=np.float64)
        center, nbr, _, vec = self._nlist(atoms.get_positions(), cell if pbc else None,
                                          self.cutoff, (pbc,) * 3)
        types = torch.as_tensor(self._types(atoms), dtype=torch.int32, device=self.device)
        res = self.model.energy_forces(types, center, nbr, vec)
        energy = float(res['energy'].item())
        self.results = {
            'free_energy': energy,
            'energy': energy,
            'energies': res['atomic_energy'].cpu().numpy(),
            'forces': res['forces'].cpu().numpy(),
        }
        if pbc:
            sigma = res['virial'].cpu().numpy() / abs(np.linalg.det(cell))
            self.results['stress'] = -sigma[[0, 1, 2, 4, 5, 3]]
        return res

    def calculate(self, atoms=None, properties=None, system_changes=all_changes):
        Calculator.calculate(self, atoms, properties, system_changes)
        if atoms is None:
            raise ValueError('No atoms to evaluate')
        pbc = np.asarray(atoms.get_pbc(), dtype=bool).reshape(-1)
        if pbc.all() or not pbc.any():
            return self._calculate_device_graph(atoms)
        # mixed periodicity (slabs): the host list (util.unlabeled_atoms_to_graph)
        data = unlabeled_atoms_to_graph(atoms, self.cutoff)
        data[KEY.NODE_FEATURE] = self._types(atoms)
        out = self.model(data)
        energy = float(out[KEY.PRED_TOTAL_ENERGY].item())
        self.results = {
            'free_energy': energy,
            'energy': energy,
            'energies': out[KEY.ATOMIC_ENERGY].detach().cpu().reshape(len(atoms)).numpy(),
            'forces': out[KEY.PRED_FORCE].detach().cpu().numpy(),
        }
        if KEY.PRED_STRESS in out:
            self.results['stress'] = np.array(
                (-out[KEY.PRED_STRESS]).detach().cpu().numpy()[[0, 1, 2, 4, 5, 3]])


class SevenNetD3Calculator(Calculator):
    """SevenNet-0 + DFT-D3 in one calculator: what LAMMPS runs as
    ``pair_style hybrid/overlay e3gnn d3 <rthr> <cn_thr> <damping> <functional>``
    (the reference's pair_e3gnn.cpp + pair_d3.cu), i.e. energies, forces and
    stresses of the two terms summed.  Per-atom energies are the SevenNet
    ones (the D3 term is not atom-decomposed, as in pair_d3.cu)."""

    def __init__(self, model='SevenNet-0', file_type='checkpoint', device='auto',
                 damping_type='damp_bj', functional_name='pbe', vdw_cutoff=9000.0,
                 cn_cutoff=1600.0, **kwargs):
        super().__init__(**kwargs)
        from .d3 import D3Calculator
        self.sevennet = SevenNetCalculator(model, file_type, device)
        dev = self.sevennet.device
        self.d3 = D3Calculator(damping_type, functional_name, vdw_cutoff, cn_cutoff,
                               device=dev.index or 0)
        self.implemented_properties = ['free_energy', 'energy', 'forces', 'stress', 'energies']

    def calculate(self, atoms=None, properties=None, system_changes=all_changes):
        a = self.sevennet
        a.calculate(atoms, properties, system_changes)
        b = self.d3.calculate(atoms)
        r = dict(a.results)
        r['energy'] = r['free_energy'] = a.results['energy'] + b['energy']
        r['forces'] = a.results['forces'] + b['forces']
        # stress only where both terms define one (periodic cells)
        if 'stress' in a.results and 'stress' in b:
            r['stress'] = a.results['stress'] + b['stress']
        else:
            r.pop('stress', None)
        self.results = r
        self.atoms = atoms
        return r
