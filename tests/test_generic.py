"""Host logic of the nequip-family generalisation on the CPU (no GPU): the
trainable model of nn.py on a generic (runtime path table) convolution double
reproduces the fp64 oracle for the HfO2 example deployment, and the runtime
path tables reproduce the SevenNet-0 kernel kinds."""
import os

import numpy as np
import torch

from _conv_cpu import CpuConvBackend, GenericCpuConvBackend
from _systems import GOLD, load_manifest_symbols, system
from sevennet_finetuning_amd import _keys as KEY
from sevennet_finetuning_amd import conv_ops, train
from sevennet_finetuning_amd.nn import SevenNetTrainable, parse_irreps, path_table

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HFO2 = os.path.join(ROOT, 'sevennet_finetuning_amd', 'assets', 'hfo2_example')


def test_trainable_hfo2_example_equals_oracle():
    from oracle.neighbor import neighbor_list
    from oracle.nequip_ref import NequIPRef
    m = SevenNetTrainable(model_dir=HFO2, device='cpu', conv_backend=GenericCpuConvBackend(),
                          dtype=torch.float64)
    m.eval()
    d = np.load(f'{GOLD}/hfo2_resdat.npz')
    types = np.array([m.chemical_symbols.index(str(s)) for s in d['symbols']])
    out = m(train.collate([train.labeled_graph(d['pos'], d['cell'], types, m.cutoff)],
                          dtype=torch.float64))
    ei, sh = neighbor_list(d['pos'], d['cell'], 4.0)
    ref = NequIPRef(HFO2)(torch.tensor(d['pos']), torch.tensor(types), torch.tensor(ei),
                          torch.tensor(sh), torch.tensor(d['cell']))
    e = float(out[KEY.PRED_TOTAL_ENERGY][0])
    assert abs(e - float(ref['energy'])) < 1e-9 * abs(e)
    assert float((out[KEY.PRED_FORCE] - ref['forces']).abs().max()) < 1e-9
    assert float((out[KEY.PRED_STRESS][0] - ref['stress']).abs().max()) < 1e-9


def test_runtime_tables_reproduce_sevennet0_kinds():
    """The SevenNet-0 blocks through path_table + the generic double equal the
    kind-specialised double (same instruction order and mid-irreps sort)."""
    mid = parse_irreps('128x0e+64x1e+32x2e')
    tabs = [path_table(parse_irreps('128x0e'), 2, 1, mid)[0], path_table(mid, 2, 1, mid)[0],
            path_table(mid, 2, 1, parse_irreps('128x0e'))[0]]
    gen, spec = GenericCpuConvBackend(), CpuConvBackend()
    gen.configure(tabs)
    rng = np.random.default_rng(0)
    n = 7
    center = torch.tensor(np.repeat(np.arange(n), 3))
    nbr = torch.tensor(rng.integers(0, n, len(center)))
    for kind in range(3):
        assert gen.dims[kind] == spec.dims[kind]
        dx, dw, dm = spec.dims[kind]
        h = torch.tensor(rng.normal(size=(n, dx)))
        Y = torch.tensor(rng.normal(size=(len(center), 9)))
        w = torch.tensor(rng.normal(size=(len(center), dw)))
        g = conv_ops.ConvGraph(n, center, nbr, gen)
        assert torch.allclose(gen.forward(kind, g, h, Y, w), spec.forward(kind, g, h, Y, w),
                              rtol=1e-12, atol=1e-12)


def test_sevennet0_kinds_selected_for_sevennet0_only():
    syms = load_manifest_symbols()
    m = SevenNetTrainable(device='cpu', conv_backend=CpuConvBackend(), dtype=torch.float64)
    assert m._sevennet0_kinds() == [0, 1, 1, 1, 2]
    h = SevenNetTrainable(model_dir=HFO2, device='cpu', conv_backend=GenericCpuConvBackend(),
                          dtype=torch.float64)
    assert h._sevennet0_kinds() is None
    assert [b['kind'] for b in h.blocks] == [0, 1, 2, 3]
    pos, cell, types = system('si_rng0_1x1x1', syms)
    assert len(pos) == 8


def test_gate_layout_matches_hand_derived_e3nn_gate():
    """nn._gate_irreps against e3nn's Gate layout derived by hand
    (equivariant_gate.py:30-51 builds Gate(scalars, gates, gated); e3nn's
    _Sortcut simplifies each group, stable-sorts the concatenation by the Irrep
    tuple (l, p) -- p = -1 before +1 -- and simplifies again):
      '4x0e+4x0o+4x1e': gates '4x0e' ('0e' is among the scalars);
        pieces [4x0e | 4x0o | gates 4x0e | 4x1e] sort to 0o(1), 0e(0), 0e(2), 1e(3)
        -> irreps_in 4x0o+8x0e+4x1e, offsets 4, 0, 8, 12, not the natural order;
      '4x0o+4x1e': gates '4x0o' (no '0e') -> 8x0o+4x1e, offsets 0, 4, 8, natural."""
    from sevennet_finetuning_amd.nn import _gate_irreps
    simp, scal, gated, (gate_p, offs, natural) = _gate_irreps([(4, 0, 1), (4, 0, -1), (4, 1, 1)])
    assert simp == [(4, 0, -1), (8, 0, 1), (4, 1, 1)]
    assert scal == [(4, 0, 1), (4, 0, -1)] and gated == [(4, 1, 1)]
    assert gate_p == 1 and offs == [4, 0, 8, 12] and natural is False
    simp, scal, gated, (gate_p, offs, natural) = _gate_irreps([(4, 0, -1), (4, 1, 1)])
    assert simp == [(8, 0, -1), (4, 1, 1)]
    assert gate_p == -1 and offs == [0, 4, 8] and natural is True
    # the oracle's restatement gives the same hand-derived layout
    from oracle.nequip_ref import gate_irreps
    ir, _, _, gp, offs = gate_irreps([(4, 0, 1), (4, 0, -1), (4, 1, 1)])
    assert [tuple(t) for t in ir] == [(4, 0, -1), (8, 0, 1), (4, 1, 1)] and gp == 1 and offs == [4, 0, 8, 12]
    ir, _, _, gp, offs = gate_irreps([(4, 0, -1), (4, 1, 1)])
    assert [tuple(t) for t in ir] == [(8, 0, -1), (4, 1, 1)] and gp == -1 and offs == [0, 4, 8]
