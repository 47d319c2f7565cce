"""Model build / checkpoint / deploy surface (sevennet_finetuning_amd/model_build.py;
reference: model_build.py:186-445, util.py:186-231, scripts/deploy.py:15-117).
CPU tests: the configuration of the reference's fine-tuning input builds a
model whose parameter table is the SevenNet-0 deployment's (names, shapes,
order), e3nn initialisation, checkpoint and deploy round trips bit-exact,
derived irreps, and unsupported configurations refused with the reason."""
import json
import os

import numpy as np
import pytest
import torch

from _conv_cpu import CpuConvBackend
from sevennet_finetuning_amd import model_build as mb

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAN = json.load(open(os.path.join(ROOT, 'sevennet_finetuning_amd', 'assets', 'sevennet0',
                                  'manifest.json')))
# model section of example_inputs/fine_tuning/FT_w_reEWC/input_full.yaml
FT_MODEL = {
    'chemical_species': 'auto', 'cutoff': 5.0, 'channel': 128, 'is_parity': False, 'lmax': 2,
    'num_convolution_layer': 5,
    'irreps_manual': ['128x0e'] + ['128x0e+64x1e+32x2e'] * 4 + ['128x0e'],
    'weight_nn_hidden_neurons': [64, 64],
    'radial_basis': {'radial_basis_name': 'bessel', 'bessel_basis_num': 8},
    'cutoff_function': {'cutoff_function_name': 'XPLOR', 'cutoff_on': 4.5},
    'act_gate': {'e': 'silu', 'o': 'tanh'}, 'act_scalar': {'e': 'silu', 'o': 'tanh'},
    'train_shift_scale': True, 'train_denominator': True, 'self_connection_type': 'linear',
}


def ft_config():
    c = dict(FT_MODEL)
    c['chemical_species'] = list(MAN['chemical_symbols'])
    c['conv_denominator'] = MAN['conv_denominator'][0]
    return c


def test_config_builds_the_sevennet0_parameter_table():
    cfg = mb.resolve_config(ft_config())
    man = mb.model_manifest(cfg)
    assert cfg['chemical_species'] == MAN['chemical_symbols']       # alphabetical type map
    assert cfg['_type_map'][14] == MAN['chemical_symbols'].index('Si')
    key = lambda m: [(t['name'], t['shape'], t['offset'], t['numel']) for t in m['tensors']]
    assert key(man) == key(MAN)
    assert man['num_params'] == MAN['num_params'] == 842623
    assert man['irreps_manual'] == MAN['irreps_manual']
    mb._check_kernel_support(man)


def test_derived_irreps_and_refusals():
    c = ft_config()
    c['irreps_manual'] = False
    cfg = mb.resolve_config(c)
    assert [mb._irreps_str(i) for i in cfg['_irreps']] == \
        ['128x0e'] + ['128x0e+128x1e+128x2e'] * 4 + ['128x0e']
    # other family members are served by the runtime path tables (gtp.hip)
    mb._check_kernel_support(mb.model_manifest(cfg))
    c = ft_config()
    c['cutoff_function'] = {'cutoff_function_name': 'poly_cut'}
    man = mb.model_manifest(mb.resolve_config(c))
    mb._check_kernel_support(man)
    assert man['cutoff_function'] == {'name': 'poly_cut', 'p': 6.0}
    c = ft_config()
    c['self_connection_type'] = 'nequip'
    man = mb.model_manifest(mb.resolve_config(c))
    assert man['family'] == 'nequip'
    assert any(t['name'] == '0_self_connection_intro.fc_tensor_product.weight'
               for t in man['tensors'])
    c = ft_config()
    c['self_connection_type'] = 'mace'
    with pytest.raises(NotImplementedError, match='mace'):
        mb.model_manifest(mb.resolve_config(c))
    c = ft_config()
    c['irreps_manual'] = ['128x0e'] + ['128x0e+64x1e+32x3e'] * 4 + ['128x0e']
    with pytest.raises(NotImplementedError, match='l > 2'):
        mb._check_kernel_support(mb.model_manifest(mb.resolve_config(c)))
    c = ft_config()
    c['conv_denominator'] = 'avg_num_neigh'
    with pytest.raises(ValueError, match='dataset statistic'):
        mb.resolve_config(c)
    # parity: e3nn order ((l, p) tuples: 1o before 1e, as in the HfO2 example
    # deployment's mid irreps 8x0e+8x1o+4x1e) of the full tensor product
    out = mb.infer_irreps_out([(4, 0, 1), (4, 1, -1)], 1, -1, 1, 'full', False)
    assert mb._irreps_str(out) == '8x0e+8x1o+4x1e'


def test_init_weights_is_e3nn_initialisation():
    cfg = mb.resolve_config(ft_config())
    man = mb.model_manifest(cfg)
    flat = mb.init_weights(man, cfg, seed=3)
    t = {x['name']: x for x in man['tensors']}
    c = t['edge_embedding.basis_function.coeffs']
    assert np.allclose(flat[c['offset']:c['offset'] + 8], np.arange(1, 9) * np.pi / 5.0)
    d = t['2_convolution.denominator']
    assert flat[d['offset']] == np.float32(MAN['conv_denominator'][0])
    w = t['1_self_interaction_2.linear.weight']
    v = flat[w['offset']:w['offset'] + w['numel']]
    assert abs(v.mean()) < 0.02 and abs(v.std() - 1.0) < 0.02
    s = t['rescale_atomic_energy.scale']
    assert np.all(flat[s['offset']:s['offset'] + s['numel']] == 1.0)


def _build_cpu(seed):
    from sevennet_finetuning_amd.nn import SevenNetTrainable
    cfg = mb.resolve_config(ft_config())
    man = mb.model_manifest(cfg)
    m = SevenNetTrainable(device='cpu', conv_backend=CpuConvBackend(), manifest=man,
                          weights=mb.init_weights(man, cfg, seed))
    m.config = cfg
    return m


def test_checkpoint_and_deploy_round_trips(tmp_path):
    from sevennet_finetuning_amd.nn import SevenNetTrainable
    m = _build_cpu(1)
    with torch.no_grad():
        m.flat.add_(torch.randn_like(m.flat) * 1e-3)     # "fine-tuned"
    ck = mb.checkpoint_of(m)
    assert set(ck['model_state_dict']) == set(m.slices)
    torch.save(ck, tmp_path / 'ck.pth')
    back = torch.load(tmp_path / 'ck.pth', weights_only=True)   # a plain weights-only file
    m2 = _build_cpu(7)
    missing, unused = mb.load_state_dict(m2, back['model_state_dict'])
    assert not missing and not unused
    assert torch.equal(m2.flat, m.flat)
    out = mb.deploy(m, str(tmp_path / 'dep'))
    man = json.load(open(os.path.join(out, 'manifest.json')))
    assert man['comm_size'] == 480 and man['format'] == mb.FORMAT
    m3 = SevenNetTrainable(model_dir=out, device='cpu', conv_backend=CpuConvBackend())
    assert torch.equal(m3.flat, m.flat)
    raw = np.fromfile(os.path.join(out, 'weights.bin'), dtype='<f4')
    assert np.array_equal(raw, m.flat.numpy())


def test_hfo2_example_config_builds_the_exported_parameter_table():
    """The reference config of the HfO2 example deployment (sevenn 0.8.6:
    channel 4, lmax 1, is_parity, nequip self-connection, poly_cut, 4 blocks,
    full irreps in the last block) through model_build gives exactly the
    parameter table exported from the frozen archive (tools/export_hfo2.py)."""
    import json
    import os
    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                        'sevennet_finetuning_amd', 'assets', 'hfo2_example')
    ref = json.load(open(os.path.join(root, 'manifest.json')))
    cfg = mb.resolve_config({
        'chemical_species': 'Hf O', 'cutoff': 4.0, 'channel': 4, 'lmax': 1, 'is_parity': True,
        'num_convolution_layer': 4, 'irreps_manual': ref['irreps_manual'],
        'self_connection_type': 'nequip', 'conv_denominator': ref['conv_denominator'][0],
        '_normalize_sph': False,
        'cutoff_function': {'cutoff_function_name': 'poly_cut', 'poly_cut_p_value': 6}})
    man = mb.model_manifest(cfg)
    assert [(t['name'], t['numel']) for t in man['tensors']] == \
        [(t['name'], t['numel']) for t in ref['tensors']]
    assert man['family'] == 'nequip' and man['sh_normalize'] is False
    assert man['readout_hidden'] == ref['readout_hidden']
