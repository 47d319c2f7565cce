"""Model construction, checkpoints and deployment -- the reference's
``model_build`` / ``util`` / ``deploy`` surface for this build.

* ``build_E3_equivariant_model(config, parallel=False)``
  (sevenn/model_build.py:186-445): the reference's model config (same keys,
  ``sevenn/_keys.py``; defaults of ``_const.DEFAULT_E3_EQUIVARIANT_MODEL_CONFIG``)
  -> a trainable model (``nn.SevenNetTrainable``, reference parameter names and
  order) with e3nn's initialisation.  ``parallel=True`` returns the same model:
  here the parallel split is the segment C ABI over one deployment
  (``_to_parallel_model``, model_build.py:103-182, cuts at the same layer
  boundaries; ``parallel.py`` drives it).
* ``model_from_checkpoint(checkpoint)`` (util.py:186-231): a
  ``{'model_state_dict', 'config'}`` dict (or a file of one, loaded
  weights-only) -> (model, config).
* ``deploy(model, out_dir)`` (scripts/deploy.py:15-51, :55-117): the model's
  parameters -> this build's deployment format (``weights.bin`` fp32 +
  ``manifest.json``, the ``_extra_files`` metadata incl. ``comm_size``), which
  ``model.E3GNNModel``, ``SevenNetCalculator``, the segment API and
  ``native/e3gnn_md`` load.  One deployment serves the serial and the parallel
  path (the reference writes one TorchScript file per segment).

``build_E3_equivariant_model`` derives the irreps from the config exactly as
the reference does.  SevenNet-0's architecture (128x0e -> 4 x
128x0e+64x1e+32x2e -> 128x0e, lmax 2, even parity, linear self-connection)
runs on its specialised kernels (csrc/tp.h, fused.hip); every other member of
the nequip family -- odd parity, other multiplicities / lmax <= 2, the
``nequip`` FullyConnectedTensorProduct self-connection, the polynomial cutoff
(the reference's HfO2 example deployment is one) -- on the runtime path tables
(gtp.hip).  Configurations outside that (l > 2, other interaction types) are
refused with the reason.
"""
import datetime
import json
import math
import os

import numpy as np
import torch

from .structures import CHEMICAL_SYMBOLS

# sevenn/_const.py:92-124 (the keys this build reads)
DEFAULTS = {
    'irreps_manual': False,
    'channel': 32,
    'lmax': 1,
    'lmax_edge': -1,
    'lmax_node': -1,
    'is_parity': True,
    'radial_basis': {'radial_basis_name': 'bessel'},
    'cutoff_function': {'cutoff_function_name': 'poly_cut'},
    'act_radial': 'silu',
    'cutoff': 4.5,
    'weight_nn_hidden_neurons': [64, 64],
    'num_convolution_layer': 3,
    'conv_denominator': 'avg_num_neigh',
    'train_denominator': False,
    'train_shift_scale': False,
    'use_bias_in_linear': False,
    'readout_as_fcn': False,
    'readout_fcn_hidden_neurons': [30, 30],
    'readout_fcn_activation': 'relu',
    'self_connection_type': 'nequip',
    'interaction_type': 'nequip',
    'act_scalar': {'e': 'silu', 'o': 'tanh'},
    'act_gate': {'e': 'silu', 'o': 'tanh'},
    '_normalize_sph': True,
    'use_species_wise_shift_scale': True,
    'shift': 0.0,
    'scale': 1.0,
}
# e3nn normalize2mom(silu) (sevenn/_const.py act table; frozen c5 of the
# SevenNet-0 deployment, reproduced by tools/export_weights.py)
SILU_NORM = 1.6791767923989418
# e3nn normalize2mom(tanh) (the HfO2 example deployment's frozen constant)
TANH_NORM = 1.5937334472592695
FORMAT = 'e3gnn-mi355x/1'
BUILD_VERSION = 'sevennet_finetuning_amd-0.2'


# ------------------------------------------------------------------ irreps
def _irreps_str(irreps):
    return '+'.join(f'{m}x{l}{"e" if p == 1 else "o"}' for m, l, p in irreps)


def _parse(s):
    out = []
    for term in str(s).split('+'):
        mul, ir = term.strip().split('x')
        out.append((int(mul), int(ir[:-1]), 1 if ir[-1] == 'e' else -1))
    return out


def _dim(irreps):
    return sum(m * (2 * l + 1) for m, l, _ in irreps)


def infer_irreps_out(irreps_x, lmax_filter, parity_filter, drop_l, parity_mode,
                     fix_multiplicity):
    """util.infer_irreps_out (util.py:289-313) for an SH filter
    0e+1p+2e... (p = parity_filter^l): the full tensor product's output irreps,
    sorted and merged like e3nn (by the (l, p) tuple: 1o before 1e, as
    the HfO2 example deployment's frozen mid irreps show), l > drop_l removed, odd
    ones removed in 'even' mode, multiplicity optionally fixed."""
    acc = {}
    for mul, l1, p1 in irreps_x:
        for l2 in range(lmax_filter + 1):
            p2 = parity_filter ** l2
            for l3 in range(abs(l1 - l2), l1 + l2 + 1):
                key = (l3, p1 * p2)
                acc[key] = acc.get(key, 0) + mul
    out = []
    for (l, p) in sorted(acc):
        if drop_l is not False and l > drop_l:
            continue
        if parity_mode == 'even' and p == -1:
            continue
        out.append((fix_multiplicity if fix_multiplicity else acc[(l, p)], l, p))
    return out


def resolve_config(config):
    """Reference defaults + derived keys (type map, species count, per-layer
    irreps, denominators) of a model config."""
    cfg = dict(DEFAULTS)
    cfg.update(config or {})
    species = cfg.get('chemical_species')
    if isinstance(species, str) and species.lower() != 'auto':
        species = species.split()
    if not species or (isinstance(species, str)):
        if '_type_map' in cfg:   # {Z: type index}
            tm = {int(z): int(i) for z, i in dict(cfg['_type_map']).items()}
            species = [CHEMICAL_SYMBOLS[z] for z in sorted(tm, key=tm.get)]
        else:
            raise ValueError('chemical_species must be given (no dataset to infer it from)')
    # util.chemical_species_preprocess (util.py:248-261): type index = position
    # in the alphabetically sorted symbols
    species = sorted(s.strip() for s in species)
    cfg['chemical_species'] = species
    cfg['_number_of_species'] = len(species)
    cfg['_type_map'] = {CHEMICAL_SYMBOLS.index(s): i for i, s in enumerate(species)}
    L = int(cfg['num_convolution_layer'])
    lmax = int(cfg['lmax'])
    lmax_edge = int(cfg['lmax_edge']) if int(cfg['lmax_edge']) > 0 else lmax
    lmax_node = int(cfg['lmax_node']) if int(cfg['lmax_node']) > 0 else lmax
    parity = -1 if cfg['is_parity'] else 1
    if cfg['irreps_manual'] is not False:
        irreps = [_parse(s) for s in cfg['irreps_manual']]
        if len(irreps) != L + 1:
            raise RuntimeError('invalid irreps_manual input given')
    else:
        ch = int(cfg['channel'])
        irreps = [[(ch, 0, 1)]]
        for t in range(L):
            last = t == L - 1
            irreps.append(infer_irreps_out(irreps[-1], lmax_edge, parity,
                                           0 if last else lmax_node,
                                           'even' if last else 'full', ch))
    cfg['_irreps'] = irreps
    cfg['_lmax_edge'] = lmax_edge
    cfg['_lmax_node'] = lmax_node
    den = cfg['conv_denominator']
    if isinstance(den, str):
        if 'avg_num_neigh' in cfg and not isinstance(cfg['avg_num_neigh'], str):
            v = float(cfg['avg_num_neigh'])
            den = math.sqrt(v) if den == 'sqrt_avg_num_neigh' else v
        else:
            raise ValueError(f'conv_denominator {den!r} needs a dataset statistic: '
                             'give a number (or avg_num_neigh)')
    cfg['_conv_denominator'] = [float(d) for d in den] if isinstance(den, (list, tuple)) \
        else [float(den)] * L
    return cfg


def _gate_irreps(irreps_out):
    """EquivariantGate irreps_in (equivariant_gate.py:30-51): nn._gate_irreps
    (gate parity by the scalars, e3nn's (l, p) sort, equal neighbours merged)."""
    from .nn import _gate_irreps as gate_irreps
    return gate_irreps(irreps_out)[0]


def _conv_instructions(irreps_x, lmax_filter, parity_filter, irreps_out):
    """IrrepsConvolution instructions (convolution.py:72-95): every (x irrep,
    filter irrep, output irrep) whose output irrep is one of the block's output
    irreps ("here we drop l > lmax"); weight numel = mul."""
    allowed = {(l, p) for _, l, p in irreps_out}
    ins = []
    for mul, l1, p1 in irreps_x:
        for l2 in range(lmax_filter + 1):
            for l3 in range(abs(l1 - l2), l1 + l2 + 1):
                if (l3, p1 * parity_filter ** l2) in allowed:
                    ins.append((mul, l1, l2, l3, p1 * parity_filter ** l2))
    return ins


def _linear_numel(irreps_in, irreps_out):
    """e3nn o3.Linear weight numel: mul_in * mul_out per equal (l, p) pair."""
    return sum(mi * mo for mi, li, pi in irreps_in for mo, lo, po in irreps_out
               if (li, pi) == (lo, po))


def _bias_numel(irreps_out):
    """e3nn o3.Linear(biases=True): a bias per channel of every 0e output
    irrep (``biases and ir.is_scalar()``)"""
    return sum(m for m, l, p in irreps_out if (l, p) == (0, 1))


def act_norm(name):
    """e3nn normalize2mom(act): 1 / sqrt(E[act(z)^2]) over e3nn's fixed
    sample (1e6 float64 normals from a CPU generator seeded 0) -- reproduces
    the frozen constants of the reference deployments (silu 1.6791767923989418,
    tanh 1.5937334472592695)"""
    f = {'relu': torch.relu, 'silu': torch.nn.functional.silu, 'tanh': torch.tanh,
         'sigmoid': torch.sigmoid, 'abs': torch.abs, 'elu': torch.nn.functional.elu}.get(name)
    if f is None:
        raise ValueError(f'activation {name!r} (reference _const.ACTIVATION: relu silu tanh abs '
                         'ssp sigmoid elu; ssp is not built)')
    gen = torch.Generator(device='cpu').manual_seed(0)
    z = torch.randn(1_000_000, generator=gen, dtype=torch.float64)
    c = float(f(z).pow(2).mean().pow(-0.5))
    return 1.0 if abs(c - 1.0) < 1e-4 else c


def model_manifest(cfg):
    """The deployment manifest (parameter table in the reference's
    named_parameters order) of a resolved config."""
    irreps = cfg['_irreps']
    L = int(cfg['num_convolution_layer'])
    nsp = cfg['_number_of_species']
    nb = int(cfg['radial_basis'].get('bessel_basis_num', 8))
    hid = [int(h) for h in cfg['weight_nn_hidden_neurons']]
    parity = -1 if cfg['is_parity'] else 1
    sc_type = cfg['self_connection_type']
    if sc_type not in ('linear', 'nequip'):
        # the reference accepts exactly these (_const.py:13 IMPLEMENTED_SELF_CONNECTION_TYPE,
        # checked at :153 / :207); 'none' passes init_self_connection (model_build.py:48)
        # but its interaction block then calls the missing intro (interaction_blocks.py:44-49)
        raise ValueError(f'self_connection_type {sc_type!r}: the reference implements '
                         "'nequip' and 'linear' only (sevenn/_const.py IMPLEMENTED_SELF_CONNECTION_TYPE)")
    bias = bool(cfg['use_bias_in_linear'])
    fcn = bool(cfg['readout_as_fcn'])
    tensors = []

    def add(name, shape):
        tensors.append({'name': name, 'shape': list(shape)})

    def add_linear(name, irreps_in, irreps_out, biases=bias):
        """e3nn o3.Linear's parameters in registration order: the flat
        weight, then (biases=True) one bias per scalar 0e output channel,
        zero-initialised (IrrepsLinear(..., biases=use_bias_in_linear),
        model_build.py:194, :237, :386, :393; interaction_blocks.py:58, :80)"""
        add(f'{name}.linear.weight', [_linear_numel(irreps_in, irreps_out)])
        nbias = _bias_numel(irreps_out) if biases else 0
        if nbias:
            add(f'{name}.linear.bias', [nbias])
    add('edge_embedding.basis_function.coeffs', [nb])
    add_linear('onehot_to_feature_x', [(nsp, 0, 1)], irreps[0])
    conv_out = []
    for t in range(L):
        last = t == L - 1
        xin, xout = irreps[t], irreps[t + 1]
        gin = _gate_irreps(xout)
        # the convolution's output irreps (model_build.py:303-315): the full
        # tensor product's, l <= lmax_node, scalars 0e only in the last block
        # -- irreps_manual sets only the block's node irreps; sevenn < 0.9
        # built the convolution on irreps_manual (config key
        # '_conv_irreps_manual': True; the 0.8.6 HfO2 example deployment)
        if cfg.get('_conv_irreps_manual', False):
            tp_out = xout
        else:
            tp_out = infer_irreps_out(xin, cfg['_lmax_edge'], parity,
                                      0 if last else cfg['_lmax_node'],
                                      'even' if last else 'full', False)
        conv_out.append(_irreps_str(tp_out))
        ins = _conv_instructions(xin, cfg['_lmax_edge'], parity, tp_out)
        mid = {}
        for mul, _, _, l3, p3 in ins:
            mid[(l3, p3)] = mid.get((l3, p3), 0) + mul
        mid_irreps = [(m, l, p) for (l, p), m in sorted(mid.items())]
        W = sum(i[0] for i in ins)
        if sc_type == 'linear':   # SelfConnectionLinearIntro: o3.Linear without biases
            add_linear(f'{t}_self_connection_intro', xin, gin, biases=False)
        else:   # FullyConnectedTensorProduct(x, nsp x 0e -> gin), self_connection.py:11-38
            add(f'{t}_self_connection_intro.fc_tensor_product.weight',
                [_linear_numel(xin, gin) * nsp])
        add_linear(f'{t}_self_interaction_1', xin, xin)
        add(f'{t}_convolution.denominator', [1])
        dims = [nb] + hid + [W]
        for k in range(len(dims) - 1):
            add(f'{t}_convolution.weight_nn.layer{k}.weight', [dims[k], dims[k + 1]])
        add_linear(f'{t}_self_interaction_2', mid_irreps, gin)
    hidden = sum(m for m, l, p in irreps[-1] if (l, p) == (0, 1)) // 2
    readout = {'type': 'linear'}
    if fcn:
        # FCN_e3nn (nn/linear.py:94-129): e3nn FullyConnectedNet([dim] + hidden
        # + [1], act) on the last block's scalars (model_build.py:396-408)
        if any(l != 0 for _, l, _ in irreps[-1]):
            raise ValueError('readout_as_fcn: the last block must output scalars only')
        rh = [int(h) for h in cfg['readout_fcn_hidden_neurons']]
        ract = str(cfg['readout_fcn_activation'])
        fdims = [_dim(irreps[-1])] + rh + [1]
        for k in range(len(fdims) - 1):
            add(f'readout_FCN.fcn.layer{k}.weight', [fdims[k], fdims[k + 1]])
        readout = {'type': 'fcn', 'hidden': rh, 'act': ract, 'act_norm': act_norm(ract)}
    else:
        add_linear('reduce_input_to_hidden', irreps[-1], [(hidden, 0, 1)])
        add_linear('reduce_hidden_to_energy', [(hidden, 0, 1)], [(1, 0, 1)])
    add('rescale_atomic_energy.shift', [nsp])
    add('rescale_atomic_energy.scale', [nsp])
    off = 0
    for t in tensors:
        t['numel'] = int(np.prod(t['shape']))
        t['offset'] = off
        off += t['numel']
    cf = cfg['cutoff_function']
    cname = cf.get('cutoff_function_name', 'poly_cut')
    cutoff_function = {'name': cname}
    if cname == 'XPLOR':
        cutoff_function['cutoff_on'] = float(cf.get('cutoff_on', 4.5))
    elif cname == 'poly_cut':
        cutoff_function['p'] = float(cf.get('poly_cut_p_value', 6))
    man = {
        'format': FORMAT,
        'model_type': 'E3_equivariant_model',
        'source_version': BUILD_VERSION,
        'source_time': datetime.date.today().isoformat(),
        'dtype': 'single',
        'num_species': nsp,
        'chemical_symbols': list(cfg['chemical_species']),
        'cutoff': float(cfg['cutoff']),
        'cutoff_function': cutoff_function,
        'radial_basis': {'name': 'bessel', 'num': nb},
        'lmax': int(cfg['lmax']),
        'is_parity': bool(cfg['is_parity']),
        'channel': int(cfg['channel']),
        'num_convolution_layer': L,
        'irreps_manual': [_irreps_str(ir) for ir in irreps],
        'conv_irreps_out': conv_out,
        'weight_nn_hidden_neurons': hid,
        'act_radial': 'silu',
        'act_scalar': {'e': 'silu', 'o': 'tanh'}, 'act_gate': {'e': 'silu', 'o': 'tanh'},
        'act_norm': {'silu': SILU_NORM, 'tanh': TANH_NORM},
        'silu_norm': SILU_NORM,
        'sh_normalize': bool(cfg['_normalize_sph']),
        'lmax_edge': int(cfg['_lmax_edge']),
        'readout_hidden': hidden,
        'self_connection_type': sc_type,
        'use_bias_in_linear': bias,
        'readout': readout,
        'conv_denominator': cfg['_conv_denominator'],
        'species_wise_rescale': True,
        'num_params': off,
        'tensors': tensors,
    }
    # the same predicate routes the deployment (model.load_model)
    from .nn import sevennet0_kinds
    man['family'] = 'sevennet0' if sevennet0_kinds(man) is not None else 'nequip'
    return man


def _check_kernel_support(man):
    """What the HIP paths serve: SevenNet-0's architecture on its specialised
    kernels (csrc/tp.h, fused.hip; also the native engine e3gnn_load), every
    other nequip-family model on the runtime path tables (gtp.hip), which take
    l <= 2."""
    irreps = [_parse(s) for s in man['irreps_manual']]
    if max(l for ir in irreps for _, l, _ in ir) > 2 or int(man['lmax']) > 2:
        raise NotImplementedError('irreps with l > 2: the coupling tables stop at l = 2')
    if man['cutoff_function']['name'] not in ('XPLOR', 'poly_cut'):
        raise NotImplementedError(f"cutoff function {man['cutoff_function']['name']!r}")


def init_weights(man, cfg, seed=0):
    """e3nn's initialisation: Linear and FullyConnectedNet weights N(0, 1)
    (normalisation is applied in the forward), Bessel coefficients n pi / rc
    (edge_embedding.py:105-110), denominators, species-wise shift / scale."""
    g = np.random.default_rng(seed)
    flat = np.empty(man['num_params'], dtype=np.float32)
    rc = float(man['cutoff'])
    nsp = man['num_species']
    den = man['conv_denominator']

    def per_species(v):
        a = np.asarray(v, dtype=np.float64).reshape(-1)
        return np.full(nsp, a[0]) if a.size == 1 else a
    for t in man['tensors']:
        n, o = t['numel'], t['offset']
        name = t['name']
        if name == 'edge_embedding.basis_function.coeffs':
            v = np.arange(1, n + 1) * math.pi / rc
        elif name.endswith('.linear.bias'):   # e3nn: zeros
            v = np.zeros(n)
        elif name.endswith('.denominator'):
            v = np.array([den[int(name.split('_')[0])]])
        elif name == 'rescale_atomic_energy.shift':
            v = per_species(cfg['shift'])
        elif name == 'rescale_atomic_energy.scale':
            v = per_species(cfg['scale'])
        else:
            v = g.standard_normal(n)
        flat[o:o + n] = np.asarray(v, dtype=np.float32).reshape(-1)
    return flat


def build_E3_equivariant_model(config, parallel=False, device='cuda', seed=0, dtype=None):
    """model_build.py:186 for this build -> nn.SevenNetTrainable."""
    from .nn import SevenNetTrainable
    cfg = resolve_config(config)
    man = model_manifest(cfg)
    _check_kernel_support(man)
    flat = init_weights(man, cfg, seed)
    kw = {} if dtype is None else {'dtype': dtype}
    model = SevenNetTrainable(device=device, manifest=man, weights=flat,
                              train_shift_scale=bool(cfg['train_shift_scale']),
                              train_denominator=bool(cfg['train_denominator']), **kw)
    model.config = cfg
    return model


def load_state_dict(model, state_dict, strict=True):
    """Copy a reference-named state dict into the model's flat buffer."""
    missing = [n for n in model.slices if n not in state_dict]
    unused = [k for k in state_dict if k not in model.slices]
    if strict and (missing or unused):
        raise KeyError(f'state dict mismatch: missing {missing}, unused {unused}')
    with torch.no_grad():
        for name, (off, n, shape) in model.slices.items():
            if name in state_dict:
                v = torch.as_tensor(state_dict[name]).reshape(-1)
                if v.numel() != n:
                    raise ValueError(f'{name}: {v.numel()} values, model has {n}')
                model.flat[off:off + n].copy_(v.to(model.flat.dtype))
    return missing, unused


def _patch_old_config(config):
    """util.py:130-146, the old-checkpoint fixes: XPLOR configs lose a stray
    ``poly_cut_p_value``; ``train_avg_num_neigh`` is the old name of
    ``train_denominator``; ``optimize_by_reduce: False`` checkpoints are
    refused; a missing ``conv_denominator`` is 0.0 (the trained denominator
    comes from the state dict); a missing ``_normalize_sph`` means the raw
    edge vector went into the spherical harmonics (sevenn < 0.9, e.g.
    SevenNet-0 22May2024 and the 0.8.6 HfO2 example)."""
    cf = config.get('cutoff_function')
    if isinstance(cf, dict) and cf.get('cutoff_function_name') == 'XPLOR':
        cf = dict(cf)
        cf.pop('poly_cut_p_value', None)
        config['cutoff_function'] = cf
    if 'train_denominator' not in config:
        config['train_denominator'] = config.pop('train_avg_num_neigh', False)
    if config.pop('optimize_by_reduce', None) is False:
        raise ValueError('This checkpoint(optimize_by_reduce: False) is no longer supported')
    if 'conv_denominator' not in config:
        config['conv_denominator'] = 0.0
    if '_normalize_sph' not in config:
        config['_normalize_sph'] = False
    return config


def _map_old_model(state_dict):
    """util.py:149-183: module names before the reference's 240501 rename
    ('0 convolution.x' -> '0_convolution.x', 'EdgeEmbedding' ->
    'edge_embedding', ..., 'denumerator' -> 'denominator')."""
    names = {'EdgeEmbedding': 'edge_embedding',
             'reducing nn input to hidden': 'reduce_input_to_hidden',
             'reducing nn hidden to energy': 'reduce_hidden_to_energy',
             'rescale atomic energy': 'rescale_atomic_energy'}
    for i in range(10):
        for old, new in (('self connection intro', 'self_connection_intro'),
                         ('convolution', 'convolution'),
                         ('self interaction 2', 'self_interaction_2'),
                         ('equivariant gate', 'equivariant_gate')):
            names[f'{i} {old}'] = f'{i}_{new}'
    out = {}
    for k, v in state_dict.items():
        head, _, rest = k.partition('.')
        rest = rest.replace('denumerator', 'denominator')
        out[f'{names[head]}.{rest}' if head in names else k] = v
    return out


def model_from_checkpoint(checkpoint, device='cuda'):
    """util.py:186-231: ``{'model_state_dict': ..., 'config': ...}`` (or the
    path of one, read weights-only) -> (model, config).  Old configs are
    patched first (``_patch_old_config``) and old module names mapped when
    keys are missing (``_map_old_model``), as the reference does."""
    if isinstance(checkpoint, str):
        checkpoint = torch.load(checkpoint, map_location='cpu', weights_only=True)
    elif not isinstance(checkpoint, dict):
        raise ValueError('checkpoint must be either str or dict')
    config = {k: (v.cpu().tolist() if torch.is_tensor(v) else v)
              for k, v in checkpoint['config'].items()}
    config = _patch_old_config(config)
    model = build_E3_equivariant_model(config, device=device)
    sd = checkpoint['model_state_dict']
    missing, _ = load_state_dict(model, sd, strict=False)
    if missing:
        missing, _ = load_state_dict(model, _map_old_model(sd), strict=False)
    assert len(missing) == 0, f'Missing keys: {missing}'
    return model, model.config


def checkpoint_of(model):
    """The reference checkpoint layout of a model: state dict + config."""
    sd = {n: model.flat[o:o + k].detach().cpu().clone().view(shape)
          for n, (o, k, shape) in model.slices.items()}
    # the user-level keys plus the two underscore keys that change the
    # architecture: '_normalize_sph' (model_from_checkpoint reads its absence as
    # a pre-0.9 checkpoint) and '_conv_irreps_manual' (the convolution built on
    # irreps_manual, the sevenn 0.8.6 layout); the keys resolve_config derives
    # are recomputed on load
    derived = ('_irreps', '_lmax_edge', '_lmax_node', '_conv_denominator')
    kept = ('_normalize_sph', '_conv_irreps_manual')
    cfg = {k: v for k, v in getattr(model, 'config', {}).items()
           if (not k.startswith('_') or k in kept) and k not in derived}
    if not cfg:
        raise ValueError('model has no config (build it with build_E3_equivariant_model)')
    return {'model_state_dict': sd, 'config': cfg}


def deploy(model, out_dir):
    """scripts/deploy.py:15-117: parameters -> weights.bin + manifest.json
    (metadata of the reference's _extra_files incl. comm_size).  Returns
    out_dir."""
    man = json.loads(json.dumps(model.manifest))
    flat = model.flat.detach().float().cpu().numpy().astype('<f4')
    off = 0
    for t in man['tensors']:
        o, n, _ = model.slices[t['name']]
        if o != off:
            raise RuntimeError('parameter table is not contiguous')
        off += n
    if off != flat.size:
        raise RuntimeError('parameter count mismatch')
    irreps = [_parse(s) for s in man['irreps_manual']]
    man['comm_size'] = max(_dim(ir) for ir in irreps[1:-1]) if len(irreps) > 2 else _dim(irreps[0])
    man['deploy_time'] = datetime.datetime.now().strftime('%Y-%m-%d')
    man['deployed_by'] = BUILD_VERSION
    os.makedirs(out_dir, exist_ok=True)
    tmp = os.path.join(out_dir, 'weights.bin.tmp')
    flat.tofile(tmp)
    os.replace(tmp, os.path.join(out_dir, 'weights.bin'))
    with open(os.path.join(out_dir, 'manifest.json'), 'w') as f:
        json.dump(man, f, indent=1)
    return out_dir


deploy_parallel = deploy  # one deployment serves the segment API (comm_size in the manifest)


def deploy_config(config, out_dir, seed=0):
    """A config straight to a deployment (weights.bin + manifest.json) with
    e3nn's initialisation (``init_weights``), without building the trainable
    model: what ``deploy(build_E3_equivariant_model(config))`` writes, for
    hosts and benchmarks that only serve the model (no GPU needed to write it)."""
    cfg = resolve_config(config)
    man = model_manifest(cfg)
    _check_kernel_support(man)
    flat = init_weights(man, cfg, seed).astype('<f4')
    irreps = [_parse(s) for s in man['irreps_manual']]
    man['comm_size'] = max(_dim(ir) for ir in irreps[1:-1]) if len(irreps) > 2 else _dim(irreps[0])
    man['deploy_time'] = datetime.datetime.now().strftime('%Y-%m-%d')
    man['deployed_by'] = BUILD_VERSION
    os.makedirs(out_dir, exist_ok=True)
    tmp = os.path.join(out_dir, 'weights.bin.tmp')
    flat.tofile(tmp)
    os.replace(tmp, os.path.join(out_dir, 'weights.bin'))
    with open(os.path.join(out_dir, 'manifest.json'), 'w') as f:
        json.dump(man, f, indent=1)
    return out_dir


def sevennet_shaped_config(channel, num_convolution_layer, species=None, avg_num_neigh=28.0):
    """The SevenNet-0 preset (sevenn/presets/sevennet-0.yaml: lmax 2, even
    parity, XPLOR 4.5-5.0 A, 8 Bessel functions, a 64-64 radial MLP, linear
    self-connection) without its irreps_manual: ``channel`` x (0e+1e+2e) per
    block, ``num_convolution_layer`` blocks (model_build.py:196-372)."""
    return {'chemical_species': species or ['Cl', 'Li', 'P', 'S', 'Si'], 'cutoff': 5.0,
            'channel': channel, 'is_parity': False, 'lmax': 2,
            'num_convolution_layer': num_convolution_layer,
            'weight_nn_hidden_neurons': [64, 64],
            'radial_basis': {'radial_basis_name': 'bessel', 'bessel_basis_num': 8},
            'cutoff_function': {'cutoff_function_name': 'XPLOR', 'cutoff_on': 4.5},
            'act_gate': {'e': 'silu', 'o': 'tanh'}, 'act_scalar': {'e': 'silu', 'o': 'tanh'},
            'conv_denominator': float(avg_num_neigh), 'self_connection_type': 'linear',
            'train_shift_scale': False, 'train_denominator': False}
