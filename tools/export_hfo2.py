"""Export the reference's HfO2 example deployment into this build's deploy
format (``sevennet_finetuning_amd/assets/hfo2_example/``).

Runs in the build container only (reads /root/reference, which never travels
to the GPU box).  Source: ``example_inputs/md_serial_example/deployed_serial.pt``
(sevenn 0.8.6, species "Hf O", rc 4.0).  Nothing from the archive is executed
or unpickled: the constant tensors are read by ``tools/frozen_constants.py``
(a pickle-opcode parser over ``constants.pkl`` + the raw storages) and the
metadata from the plain-text ``extra/*`` members.  The archive has no named
parameters, so the constant -> parameter map below was read off its frozen code
(``code/__torch__/sevenn/nn/sequential/___torch_mangle_185.py``, studied as
text):

* the model is the reference's ``nequip`` family (model_build.py:186-445,
  interaction_blocks.py:22-86): 4 interaction blocks, channel 4, lmax 1,
  is_parity, 8 Bessel functions x PolynomialCutoff(p = 6)
  (edge_embedding.py:119-145), spherical harmonics of the UNnormalised edge
  vector (sevenn 0.8.6 checkpoints have no ``_normalize_sph``; util.py:143-144),
  SelfConnectionIntro = FullyConnectedTensorProduct(x, one-hot)
  (self_connection.py:11-38), gate scalars silu (even) / tanh (odd), scalar
  shift/scale (Rescale, scale.py:12-40);
* irreps 4x0e -> 4x0e+4x1o -> 4x0e+4x1o+4x1e -> 4x0o+4x0e+4x1o+4x1e (x2): in
  0.8.6 the last block keeps the full irreps (the readout linear takes its 4x0e);
  convolution instructions = every (x, filter, out) with out in the block's
  output irreps (convolution.py:72-95), so W = 8, 20, 32, 40;
* e3nn's code generator folds the path weight 1/sqrt(fan_in) into the frozen
  constant of some linear blocks (the l > 0 blocks of every IrrepsLinear, both
  readout linears) and multiplies the input by it in others; the folded ones
  are divided back here, so ``weights.bin`` holds reference-convention
  (unscaled) parameters and the consumers apply the path weights themselves
  (the same convention as the SevenNet-0 assets).  The radial MLP constants
  are W/sqrt(fan_in) as in every e3nn FullyConnectedNet freeze.

usage: python tools/export_hfo2.py
"""
import json
import math
import os
import sys
import zipfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from frozen_constants import frozen_constants  # noqa: E402

REF = '/root/reference'
SERIAL = f'{REF}/example_inputs/md_serial_example/deployed_serial.pt'
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'sevennet_finetuning_amd',
                   'assets', 'hfo2_example')

IRREPS = ['4x0e', '4x0e+4x1o', '4x0e+4x1o+4x1e', '4x0o+4x0e+4x1o+4x1e',
          '4x0o+4x0e+4x1o+4x1e']
R8, R12, R2 = 1 / math.sqrt(8), 1 / math.sqrt(12), 1 / math.sqrt(2)


def main():
    c = frozen_constants(SERIAL)
    z = zipfile.ZipFile(SERIAL)
    extra = {n.rsplit('/', 1)[-1]: z.read(n).decode()
             for n in z.namelist() if '/extra/' in n}
    symbols = extra['chemical_symbols_to_index'].split()
    nsp = int(extra['num_species'])
    assert symbols == ['Hf', 'O'] and nsp == 2
    cut = float(extra['cutoff'])

    def raw(k):
        return c[k].astype(np.float32)

    def unfold(k, alpha):   # constant = alpha * W  ->  W
        return (c[k].astype(np.float64) / alpha).astype(np.float32)

    def cat(*a):
        return np.concatenate([x.reshape(-1) for x in a])

    t = []   # (name, array) in the reference's named_parameters() order

    t.append(('edge_embedding.basis_function.coeffs', raw(0)))
    t.append(('onehot_to_feature_x.linear.weight', raw(1).reshape(-1)))
    # per block: SC intro (FCTP weights per instruction [mul_x, nsp, mul_out]),
    # si1, denominator, radial MLP (frozen W/sqrt(fan_in)), si2
    blocks = [
        dict(sc=[3], si1=cat(raw(4)), mlp=(5, 7, 8), si2=cat(raw(10), unfold(11, 0.5))),
        dict(sc=[12, 13], si1=cat(raw(14), unfold(15, 0.5)), mlp=(16, 17, 18),
             si2=cat(raw(20), unfold(21, R8), unfold(22, 0.5))),
        dict(sc=[23, 24, 25], si1=cat(raw(26), unfold(27, 0.5), unfold(28, 0.5)),
             mlp=(29, 30, 31),
             si2=cat(raw(32), raw(33), unfold(34, R12), unfold(35, R8))),
        dict(sc=[37, 38, 39, 40],
             si1=cat(raw(41), raw(42), unfold(43, 0.5), unfold(44, 0.5)), mlp=(45, 46, 47),
             si2=cat(raw(48), raw(49), unfold(50, R12), unfold(51, R12))),
    ]
    den = float(c[9][0])
    for i, b in enumerate(blocks):
        t.append((f'{i}_self_connection_intro.fc_tensor_product.weight',
                  cat(*[raw(k) for k in b['sc']])))
        t.append((f'{i}_self_interaction_1.linear.weight', b['si1']))
        t.append((f'{i}_convolution.denominator', np.array([den], np.float32)))
        k0, k1, k2 = b['mlp']
        for k, (kk, fan) in enumerate(((k0, 8), (k1, 64), (k2, 64))):
            t.append((f'{i}_convolution.weight_nn.layer{k}.weight',
                      (c[kk].astype(np.float64) * math.sqrt(fan)).astype(np.float32)))
        t.append((f'{i}_self_interaction_2.linear.weight', b['si2']))
    t.append(('reduce_input_to_hidden.linear.weight', unfold(52, 0.5).reshape(-1)))
    t.append(('reduce_hidden_to_energy.linear.weight', unfold(53, R2).reshape(-1)))
    t.append(('rescale_atomic_energy.shift', np.full(nsp, c[55][0], np.float32)))
    t.append(('rescale_atomic_energy.scale', np.full(nsp, c[54][0], np.float32)))

    tensors, off, flat = [], 0, []
    for name, a in t:
        a = np.ascontiguousarray(a, dtype='<f4')
        shape = list(a.shape) if 'weight_nn' in name else [a.size]
        tensors.append({'name': name, 'shape': shape, 'offset': off, 'numel': int(a.size)})
        flat.append(a.reshape(-1))
        off += a.size
    man = {
        'format': 'e3gnn-mi355x/1',
        'model_type': extra['model_type'],
        'family': 'nequip',
        'source_version': extra['version'],
        'source_time': extra['time'],
        'dtype': extra['dtype'],
        'num_species': nsp,
        'chemical_symbols': symbols,
        'cutoff': cut,
        'cutoff_function': {'name': 'poly_cut', 'p': 6.0},
        'radial_basis': {'name': 'bessel', 'num': 8},
        'lmax': 1,
        'is_parity': True,
        'channel': 4,
        'num_convolution_layer': 4,
        'irreps_manual': IRREPS,
        'weight_nn_hidden_neurons': [64, 64],
        'act_radial': 'silu',
        'act_scalar': {'e': 'silu', 'o': 'tanh'},
        'act_gate': {'e': 'silu', 'o': 'tanh'},
        # e3nn normalize2mom constants as frozen (c6, c36)
        'act_norm': {'silu': float(c[6]), 'tanh': float(c[36])},
        'silu_norm': float(c[6]),
        'sh_normalize': False,
        'self_connection_type': 'nequip',
        'conv_denominator': [den] * 4,
        'readout_hidden': 2,
        'species_wise_rescale': False,
        'num_params': int(off),
        'tensors': tensors,
    }
    os.makedirs(OUT, exist_ok=True)
    np.concatenate(flat).astype('<f4').tofile(os.path.join(OUT, 'weights.bin'))
    with open(os.path.join(OUT, 'manifest.json'), 'w') as f:
        json.dump(man, f, indent=1)
    # the frozen w3j(1,1,1) table (c19) pins the oracle's CG sign convention
    np.savez(os.path.join(os.path.dirname(OUT), '..', '..', 'tests', 'golden',
                          'hfo2_frozen_w3j111.npz'), w3j_111=c[19])
    print(f'wrote {OUT}: {off} parameters')


if __name__ == '__main__':
    main()
