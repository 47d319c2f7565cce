"""Export SevenNet-0 parameters into this build's deploy format.

Runs in the build container only (reads /root/reference, which never travels
to the GPU box).  Output: ``sevennet_finetuning_amd/assets/sevennet0/``
``weights.bin`` (little-endian fp32, tensors back to back) + ``manifest.json``
(model config + tensor table).  This replaces the reference's TorchScript
``_extra_files`` + frozen constants (sevenn/scripts/deploy.py:15-51).

Sources (both loaded with loaders that execute nothing from the file):
* named parameters: example_inputs/fine_tuning/estimate_Fisher/
  opt_params_sevenn.pt via ``torch.load(weights_only=True)`` -- bit-identical
  to the frozen deployment constants;
* deployment metadata: the plain-text ``extra/*`` members of
  serial_model/deployed_serial.pt read with ``zipfile`` (deploy.py:34-51).
"""
import json
import os
import sys
import zipfile

import numpy as np
import torch

REF = '/root/reference'
PARAMS = f'{REF}/example_inputs/fine_tuning/estimate_Fisher/opt_params_sevenn.pt'
SERIAL = (f'{REF}/sevenn/pretrained_potentials/SevenNet_0__11July2024/'
          'serial_model/deployed_serial.pt')
OUT = os.path.join(os.path.dirname(__file__), '..', 'sevennet_finetuning_amd',
                   'assets', 'sevennet0')

# e3nn normalize2mom(silu): 1/sqrt(E[silu(z)^2]) estimated by e3nn from 1e6
# float64 N(0,1) samples of a CPU generator seeded 0 (reproduced exactly here;
# equals the frozen constant c5 of serial_code.py).
SILU_NORM = 1.6791767923989418


def main():
    params = torch.load(PARAMS, weights_only=True, map_location='cpu')
    z = zipfile.ZipFile(SERIAL)
    extra = {n.rsplit('/', 1)[1]: z.read(n).decode()
             for n in z.namelist() if '/extra/' in n}
    symbols = extra['chemical_symbols_to_index'].split()
    assert len(symbols) == int(extra['num_species'])

    tensors, blobs, off = [], [], 0
    for name, t in params.items():
        a = t.detach().cpu().numpy().astype('<f4')
        tensors.append({'name': name, 'shape': list(a.shape), 'offset': off,
                        'numel': int(a.size)})
        blobs.append(a.ravel())
        off += a.size
    flat = np.concatenate(blobs)
    denoms = [float(params[f'{t}_convolution.denominator'][0]) for t in range(5)]

    manifest = {
        'format': 'e3gnn-mi355x/1',
        'model_type': extra['model_type'],
        'source_version': extra['version'],
        'source_time': extra['time'],
        'dtype': extra['dtype'],
        'num_species': len(symbols),
        'chemical_symbols': symbols,
        'cutoff': float(extra['cutoff']),
        'cutoff_function': {'name': 'XPLOR', 'cutoff_on': 4.5},
        'radial_basis': {'name': 'bessel', 'num': 8},
        'lmax': 2,
        'is_parity': False,
        'channel': 128,
        'num_convolution_layer': 5,
        'irreps_manual': ['128x0e'] + ['128x0e+64x1e+32x2e'] * 4 + ['128x0e'],
        'weight_nn_hidden_neurons': [64, 64],
        'act_radial': 'silu', 'act_scalar': 'silu', 'act_gate': 'silu',
        'silu_norm': SILU_NORM,
        'self_connection_type': 'linear',
        'conv_denominator': denoms,
        'species_wise_rescale': True,
        'num_params': int(flat.size),
        'tensors': tensors,
    }
    os.makedirs(OUT, exist_ok=True)
    flat.tofile(os.path.join(OUT, 'weights.bin'))
    with open(os.path.join(OUT, 'manifest.json'), 'w') as f:
        json.dump(manifest, f, indent=1)
    print(f'wrote {flat.size} params ({flat.nbytes/1e6:.2f} MB) to {OUT}')


if __name__ == '__main__':
    sys.exit(main())
