"""NVE energy drift of the native MD host (native/e3gnn_md, velocity Verlet
over the C ABI) for the shipped fused kernels against reference force fields
of the same model: the generic engine (E3GNN_GENERIC=1: independent f32
kernels, plain f32 radial-MLP GEMMs, forces the exact gradient of its energy
to f32 rounding) and, when present, an in-tree variant library built with the
six-product backward (E3GNN_DH2_X3=0 E3GNN_BWD_W_X3=0
E3GNN_CHAIN_X3=0).

    python tools/nve_drift.py [--cells 3] [--steps 2000] [--dt 1.0] [--temp 600]
                              [--variant sevennet_finetuning_amd/variants/six.so]

Prints one JSON line per run: drift = least-squares slope of the total energy
per atom (meV/atom/ps), max |E_tot - E_tot(0)| per atom (meV), the detrended
fluctuation, and the mean device time per step."""
import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, 'native', 'e3gnn_md')
ASSET = os.path.join(ROOT, 'sevennet_finetuning_amd', 'assets', 'sevennet0')


def run(cells, steps, dt, temp, seed=0, env=None, exe=EXE, timeout=600):
    r = subprocess.run([exe, os.path.join(ASSET, 'weights.bin'), os.path.join(ASSET, 'manifest.json'),
                        str(cells), str(steps), str(dt), str(temp), str(seed)],
                       capture_output=True, text=True, timeout=timeout,
                       env=dict(os.environ, **(env or {})))
    if r.returncode != 0:
        raise RuntimeError(r.stderr)
    return [json.loads(line) for line in r.stdout.splitlines() if line.startswith('{')]


def drift_stats(rows, dt):
    n = rows[0]['n_atoms']
    et = np.array([r['etot'] for r in rows], dtype=np.float64) / n
    t = np.arange(len(et)) * dt * 1e-3          # ps
    slope, icpt = np.polyfit(t, et, 1)
    resid = et - (slope * t + icpt)
    return {'n_atoms': n, 'steps': len(rows) - 1, 'dt_fs': dt,
            'drift_meV_per_atom_ps': float(slope * 1e3),
            'max_dev_meV_per_atom': float(np.abs(et - et[0]).max() * 1e3),
            'fluct_meV_per_atom': float(resid.std() * 1e3),
            'ekin_final_eV': rows[-1]['ekin'], 'epot_0_eV': rows[0]['epot'],
            'device_ms_mean': float(np.mean([r['device_ms'] for r in rows]))}


def variant_exe(lib):
    """e3gnn_md against another build of the library: the binary resolves
    libe3gnn_hip.so through its $ORIGIN/../sevennet_finetuning_amd rpath, so a
    copy in a scratch tree next to the variant is what runs"""
    d = tempfile.mkdtemp()
    os.makedirs(os.path.join(d, 'native'))
    os.makedirs(os.path.join(d, 'sevennet_finetuning_amd'))
    shutil.copy(EXE, os.path.join(d, 'native', 'e3gnn_md'))
    shutil.copy(lib, os.path.join(d, 'sevennet_finetuning_amd', 'libe3gnn_hip.so'))
    return os.path.join(d, 'native', 'e3gnn_md')


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--cells', type=int, default=3)
    ap.add_argument('--steps', type=int, default=2000)
    ap.add_argument('--dt', type=float, default=1.0)
    ap.add_argument('--temp', type=float, default=600.0)
    ap.add_argument('--seeds', default='0')
    ap.add_argument('--variant', default=os.path.join(ROOT, 'sevennet_finetuning_amd', 'variants', 'six.so'))
    ap.add_argument('--label', default='six_product', help='name of the variant leg')
    a = ap.parse_args()
    legs = [('shipped', None, EXE), ('generic_f32', {'E3GNN_GENERIC': '1'}, EXE)]
    if os.path.exists(a.variant):
        legs.append((a.label, None, variant_exe(a.variant)))
    for seed in [int(s) for s in a.seeds.split(',')]:
        for name, env, exe in legs:
            st = drift_stats(run(a.cells, a.steps, a.dt, a.temp, seed, env, exe), a.dt)
            print(json.dumps({'leg': name, 'seed': seed, 'temp_K': a.temp, **st}), flush=True)


if __name__ == '__main__':
    sys.exit(main())
