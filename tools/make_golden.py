"""Write the reference-derived fixtures under tests/golden/ (build container only).

* hfo2_resdat.npz   -- positions/cell/species of the reference's example input
                       example_inputs/md_serial_example/res.dat (LAMMPS data
                       file, parsed as text).
* kat_reference.json -- known-answer values measured by the survey with the
                       reference's frozen SevenNet-0 model.
* cg_frozen.npz     -- see tools/extract_cg_frozen.py.
"""
import json
import os

import numpy as np

REF = '/root/reference'
GOLD = os.path.join(os.path.dirname(__file__), '..', 'tests', 'golden')


def parse_lammps_data(path):
    lines = open(path).read().split('\n')

    def grab(key):
        for line in lines:
            if key in line:
                return line.split()
    xl, yl, zl, tl = grab('xlo xhi'), grab('ylo yhi'), grab('zlo zhi'), grab('xy xz yz')
    lx = float(xl[1]) - float(xl[0])
    ly = float(yl[1]) - float(yl[0])
    lz = float(zl[1]) - float(zl[0])
    xy, xz, yz = map(float, tl[:3])
    cell = np.array([[lx, 0, 0], [xy, ly, 0], [xz, yz, lz]])
    natom = int(grab(' atoms')[0])
    start = [i for i, line in enumerate(lines) if line.strip() == 'Atoms'][0] + 2
    rows = [line.split() for line in lines[start:start + natom]]
    typ = np.array([int(r[1]) for r in rows])
    pos = np.array([[float(v) for v in r[2:5]] for r in rows])
    return pos, cell, typ


def main():
    pos, cell, typ = parse_lammps_data(f'{REF}/example_inputs/md_serial_example/res.dat')
    symbols = np.array(['Hf' if t == 1 else 'O' for t in typ])
    np.savez(os.path.join(GOLD, 'hfo2_resdat.npz'), pos=pos, cell=cell, symbols=symbols)
    kat = {
        'source': ('SURVEY.md section 8c: values measured in the survey container by '
                   "running the reference's own frozen SevenNet-0 deployment "
                   '(serial_model/deployed_serial.pt, fp32 CPU). Full periodic '
                   'neighbor list, r < 5.0 A, i != j or non-zero image.'),
        'kats': [
            {'name': 'si_perfect_1x1x1', 'cells': [1, 1, 1], 'displace': False,
             'n_edges': 224, 'energy': -43.206638, 'stress_diag': 0.011943,
             'max_abs_force': 3.4e-6},
            {'name': 'si_rng0_2x2x1', 'cells': [2, 2, 1], 'displace': True,
             'n_edges': 896, 'energy': -171.709259},
            {'name': 'si_rng0_3x3x3', 'cells': [3, 3, 3], 'displace': True,
             'n_edges': 6048, 'energy': -1158.691895},
            {'name': 'hfo2_resdat', 'n_edges': 4274, 'energy': -972.006409},
        ],
    }
    with open(os.path.join(GOLD, 'kat_reference.json'), 'w') as f:
        json.dump(kat, f, indent=1)


if __name__ == '__main__':
    main()
