"""Extract the frozen CG tables of the reference deployment as a fixture.

Build-container only.  Reads the raw little-endian float32 bytes of constant
storages 16..23 of SevenNet-0's deployed_serial.pt with ``zipfile`` (no
unpickling, nothing executed).  Shapes/strides come from disassembling
constants.pkl with ``pickletools`` (a parser, not an unpickler); they are the
(l1, l2, l3) tables consumed as c22..c29 in the frozen TP code
(serial_code.py:520-587), index order [m1 (x), m2 (filter), m3 (out)].
Output: tests/golden/cg_frozen.npz
"""
import os
import zipfile

import numpy as np

SERIAL = ('/root/reference/sevenn/pretrained_potentials/SevenNet_0__11July2024/'
          'serial_model/deployed_serial.pt')
SPECS = {16: ((3, 3, 3), (3, 1, 9)), 17: ((3, 3, 5), (5, 15, 1)),
         18: ((3, 5, 3), (5, 1, 15)), 19: ((3, 5, 5), (25, 1, 5)),
         20: ((5, 3, 3), (1, 15, 5)), 21: ((5, 3, 5), (1, 25, 5)),
         22: ((5, 5, 3), (5, 1, 25)), 23: ((5, 5, 5), (5, 1, 25))}


def main():
    z = zipfile.ZipFile(SERIAL)
    out = {}
    for key, (shape, stride) in SPECS.items():
        raw = np.frombuffer(z.read(f'deployed_serial/constants/{key}'), dtype='<f4')
        arr = np.lib.stride_tricks.as_strided(
            raw, shape=shape, strides=tuple(4 * s for s in stride)).copy()
        l1, l2, l3 = ((d - 1) // 2 for d in shape)
        out[f'cg_{l1}{l2}{l3}'] = arr
    path = os.path.join(os.path.dirname(__file__), '..', 'tests', 'golden', 'cg_frozen.npz')
    np.savez(path, **out)
    print('wrote', sorted(out))


if __name__ == '__main__':
    main()
