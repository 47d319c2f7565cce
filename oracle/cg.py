"""Real-basis Clebsch-Gordan coefficients in e3nn's convention (oracle copy).

TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py.

The reference never computes CG coefficients itself: its uvu tensor product
(sevenn/nn/convolution.py:72-95, e3nn ``o3.TensorProduct``) uses e3nn's
``wigner_3j(l1,l2,l3) * sqrt(2*l3+1)`` (component normalisation, path weight 1
for uvu with a multiplicity-1 filter).  The deployment froze those tables as
constants (``serial_code.py:562-587``: c22..c29).  e3nn is not installed here,
so we restate its published algorithm:

* complex SU(2) CG by the Racah formula;
* change of basis real<->complex (Wikipedia "real form", times (-i)^l);
* normalise to unit Frobenius norm;
* e3nn's precomputed tables additionally carry a per-triple overall sign that
  the algebra alone does not fix for odd l1+l2+l3 triples.  It is pinned here
  by ``E3NN_SIGN`` and checked against the frozen tables in
  ``tests/golden/cg_frozen.npz`` (test_oracle_cg.py).
"""
from functools import lru_cache
from math import factorial

import numpy as np

# Per-triple overall sign of e3nn's wigner_3j relative to the Racah/real-basis
# construction below (pinned against the frozen deployment constants).
E3NN_SIGN = {(1, 2, 2): -1.0, (2, 1, 2): -1.0, (2, 2, 1): -1.0}


def _f(n):
    return factorial(int(round(n)))


def su2_cg_coeff(j1, m1, j2, m2, j3, m3):
    if m3 != m1 + m2:
        return 0.0
    vmin = int(max(-j1 + j2 + m3, -j1 + m1, 0))
    vmax = int(min(j2 + j3 + m1, j3 - j1 + j2, j3 + m3))
    pre = ((2.0 * j3 + 1.0) * _f(j3 + j1 - j2) * _f(j3 - j1 + j2)
           * _f(j1 + j2 - j3) / _f(j1 + j2 + j3 + 1)
           * _f(j3 + m3) * _f(j3 - m3)
           / (_f(j1 + m1) * _f(j1 - m1) * _f(j2 + m2) * _f(j2 - m2))) ** 0.5
    s = 0.0
    for v in range(vmin, vmax + 1):
        s += ((-1) ** int(v + j2 + m2) / _f(v) * _f(j2 + j3 + m1 - v)
              * _f(j1 - m1 + v) / _f(j3 - j1 + j2 - v) / _f(j3 + m3 - v)
              / _f(v + j1 - j2 - m3))
    return pre * s


def _su2_cg(l1, l2, l3):
    mat = np.zeros((2 * l1 + 1, 2 * l2 + 1, 2 * l3 + 1))
    for m1 in range(-l1, l1 + 1):
        for m2 in range(-l2, l2 + 1):
            if abs(m1 + m2) <= l3:
                mat[l1 + m1, l2 + m2, l3 + m1 + m2] = su2_cg_coeff(
                    l1, m1, l2, m2, l3, m1 + m2)
    return mat


def _real_to_complex(l):
    q = np.zeros((2 * l + 1, 2 * l + 1), dtype=complex)
    for m in range(-l, 0):
        q[l + m, l + abs(m)] = 1 / 2 ** 0.5
        q[l + m, l - abs(m)] = -1j / 2 ** 0.5
    q[l, l] = 1
    for m in range(1, l + 1):
        q[l + m, l + abs(m)] = (-1) ** m / 2 ** 0.5
        q[l + m, l - abs(m)] = 1j * (-1) ** m / 2 ** 0.5
    return (-1j) ** l * q


@lru_cache(maxsize=None)
def wigner_3j(l1, l2, l3):
    """Unit-norm real CG tensor C[m1, m2, m3] in e3nn's basis and sign."""
    assert abs(l1 - l2) <= l3 <= l1 + l2
    q1, q2, q3 = _real_to_complex(l1), _real_to_complex(l2), _real_to_complex(l3)
    c = _su2_cg(l1, l2, l3).astype(complex)
    c = np.einsum('ij,kl,mn,ikn->jlm', q1, q2, np.conj(q3.T), c)
    assert np.abs(c.imag).max() < 1e-10
    c = c.real / np.linalg.norm(c.real)
    return c * E3NN_SIGN.get((l1, l2, l3), 1.0)


def tp_cg(l1, l2, l3):
    """CG used by the uvu TP: wigner_3j * sqrt(2*l3+1) (component norm)."""
    return wigner_3j(l1, l2, l3) * np.sqrt(2 * l3 + 1)
