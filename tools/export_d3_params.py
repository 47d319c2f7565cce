"""Export the DFT-D3 parameter DATA the reference ships (Grimme's published
reference tables) into this build's own asset files.

Reads, as text, from the reference checkout (never executed, never copied as
source):
  sevenn/pair_e3gnn/pair_d3_pars.h   R0AB_TABLE (94 x 94, Angstrom) and
                                      C6AB_TABLE (32385 x [C6, Z_i, Z_j, CN_i, CN_j])
  sevenn/pair_e3gnn/pair_d3.cu       r2r4_ref[94], rcov_ref[94] (:714-773) and the
                                      functional parameter switch of
                                      PairD3::setfuncpar (:422-653)
Writes:
  sevennet_finetuning_amd/assets/d3/d3_params.npz      (numpy, no pickle)
  sevennet_finetuning_amd/assets/d3/d3_functionals.json

usage: python tools/export_d3_params.py [/root/reference]
"""
import json
import os
import re
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, 'sevennet_finetuning_amd', 'assets', 'd3')
NUM = r'[-+]?\d*\.?\d+(?:[eE][-+]?\d+)?'


def numbers_after(text, marker, count):
    i = text.index(marker) + len(marker)
    vals = []
    for m in re.finditer(NUM, text[i:]):
        vals.append(float(m.group(0)))
        if len(vals) == count:
            return np.array(vals)
    raise ValueError(f'{marker}: found {len(vals)} of {count} numbers')


def functional_tables(cu):
    """{damping: {functional: {s6, rs6, s18, rs18, alp}}} from setfuncpar.

    Follows the C control flow literally: defaults set before the name map,
    then the assignments of the matched case up to its first `break` (so an
    assignment written after `break;` has no effect, as in the reference)."""
    body = cu[cu.index('void PairD3::setfuncpar'):cu.index('void PairD3::coeff')]
    blocks = re.split(r'(?:if|else if) \(damping_type == (\w+)\)', body)
    out = {}
    names = {'zero_damping': 'zero', 'bj_damping': 'bj', 'zero_damping_modified': 'zerom',
             'bj_damping_modified': 'bjm'}
    for kind, blk in zip(blocks[1::2], blocks[2::2]):
        head = blk[:blk.index('commandMap')]
        defaults = {k: float(v) for k, v in re.findall(r'(\w+) = (' + NUM + r');', head)}
        cmap = {name: int(code) for name, code in
                re.findall(r'\{\s*"([^"]+)",\s*(\d+)\s*\}', blk)}
        cases = {}
        for code, stmts in re.findall(r'case (\d+):(.*?)(?=case \d+:|default:)', blk, re.S):
            stmts = re.sub(r'/\*.*?\*/', '', stmts, flags=re.S)
            stmts = re.sub(r'//[^\n]*', '', stmts)
            stmts = stmts.split('break;')[0]
            cases[int(code)] = {k: float(v) for k, v in re.findall(r'(\w+) = (' + NUM + r');', stmts)}
        table = {}
        for name, code in cmap.items():
            p = {'s6': 1.0, 'rs6': 0.0, 's18': 0.0, 'rs18': 1.0, 'alp': 14.0}
            p.update(defaults)
            p.update(cases[code])
            table[name] = p
        out[names[kind]] = table
    return out


def main(ref):
    pars = open(os.path.join(ref, 'sevenn/pair_e3gnn/pair_d3_pars.h')).read()
    cu = open(os.path.join(ref, 'sevenn/pair_e3gnn/pair_d3.cu')).read()
    r0ab = numbers_after(pars, '#define R0AB_TABLE', 94 * 94).reshape(94, 94)
    c6ab = numbers_after(pars, '#define C6AB_TABLE', 32385 * 5).reshape(32385, 5)
    r2r4 = numbers_after(cu, 'double r2r4_ref[94] =', 94)
    rcov = numbers_after(cu, 'double rcov_ref[94] =', 94)
    os.makedirs(OUT, exist_ok=True)
    np.savez(os.path.join(OUT, 'd3_params.npz'), r0ab=r0ab, c6ab=c6ab, r2r4=r2r4, rcov=rcov)
    funcs = functional_tables(cu)
    json.dump({'source': 'kskjs1203/SevenNet_finetuning sevenn/pair_e3gnn (Grimme DFT-D3 tables)',
               'units': {'r0ab': 'Angstrom', 'rcov': 'Bohr (k2 = 4/3 scaled)',
                         'c6ab': 'Hartree Bohr^6', 'r2r4': 'sqrt(0.5 r2r4 sqrt(Z))'},
               'functionals': funcs}, open(os.path.join(OUT, 'd3_functionals.json'), 'w'), indent=1)
    print('r0ab', r0ab.shape, 'c6ab', c6ab.shape, {k: len(v) for k, v in funcs.items()})
    print('pbe bj', funcs['bj']['pbe'], 'pbe zero', funcs['zero']['pbe'])


if __name__ == '__main__':
    main(sys.argv[1] if len(sys.argv) > 1 else '/root/reference')
