"""Build libe3gnn_hip.so in-tree for gfx950 (hipcc cross-compiles without a GPU).

    python -m sevennet_finetuning_amd.build_lib [--force]

The library is the product: the Python surface of this package only loads it
(``_lib.py``) and fails loudly when it is missing.
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, 'csrc')
INCLUDE = os.path.join(os.path.dirname(HERE), 'include')
LIB = os.path.join(HERE, 'libe3gnn_hip.so')
OBJDIR = os.path.join(HERE, 'csrc', 'build')
SOURCES = ['api.cpp', 'generic.cpp', 'gemm.hip', 'tp.hip', 'node.hip', 'fused.hip', 'neighbor.hip', 'd3.hip',
           'train_ops.hip', 'gtp.hip', 'generic.hip', 'mlp_train.hip', 'tgemm.hip']
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
FLAGS = ['--offload-arch=gfx950', '-O3', '-std=c++17', '-fPIC', f'-I{INCLUDE}',
         '-Wall', '-Wno-unused-function']
# fused.hip: no SLP packing (v_pk_* f32 pairs beside MFMA cost issue slots and
# double the live registers of the tensor-product loops: 146 -> 123 VGPRs)
FILE_FLAGS = {'fused.hip': os.environ.get('E3GNN_FUSED_FLAGS', '-fno-slp-vectorize').split()}


def _deps_mtime():
    files = [os.path.join(CSRC, f) for f in os.listdir(CSRC)
             if f.endswith(('.h', '.hip', '.cpp'))]
    files.append(os.path.join(INCLUDE, 'e3gnn.h'))
    return max(os.path.getmtime(f) for f in files)


def build(force=False, verbose=False, out=None, defines=()):
    """Compile and link the library (``out``: another path, for A/B variants
    built with extra ``-D`` ``defines``)."""
    lib = out or LIB
    if not force and os.path.exists(lib) and os.path.getmtime(lib) >= _deps_mtime():
        if out is None:
            build_native(lib, verbose, only_stale=True)
        return lib
    objdir = OBJDIR if out is None else os.path.join(OBJDIR, os.path.basename(out))
    os.makedirs(objdir, exist_ok=True)
    extra = [f'-D{d}' for d in defines]

    def compile_one(src):
        obj = os.path.join(objdir, src + '.o')
        cmd = [HIPCC, *FLAGS, *extra, *FILE_FLAGS.get(src, []), '-c', os.path.join(CSRC, src),
               '-o', obj]
        if verbose:
            print(' '.join(cmd))
        # a register-allocation pathology once kept clang busy for 30+ minutes
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
        if r.returncode != 0:
            raise RuntimeError(f'hipcc failed on {src}:\n{r.stdout}\n{r.stderr}')
        return obj

    with ThreadPoolExecutor(max_workers=4) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    os.makedirs(os.path.dirname(os.path.abspath(lib)), exist_ok=True)
    tmp = lib + '.tmp'
    cmd = [HIPCC, '--offload-arch=gfx950', '-shared', '-fPIC', '-o', tmp, *objs]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f'link failed:\n{r.stdout}\n{r.stderr}')
    os.replace(tmp, lib)
    if out is None:
        build_native(lib, verbose)
    return lib


NATIVE = os.path.join(os.path.dirname(HERE), 'native')


NATIVE_HOSTS = ('e3gnn_md', 'e3gnn_md_parallel', 'e3gnn_pair_check')
# extra translation units of a host (the LAMMPS pair-style core)
NATIVE_EXTRA = {'e3gnn_pair_check': ['pair_e3gnn_core.cpp', 'lammps/pair_e3gnn_hip.cpp',
                                     'lammps/pair_e3gnn_parallel_hip.cpp', 'lammps_mock/mini_lammps.cpp']}
# e3gnn_pair_check compiles the LAMMPS adaptors against the mini-LAMMPS scaffold
NATIVE_INCLUDES = {'e3gnn_pair_check': ['.', 'lammps_mock', 'lammps']}


def build_native(lib=LIB, verbose=False, only_stale=False):
    """native/e3gnn_md (serial MD host) and native/e3gnn_md_parallel (the
    pair_e3gnn_parallel call sequence over N in-process sub-domains): C++ over
    the C ABI (no Python), linked against the in-tree library with an
    $ORIGIN-relative rpath."""
    exes = []
    for name in NATIVE_HOSTS:
        srcs = [os.path.join(NATIVE, f) for f in [name + '.cpp'] + NATIVE_EXTRA.get(name, [])]
        incs = [os.path.join(NATIVE, d) for d in NATIVE_INCLUDES.get(name, [])]
        hdrs = [os.path.join(d, f) for d in [NATIVE, *incs] for f in os.listdir(d) if f.endswith('.h')]
        exe = os.path.join(NATIVE, name)
        exes.append(exe)
        if (only_stale and os.path.exists(exe) and os.path.getmtime(exe) >=
                max([os.path.getmtime(f) for f in srcs + hdrs] + [os.path.getmtime(lib)])):
            continue
        cmd = [HIPCC, '-O2', '-std=c++17', f'-I{INCLUDE}', *[f'-I{d}' for d in incs], *srcs, '-o', exe,
               f'-L{os.path.dirname(lib)}', '-le3gnn_hip', '-lpthread',
               "-Wl,-rpath,$ORIGIN/../sevennet_finetuning_amd"]
        if verbose:
            print(' '.join(cmd))
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            raise RuntimeError(f'hipcc failed on {name}.cpp:\n{r.stdout}\n{r.stderr}')
    return exes


if __name__ == '__main__':
    sys.stdout.reconfigure(line_buffering=True)
    args = sys.argv[1:]
    out = args[args.index('--out') + 1] if '--out' in args else None
    defs = [a[2:] for a in args if a.startswith('-D')]
    print(build(force='--force' in args, verbose=True, out=out, defines=defs))
