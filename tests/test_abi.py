"""The C-ABI library loads and exports every symbol include/e3gnn.h declares
(no compute calls: this runs without a GPU)."""
import ctypes
import subprocess

from sevennet_finetuning_amd import _lib


def test_library_exports_header_symbols():
    lib = _lib.load()
    declared = _lib.header_symbols()
    assert len(declared) >= 20
    for name in declared:
        assert hasattr(lib, name), name
    assert set(declared) == set(_lib.SIGNATURES), set(declared) ^ set(_lib.SIGNATURES)
    out = subprocess.run(['nm', '-D', '--defined-only', _lib.LIB_PATH], capture_output=True,
                         text=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if ' T ' in line}
    assert set(declared) <= exported


def test_abi_version_and_errors():
    lib = _lib.load()
    assert lib.e3gnn_abi_version() == 1
    # bad arguments are reported, not crashed on (no device needed for these)
    out = (ctypes.c_float * 27)()
    assert lib.e3gnn_cg_table(3, 3, 3, out) != 0
    assert b'coupling' in lib.e3gnn_last_error()
    assert lib.e3gnn_layer_forward(None, 0, None) != 0
    assert lib.e3gnn_ctx_create(None) is None


def test_library_is_gfx950_code_object(tmp_path):
    import shutil
    lib = tmp_path / 'lib.so'   # --offloading extracts bundles next to its input
    shutil.copy(_lib.LIB_PATH, lib)
    out = subprocess.run(['/opt/rocm/lib/llvm/bin/llvm-objdump', '--offloading', str(lib)],
                         capture_output=True, text=True, cwd=tmp_path)
    text = out.stdout + out.stderr
    assert 'gfx950' in text
