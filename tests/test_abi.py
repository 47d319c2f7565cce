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


def test_grouped_gemm_refuses_operands_beyond_32bit_offsets():
    """e3gnn_gemm_grouped addresses each operand through one buffer
    descriptor (32-bit byte offsets, csrc/tgemm.hip TG_RECORDS): a problem
    whose operand spans more is refused with E3GNN_ERR_ARG before anything
    is launched (no device is touched, so this runs on the CPU)"""
    lib = _lib.load()
    fake = ctypes.c_void_p(1 << 20)   # never dereferenced: the check comes first
    d = _lib.GemmDesc()
    d.a = d.b = d.c = fake
    d.m, d.n, d.ldc = 64, 64, 64
    # op(A) = A^T of a (K x 64) row-major matrix: K = 2^23 rows x 64 floats = 2 GB
    d.k, d.lda, d.trans_a, d.ldb, d.trans_b = 1 << 23, 64, 1, 64, 0
    rc = lib.e3gnn_gemm_grouped(1, ctypes.byref(d), None, 0, None)
    assert rc == 1   # E3GNN_ERR_ARG
    assert b'2 GB' in lib.e3gnn_last_error()
    # an int32-overflowing leading dimension is refused as well
    d.k, d.lda = 16, 1 << 33
    assert lib.e3gnn_gemm_grouped(1, ctypes.byref(d), None, 0, None) != 0
    # general layouts: K summed over segments whose stride walks past 2 GB
    lay = _lib.GemmLayouts()
    d2 = _lib.GemmDesc()
    d2.a = d2.b = d2.c = fake
    d2.m, d2.n, d2.k = 16, 16, 4 * 1000
    for g in (lay.a, lay.b):
        g.ld, g.rep, g.rs, g.kst, g.ks, g.sst = 16, 1, 0, 1 << 20, 1000, 1
    lay.ldc, lay.crep, lay.crs, lay.cns = 16, 1, 0, 1
    d2.layout = ctypes.addressof(lay)
    assert lib.e3gnn_gemm_grouped(1, ctypes.byref(d2), None, 0, None) != 0
    assert b'2 GB' in lib.e3gnn_last_error()
