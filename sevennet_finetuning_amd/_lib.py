"""ctypes binding of libe3gnn_hip.so (the C ABI declared in include/e3gnn.h).

This module is the only door from Python into the HIP path.  There is no
fallback: if the library is missing or cannot be loaded, every entry point
raises ``E3GNNError`` (build it with ``python -m sevennet_finetuning_amd.build_lib``).
"""
import ctypes
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
# E3GNN_LIB: an alternative in-tree build of the same library (A/B kernel
# variants from build_lib --out); never a different implementation
LIB_PATH = os.environ.get('E3GNN_LIB') or os.path.join(_HERE, 'libe3gnn_hip.so')
HEADER_PATH = os.path.join(os.path.dirname(_HERE), 'include', 'e3gnn.h')

_c_int, _c_i64, _c_f, _vp = ctypes.c_int, ctypes.c_int64, ctypes.c_float, ctypes.c_void_p
_cp = ctypes.c_char_p
_P = ctypes.POINTER

# name -> (restype, argtypes); pointers to device memory are passed as void*
SIGNATURES = {
    'e3gnn_last_error': (_cp, []),
    'e3gnn_abi_version': (_c_int, []),
    'e3gnn_load': (_vp, [_cp, _cp, _c_int]),
    'e3gnn_free': (None, [_vp]),
    'e3gnn_model_info': (_c_int, [_vp, _P(_c_int), _P(_c_f), _P(_c_int), _P(_c_int)]),
    'e3gnn_model_family': (_c_int, [_vp]),
    'e3gnn_gemm_workspace_floats': (_c_i64, [_c_int, _vp]),
    'e3gnn_gemm_grouped': (_c_int, [_c_int, _vp, _vp, _c_i64, _vp]),
    'e3gnn_gemm_grouped_ex': (_c_int, [_c_int, _vp, _vp, _c_i64, _c_int, _vp]),
    'e3gnn_gemm_reduce': (_c_int, [_c_int, _vp, _vp, _vp]),
    'e3gnn_loss_efs': (_c_int, [_c_int, _c_f, _c_i64, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                _c_f, _c_f, _c_f, _c_f, _vp, _vp, _vp, _vp, _vp]),
    'e3gnn_ewc_flat': (_c_int, [_c_i64, _vp, _vp, _vp, _vp, _c_f, _vp, _vp, _vp, _vp]),
    'e3gnn_ctx_create': (_vp, [_vp]),
    'e3gnn_ctx_free': (None, [_vp]),
    'e3gnn_energy_forces': (_c_int, [_vp, _c_i64, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                     _vp, _vp, _vp]),
    'e3gnn_graph_set': (_c_int, [_vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _vp, _vp, _vp]),
    'e3gnn_layer_forward': (_c_int, [_vp, _c_int, _vp]),
    'e3gnn_feature_ptr': (_vp, [_vp, _c_int]),
    'e3gnn_feature_dim': (_c_int, [_vp, _c_int]),
    'e3gnn_readout': (_c_int, [_vp, _vp, _vp, _vp]),
    'e3gnn_layer_backward': (_c_int, [_vp, _c_int, _vp]),
    'e3gnn_set_interior': (_c_int, [_vp, _c_i64]),
    'e3gnn_layer_forward_part': (_c_int, [_vp, _c_int, _c_int, _vp]),
    'e3gnn_layer_backward_part': (_c_int, [_vp, _c_int, _c_int, _vp]),
    'e3gnn_grad_ptr': (_vp, [_vp, _c_int]),
    'e3gnn_forces': (_c_int, [_vp, _vp, _vp, _vp, _vp]),
    'e3gnn_halo_pack': (_c_int, [_vp, _c_i64, _c_int, _vp, _c_i64, _vp, _vp]),
    'e3gnn_halo_unpack': (_c_int, [_vp, _c_i64, _c_int, _vp, _vp, _c_i64, _c_int, _vp]),
    'e3gnn_conv_dims': (_c_int, [_c_int, _P(_c_int), _P(_c_int), _P(_c_int)]),
    'e3gnn_conv_graph': (_c_int, [_c_i64, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    'e3gnn_conv_graph_i64': (_c_int, [_c_i64, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    'e3gnn_conv_graph_small_max_nodes': (_c_int, []),
    'e3gnn_conv_graph_small_max_edges': (_c_int, []),
    'e3gnn_conv_forward': (_c_int, [_c_int, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    'e3gnn_conv_backward': (_c_int, [_c_int, _c_i64, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                     _vp, _vp, _vp, _vp, _vp, _vp]),
    'e3gnn_conv_forward_acc': (_c_int, [_c_int, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp, _c_int,
                                        _vp]),
    'e3gnn_conv_backward_acc': (_c_int, [_c_int, _c_i64, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp,
                                         _vp, _vp, _vp, _vp, _vp, _vp, _c_int, _vp]),
    'e3gnn_conv_tangent_forward': (_c_int, [_c_int, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                            _vp, _vp, _c_int, _vp]),
    'e3gnn_conv_dual_backward': (_c_int, [_c_int, _c_i64, _c_i64] + [_vp] * 17 + [_vp]),
    'e3gnn_radial_mlp_forward': (_c_int, [_c_i64, _c_int] + [_vp] * 11 + [_c_f, _vp]),
    'e3gnn_radial_mlp_forward_p': (_c_int, [_c_i64, _c_int] + [_vp] * 12 + [_c_f, _vp]),
    'e3gnn_radial_mlp_w2_piece_bytes': (_c_i64, [_c_int]),
    'e3gnn_radial_mlp_w2_pieces': (_c_int, [_c_int, _vp, _vp, _vp, _vp]),
    'e3gnn_radial_mlp_backward': (_c_int, [_c_i64, _c_int] + [_vp] * 11 + [_c_f, _vp]),
    'e3gnn_radial_mlp_backward_p': (_c_int, [_c_i64, _c_int] + [_vp] * 12 + [_c_f, _vp]),
    'e3gnn_edge_geometry': (_c_int, [_c_i64, _vp, _vp, _c_f, _c_f, _c_int, _vp, _vp, _vp]),
    'e3gnn_edge_geometry_jvp': (_c_int, [_c_i64, _vp, _vp, _c_f, _c_f, _c_int] + [_vp] * 10),
    'e3gnn_edge_geometry_vjp': (_c_int, [_c_i64, _vp, _vp, _c_f, _c_f, _c_int, _vp, _vp, _vp, _vp]),
    'e3gnn_edge_geometry_coeff_grad': (_c_int, [_c_i64, _vp, _vp, _c_f, _c_f] + [_vp] * 5),
    'e3gnn_edge_forces_to_atoms': (_c_int, [_c_i64] + [_vp] * 6),
    'e3gnn_gtp_create': (_vp, [_c_int, _vp, _c_int, _c_int, _c_int, _c_int]),
    'e3gnn_gtp_free': (None, [_vp]),
    'e3gnn_gtp_dims': (_c_int, [_vp, _P(_c_int), _P(_c_int), _P(_c_int), _P(_c_int)]),
    'e3gnn_gtp_forward': (_c_int, [_vp, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    'e3gnn_gtp_backward': (_c_int, [_vp, _c_i64, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                    _vp, _vp, _vp, _vp, _vp, _vp]),
    'e3gnn_act': (_c_int, [_c_int, _c_i64, _vp, _vp, _vp, _vp, _vp, _c_f, _vp]),
    'e3gnn_gate': (_c_int, [_c_int, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp, _c_f, _vp]),
    'e3gnn_act_dual': (_c_int, [_c_i64, _vp, _vp, _vp, _vp, _vp, _vp, _c_f, _vp]),
    'e3gnn_gate_dual': (_c_int, [_c_int, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _c_f, _vp]),
    'e3gnn_d3_create': (_vp, [_c_int, _c_int, _vp, _c_f, _c_f, _c_int, _vp, _vp, _vp, _vp, _vp]),
    'e3gnn_d3_free': (None, [_vp]),
    'e3gnn_d3_compute': (_c_int, [_vp, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    'e3gnn_nlist_create': (_vp, [_c_int]),
    'e3gnn_nlist_free': (None, [_vp]),
    'e3gnn_nlist_build': (_c_int, [_vp, _c_i64, _vp, _P(ctypes.c_double), _P(_c_int),
                                   ctypes.c_double, _P(_c_i64), _vp]),
    'e3gnn_nlist_fetch': (_c_int, [_vp, _vp, _vp, _vp, _vp, _vp]),
    'e3gnn_set_impl': (_c_int, [_vp, _c_int]),
    'e3gnn_set_timing': (_c_int, [_vp, _c_int]),
    'e3gnn_set_stream_ordered': (_c_int, [_vp, _c_int]),
    'e3gnn_kernel_stats': (_c_int, [_vp, _P(_cp), _P(ctypes.c_double), _P(_c_i64),
                                    _P(ctypes.c_double), _P(ctypes.c_double), _c_int]),
    'e3gnn_reset_stats': (_c_int, [_vp]),
    'e3gnn_cg_table': (_c_int, [_c_int, _c_int, _c_int, _P(_c_f)]),
    'e3gnn_workspace_bytes': (_c_i64, [_vp]),
    'e3gnn_debug_ptr': (_vp, [_vp, _cp, _c_int, _P(_c_i64)]),
}


class GemmLayout(ctypes.Structure):
    """e3gnn_gemm_layout (include/e3gnn.h)"""
    _fields_ = [('ld', _c_i64), ('kst', _c_i64), ('sst', _c_i64), ('rep', ctypes.c_int32),
                ('rs', ctypes.c_int32), ('ks', ctypes.c_int32)]


class GemmLayouts(ctypes.Structure):
    """e3gnn_gemm_layouts (include/e3gnn.h)"""
    _fields_ = [('a', GemmLayout), ('b', GemmLayout), ('a2', GemmLayout), ('b2', GemmLayout),
                ('ldc', _c_i64), ('crep', ctypes.c_int32), ('crs', ctypes.c_int32),
                ('cns', ctypes.c_int32)]


class GemmDesc(ctypes.Structure):
    """e3gnn_gemm_desc (include/e3gnn.h)"""
    _fields_ = [('a', _vp), ('b', _vp), ('a2', _vp), ('b2', _vp), ('c', _vp),
                ('lda', _c_i64), ('ldb', _c_i64), ('lda2', _c_i64), ('ldb2', _c_i64),
                ('ldc', _c_i64), ('m', ctypes.c_int32), ('n', ctypes.c_int32),
                ('k', ctypes.c_int32), ('k2', ctypes.c_int32), ('trans_a', ctypes.c_int32),
                ('trans_b', ctypes.c_int32), ('trans_a2', ctypes.c_int32),
                ('trans_b2', ctypes.c_int32), ('alpha', ctypes.c_float), ('beta', ctypes.c_int32),
                ('krange', _vp), ('krange_stride_m', ctypes.c_int32), ('layout', _vp)]


class E3GNNError(RuntimeError):
    """Error raised by the HIP library (maps the reference's error->all)."""


_lib = None


def header_symbols(path=HEADER_PATH):
    """Function names declared in include/e3gnn.h."""
    text = open(path).read()
    text = re.sub(r'/\*.*?\*/', '', text, flags=re.S)
    return sorted(set(re.findall(r'\b(e3gnn_[a-z0-9_]+)\s*\(', text)))


def load():
    """Load (once) and return the configured ctypes library."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise E3GNNError(f'{LIB_PATH} is missing: the HIP path is not built '
                         '(python -m sevennet_finetuning_amd.build_lib); there is no CPU fallback')
    # torch's wheel bundles a HIP runtime with the same SONAME
    # (libamdhip64.so.7); importing torch first makes the library bind to
    # that one copy, so torch's device pointers and streams are ours too.
    import torch  # noqa: F401
    lib = ctypes.CDLL(LIB_PATH)
    variant = 'E3GNN_LIB' in os.environ
    for name, (res, args) in SIGNATURES.items():
        if variant and not hasattr(lib, name):
            # an A/B timing variant built before this entry point existed: the
            # entry is absent there, and calling it says so (the shipped
            # library must export every symbol: tests/test_abi.py)
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc):
    if rc != 0:
        raise E3GNNError(f'e3gnn error {rc}: {load().e3gnn_last_error().decode()}')
    return rc


def cg_table(l1, l2, l3):
    import numpy as np
    out = np.zeros((2 * l1 + 1) * (2 * l2 + 1) * (2 * l3 + 1), dtype=np.float32)
    check(load().e3gnn_cg_table(l1, l2, l3, out.ctypes.data_as(_P(_c_f))))
    return out.reshape(2 * l1 + 1, 2 * l2 + 1, 2 * l3 + 1)
