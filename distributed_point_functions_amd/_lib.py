"""ctypes binding of the native library (include/dpf_amd.h).

The product path has no CPU fallback: importing a compute entry point without
the built libdpf_amd.so raises immediately (build it with
``python -m distributed_point_functions_amd.build_native``).
"""
from __future__ import annotations

import ctypes
import os

PKG = os.path.dirname(os.path.abspath(__file__))
# DPF_AMD_LIB selects another in-tree build of the same library (kernel
# variants built by tools/build_variants.py for A/B measurements).
LIB_PATH = os.environ.get("DPF_AMD_LIB") or os.path.join(PKG, "_native", "libdpf_amd.so")

MAX_SCALARS = 16
MAX_CORRECTIONS = 32


class Scalar(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("bytes", ctypes.c_int32),
                ("in_offset", ctypes.c_int32), ("out_offset", ctypes.c_int32),
                ("modulus", ctypes.c_uint64 * 2)]


class ValueTypeDesc(ctypes.Structure):
    """dpf_amd_value_type."""
    _fields_ = [("num_scalars", ctypes.c_int32),
                ("directly_convertible", ctypes.c_int32),
                ("elements_per_block", ctypes.c_int32),
                ("element_size", ctypes.c_int32),
                ("blocks_needed", ctypes.c_int32),
                ("out_stride", ctypes.c_int32),
                ("reserved", ctypes.c_int32 * 2),
                ("scalars", Scalar * MAX_SCALARS)]


class DpfAmdError(RuntimeError):
    """A non-OK status from the native library (absl::StatusCode number)."""

    def __init__(self, code: int, message: str):
        super().__init__("%s: %s" % (STATUS_NAMES.get(code, str(code)), message))
        self.code = code
        self.message = message


STATUS_NAMES = {0: "OK", 3: "INVALID_ARGUMENT", 8: "RESOURCE_EXHAUSTED",
                9: "FAILED_PRECONDITION", 12: "UNIMPLEMENTED", 13: "INTERNAL"}

_lib = None

# dpf_amd_apply_fn: int (*)(void* user, int level, const void* values, int64 n)
APPLY_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                            ctypes.c_int64)

P = ctypes.c_void_p
I64 = ctypes.c_int64
U64 = ctypes.c_uint64
I32 = ctypes.c_int
SZ = ctypes.c_size_t


def _sig(lib, name, restype, *argtypes):
    f = getattr(lib, name)
    f.restype = restype
    f.argtypes = list(argtypes)


def lib():
    """Loads libdpf_amd.so; raises if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    # One HIP runtime per process: torch bundles its own libamdhip64.so.7;
    # loading it first makes libdpf_amd.so bind to the same runtime (same
    # soname) instead of pulling in a second copy from /opt/rocm.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            "native library %s is missing; build it with "
            "`python -m distributed_point_functions_amd.build_native` "
            "(there is no CPU fallback)" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    _sig(L, "dpf_amd_last_error", ctypes.c_char_p)
    _sig(L, "dpf_amd_version", ctypes.c_char_p)
    _sig(L, "dpf_amd_device_count", I32, ctypes.POINTER(ctypes.c_int))
    _sig(L, "dpf_amd_release_cached_memory", I32, ctypes.POINTER(I64))
    _sig(L, "dpf_amd_set_thread_cache_cap", I32, I32)
    _sig(L, "dpf_amd_set_force_peer_copies", None, I32)
    _sig(L, "dpf_amd_free", None, P)
    _sig(L, "dpf_amd_aes128_mmo", I32, U64, U64, P, P, I64, P)
    _sig(L, "dpf_amd_evaluate_seeds", I32, I64, I32, I64, P, P, P, I32, P, P, P,
         U64, U64, U64, U64, P, P, P)
    _sig(L, "dpf_amd_expand_and_correct", I32, I64, P, P, I32, P, P, P,
         ctypes.POINTER(ValueTypeDesc), P, I32, I32, I64, I64, P, P)
    _sig(L, "dpf_amd_expand_and_correct_batched", I32, I64, P, P, I32, P, P, P,
         ctypes.POINTER(ValueTypeDesc), P, P, I32, I64, I64, P, P)
    _sig(L, "dpf_amd_evaluate_points", I32, I64, P, P, P, I32, I32, I64, P, P, P,
         ctypes.POINTER(ValueTypeDesc), P, P, I32, P, P, P, P, P, P)
    _sig(L, "dpf_amd_dcf_evaluate", I32, I64, P, P, P, P, I32, P, P, P, P,
         ctypes.POINTER(ValueTypeDesc), P, P, P)
    _sig(L, "dpf_amd_evaluate_points_batched", I32, I64, I64, P, P, P, I32, I32, P, P, P,
         ctypes.POINTER(ValueTypeDesc), P, P, I32, P, P, P, P)
    _sig(L, "dpf_amd_gather_rows", I32, I64, P, I64, I64, P, P, P)
    _sig(L, "dpf_amd_inner_product_workspace_size", I64, I64, I64, I32)
    _sig(L, "dpf_amd_inner_product", I32, P, I64, I64, P, I64, I32, P, P, P)
    _sig(L, "dpf_amd_xor_fold", I32, P, I32, I64, P, P)
    _sig(L, "dpf_amd_set_expand_depth", I32, I32)
    _sig(L, "dpf_amd_set_expand_roots", I32, I32)
    _sig(L, "dpf_amd_set_scan_m4", I32, I32)
    _sig(L, "dpf_amd_set_scan_skip_unselected", I32, I32)
    _sig(L, "dpf_amd_set_walk_mode", I32, I32)
    _sig(L, "dpf_amd_set_dcf_kernel", I32, I32)
    _sig(L, "dpf_amd_set_prefix_expand", I32, I32)
    _bind_tier2(L)
    _lib = L
    return L


def _bind_tier2(L):
    names = [n for n in ("dpf_amd_describe_value_type",) if hasattr(L, n)]
    if not names:
        return
    PP = ctypes.POINTER(ctypes.c_void_p)
    BUF = ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8))
    _sig(L, "dpf_amd_describe_value_type", I32, P, SZ, ctypes.c_double,
         ctypes.POINTER(ValueTypeDesc))
    _sig(L, "dpf_amd_dpf_create_incremental", I32, P, P, I32, PP)
    _sig(L, "dpf_amd_dpf_destroy", None, P)
    _sig(L, "dpf_amd_dpf_tree_levels_needed", I32, P)
    _sig(L, "dpf_amd_dpf_hierarchy_to_tree", I32, P, I32)
    _sig(L, "dpf_amd_dpf_value_type", I32, P, I32, ctypes.POINTER(ValueTypeDesc))
    _sig(L, "dpf_amd_dpf_register_value_type", I32, P, P, SZ)
    _sig(L, "dpf_amd_dcf_register_value_type", I32, P, P, SZ)
    _sig(L, "dpf_amd_dpf_generate_keys", I32, P, U64, U64, P, P, P, BUF,
         ctypes.POINTER(SZ), BUF, ctypes.POINTER(SZ))
    _sig(L, "dpf_amd_ctx_create", I32, P, P, SZ, PP)
    _sig(L, "dpf_amd_ctx_parse", I32, P, P, SZ, PP)
    _sig(L, "dpf_amd_ctx_serialize", I32, P, BUF, ctypes.POINTER(SZ))
    _sig(L, "dpf_amd_ctx_destroy", None, P)
    _sig(L, "dpf_amd_ctx_previous_hierarchy_level", I32, P)
    _sig(L, "dpf_amd_ctx_partial_evaluations_level", I32, P)
    _sig(L, "dpf_amd_ctx_num_partial_evaluations", I64, P)
    _sig(L, "dpf_amd_evaluate_until", I32, P, I32, P, I64, P, SZ, P, P, I64,
         ctypes.POINTER(I64))
    _sig(L, "dpf_amd_evaluate_until_device", I32, P, I32, P, I64, P, SZ, P, P, I64,
         ctypes.POINTER(I64), P)
    _sig(L, "dpf_amd_evaluate_at", I32, P, P, SZ, I32, P, I64, P, SZ, P)
    _sig(L, "dpf_amd_evaluate_at_ctx", I32, P, I32, P, I64, P, SZ, P, P)
    _sig(L, "dpf_amd_expand_leaves_on_devices", I32, P, P, SZ, I32, P, P, P, P)
    _sig(L, "dpf_amd_evaluate_and_apply", I32, P, P, P, I64, P, I32, P, SZ, P, APPLY_FN, P)
    _sig(L, "dpf_amd_dcf_create", I32, P, SZ, PP)
    _sig(L, "dpf_amd_dcf_destroy", None, P)
    _sig(L, "dpf_amd_dcf_generate_keys", I32, P, U64, U64, P, SZ, P, BUF,
         ctypes.POINTER(SZ), BUF, ctypes.POINTER(SZ))
    _sig(L, "dpf_amd_dcf_batch_evaluate", I32, P, P, P, I64, P, I64, P, SZ, P)
    _sig(L, "dpf_amd_pir_db_create", I32, PP)
    _sig(L, "dpf_amd_pir_db_insert", I32, P, P, SZ)
    _sig(L, "dpf_amd_pir_db_insert_fixed", I32, P, P, I64, I64)
    _sig(L, "dpf_amd_pir_db_insert_packed", I32, P, P, P, I64)
    _sig(L, "dpf_amd_pir_db_build", I32, P)
    _sig(L, "dpf_amd_pir_db_destroy", None, P)
    _sig(L, "dpf_amd_pir_db_size", I64, P)
    _sig(L, "dpf_amd_pir_db_max_value_size", I64, P)
    _sig(L, "dpf_amd_pir_db_device_records", P, P, ctypes.POINTER(I64))
    _sig(L, "dpf_amd_pir_db_inner_product", I32, P, P, I64, I32, P)
    _sig(L, "dpf_amd_pir_db_set_devices", I32, P, P, I32)
    _sig(L, "dpf_amd_pir_db_insert_fixed_device", I32, P, P, I32, I64, I64)
    _sig(L, "dpf_amd_pir_db_num_shards", I32, P)
    _sig(L, "dpf_amd_pir_db_shard", I32, P, I32, ctypes.POINTER(ctypes.c_int),
         ctypes.POINTER(I64), ctypes.POINTER(I64), ctypes.POINTER(P))
    _sig(L, "dpf_amd_pir_server_create_plain", I32, P, SZ, P, PP)
    _sig(L, "dpf_amd_pir_server_destroy", None, P)
    _sig(L, "dpf_amd_pir_call_while_waiting", I32, P)
    _sig(L, "dpf_amd_pir_call_set_response", I32, P, P, SZ)
    _sig(L, "dpf_amd_pir_server_create_leader", I32, P, SZ, P, P, P, PP)
    _sig(L, "dpf_amd_pir_server_create_helper", I32, P, SZ, P, P, P, PP)
    _sig(L, "dpf_amd_pir_server_handle_request", I32, P, P, SZ, BUF,
         ctypes.POINTER(SZ))
    _sig(L, "dpf_amd_pir_server_public_params", I32, P, BUF, ctypes.POINTER(SZ))
    _sig(L, "dpf_amd_sha256_hash", I32, P, SZ, P, SZ, I32, ctypes.POINTER(I32))
    _sig(L, "dpf_amd_hash_family_evaluate", I32, P, SZ, I32, P, SZ, I32, ctypes.POINTER(I32))
    _sig(L, "dpf_amd_cuckoo_generate_params", I32, P, SZ, BUF, ctypes.POINTER(SZ))
    _sig(L, "dpf_amd_cuckoo_db_create", I32, P, SZ, PP)
    _sig(L, "dpf_amd_cuckoo_db_insert", I32, P, P, SZ, P, SZ)
    _sig(L, "dpf_amd_cuckoo_db_place", I32, P, ctypes.POINTER(I64), I64)
    _sig(L, "dpf_amd_cuckoo_db_place_keys", I32, P, P, SZ)
    _sig(L, "dpf_amd_cuckoo_db_build", I32, P)
    _sig(L, "dpf_amd_cuckoo_db_destroy", None, P)
    _sig(L, "dpf_amd_cuckoo_db_size", I64, P)
    _sig(L, "dpf_amd_cuckoo_db_num_selection_bits", I64, P)
    _sig(L, "dpf_amd_cuckoo_server_create_plain", I32, P, SZ, P, PP)
    _sig(L, "dpf_amd_cuckoo_server_create_leader", I32, P, SZ, P, P, P, PP)
    _sig(L, "dpf_amd_cuckoo_server_create_helper", I32, P, SZ, P, P, P, PP)


def check(code: int):
    if code != 0:
        raise DpfAmdError(code, lib().dpf_amd_last_error().decode(errors="replace"))


def take_buffer(ptr, size) -> bytes:
    """Copies and frees a library-allocated buffer."""
    try:
        return ctypes.string_at(ptr, size.value if hasattr(size, "value") else size)
    finally:
        lib().dpf_amd_free(ptr)


def stream_ptr(stream=None):
    """hipStream_t of a torch stream (None = current stream)."""
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def dptr(t) -> ctypes.c_void_p:
    """Device pointer of a torch tensor (or None)."""
    if t is None:
        return ctypes.c_void_p(0)
    return ctypes.c_void_p(t.data_ptr())
