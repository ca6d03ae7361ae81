"""ctypes binding of libsra.so (the C ABI declared in include/sra.h).

This is the "reference-side binding" of the engine: the reference is pure
Python, so its FFI for the aggregation path is this module.  It loads the
in-tree ``libsra.so`` (built by ``make -C csrc`` / ``__graft_entry__.build()``)
and maps the library's negative status codes onto the exception classes the
reference raises for the same conditions.

The product path has no CPU fallback: if the library is missing or cannot be
loaded, every call raises ``SraLibraryError``.
"""
from __future__ import annotations

import ctypes
import os
import re
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SRA_LIB", os.path.join(_HERE, "libsra.so"))
HEADER = os.path.join(os.path.dirname(_HERE), "include", "sra.h")

SRA_OK = 0
SRA_ERR_ARG = -1
SRA_ERR_SHAPE = -2
SRA_ERR_UNSUPPORTED = -3
SRA_ERR_EMPTY_BUCKET = -4
SRA_ERR_THETA = -5
SRA_ERR_HIP = -6
SRA_ERR_WORKSPACE = -7
SRA_ERR_INFEASIBLE = -8


class SraLibraryError(ImportError):
    """libsra.so is missing or failed to load (no CPU fallback exists)."""


class SraRuntimeError(RuntimeError):
    """A HIP runtime failure inside libsra."""


_EXC = {
    SRA_ERR_ARG: ValueError,
    SRA_ERR_SHAPE: ValueError,
    SRA_ERR_UNSUPPORTED: NotImplementedError,
    SRA_ERR_EMPTY_BUCKET: ValueError,
    SRA_ERR_THETA: IndexError,
    SRA_ERR_HIP: SraRuntimeError,
    SRA_ERR_WORKSPACE: ValueError,
    SRA_ERR_INFEASIBLE: TypeError,
}

_i64 = ctypes.c_int64
_i32 = ctypes.c_int32
_ptr = ctypes.c_void_p
_dbl = ctypes.c_double
_sz = ctypes.c_size_t

# name -> argtypes (restype is int unless listed in _RESTYPES)
_SIGS = {
    "sra_last_error": [],
    "sra_version": [],
    "sra_max_register_clients": [],
    "sra_row_fault_count": [_i32, ctypes.POINTER(ctypes.c_uint32)],
    "sra_average_f32": [_ptr, _i64, _i64, _i64, _ptr, _ptr],
    "sra_median_f32": [_ptr, _i64, _i64, _i64, _ptr, _ptr],
    "sra_trimmed_mean_f32": [_ptr, _i64, _i64, _i64, _i32, _ptr, _ptr],
    "sra_gram_workspace_bytes": [_i64, _i64, ctypes.POINTER(_sz)],
    "sra_gram_f32": [_ptr, _i64, _i64, _i64, _ptr, _ptr, _sz, _ptr],
    "sra_krum_workspace_bytes": [_i64, _i64, ctypes.POINTER(_sz)],
    "sra_krum_select_f32": [_ptr, _i64, _i64, _i64, _i32, _i32, _ptr, _ptr, _ptr, _sz, _ptr],
    "sra_krum_from_gram_workspace_bytes": [_i64, ctypes.POINTER(_sz)],
    "sra_krum_from_gram": [_ptr, _i64, _i32, _i32, _ptr, _ptr, _ptr, _sz, _ptr],
    "sra_krum_pair_sq_workspace_bytes": [_i64, _i32, ctypes.POINTER(_sz)],
    "sra_krum_pair_sq_f32": [_ptr, _i64, _i64, _i64, _i32, _ptr, _ptr, _sz, _ptr],
    "sra_krum_from_pairs_workspace_bytes": [_i64, ctypes.POINTER(_sz)],
    "sra_krum_from_pairs": [_ptr, _i64, _i32, _i32, _ptr, _ptr, _ptr, _sz, _ptr],
    "sra_gather_rows_f32": [_ptr, _i64, _i64, _i64, _ptr, _i32, _ptr, _i64, _ptr],
    "sra_gram_buckets_f32": [_ptr, _i64, _i64, _i64, _i32, _ptr, _ptr, _sz, _ptr],
    "sra_mom_krum_workspace_bytes": [_i64, _i64, _i32, ctypes.POINTER(_sz)],
    "sra_mom_krum_f32": [_ptr, _i64, _i64, _i64, _i32, _i32, _ptr, _ptr, _ptr, _sz, _ptr],
    "sra_bucket_mean_f32": [_ptr, _i64, _i64, _i64, _i32, _i32, _ptr, _i64, _ptr],
    "sra_bulyan_workspace_bytes": [_i64, _i64, _i32, _i32, ctypes.POINTER(_sz)],
    "sra_bulyan_f32": [_ptr, _i64, _i64, _i64, _i32, _i32, _ptr, _ptr, _ptr, _ptr, _sz, _ptr],
    "sra_bulyan_coordinate_f64": [_ptr, _i64, _i64, _i64, _i32, _ptr, _ptr, _ptr, _i64, _ptr],
    "sra_bulyan_stage_workspace_bytes": [_i64, _i64, ctypes.POINTER(_sz)],
    "sra_bulyan_round_workspace_bytes": [_i64, _i64, ctypes.POINTER(_sz)],
    "sra_bulyan_round_f32": [_ptr, _i64, _i64, _i64, _ptr, _i32, _i32, _i32, _ptr, _ptr, _ptr, _sz, _ptr],
    "sra_bulyan_pick": [_ptr, _ptr, _i32, _ptr, _ptr, _ptr],
    "sra_bulyan_stage_f32": [_ptr, _i64, _i64, _i64, _i32, _ptr, _ptr, _sz, _ptr],
    "sra_filter_workspace_bytes": [_i64, _i64, _i32, ctypes.POINTER(_sz)],
    "sra_filter_f32": [_ptr, _i64, _i64, _i64, _i32, _i32, _dbl, _dbl, _dbl, _ptr, _ptr, _ptr, _sz, _ptr],
    "sra_filter_trace_f32": [_ptr, _i64, _i64, _i64, _i32, _i32, _dbl, _dbl, _dbl, _ptr, _ptr, _ptr, _ptr, _sz,
                             _ptr],
    "sra_filter_debug_f32": [_ptr, _i64, _i64, _i64, _i32, _i32, _dbl, _dbl, _dbl, _ptr, _ptr, _ptr, _ptr, _sz,
                             _ptr],
    "sra_mom_filter_workspace_bytes": [_i64, _i64, _i32, ctypes.POINTER(_sz)],
    "sra_mom_filter_f32": [_ptr, _i64, _i64, _i64, _i32, _i32, _i32, _i32, _dbl, _dbl, _dbl, _ptr, _ptr, _ptr, _sz,
                           _ptr],
    "sra_window_mean_f32": [_ptr, _i64, _i64, _i64, _i32, _i32, _i32, _ptr, _i64, _ptr],
    "sra_window_mean_f64": [_ptr, _i64, _i64, _i64, _i32, _i32, _i32, _ptr, _i64, _ptr],
    "sra_clip_workspace_bytes": [_i64, ctypes.POINTER(_i64), _i32, ctypes.POINTER(_sz)],
    "sra_clip_scale_f32": [_ptr, _i64, _i64, _i64, _ptr, ctypes.POINTER(_i64), _i32, _dbl, _ptr, _ptr, _ptr, _sz,
                           _ptr],
    "sra_clip_scale_f64": [_ptr, _i64, _i64, _i64, _ptr, ctypes.POINTER(_i64), _i32, _dbl, _ptr, _ptr, _ptr, _sz,
                           _ptr],
    "sra_clipped_mean_f32": [_ptr, _i64, _i64, _i64, _ptr, _ptr, _ptr, _i64, _ptr, _ptr],
    "sra_clipped_mean_f64": [_ptr, _i64, _i64, _i64, _ptr, _ptr, _ptr, _i64, _ptr, _ptr],
    "sra_attack_krum_workspace_bytes": [_i64, _i64, _dbl, ctypes.POINTER(_sz)],
    "sra_attack_krum_f32": [_ptr, _i64, _i64, _i64, _ptr, _ptr, _i32, _dbl, _ptr, _ptr, _ptr, _ptr, _sz, _ptr],
    "sra_attack_krum_dir_f32": [_ptr, _i64, _i64, _i64, _ptr, _ptr, _i32, _ptr, _dbl, _ptr, _ptr, _ptr, _ptr, _sz,
                                _ptr],
    "sra_mt19937_words": [_ptr, _i64, _ptr, _ptr, _ptr],
    "sra_attack_trimmedmean_f32": [_ptr, _i64, _i64, _ptr, _i32, _ptr, _ptr, _dbl, _ptr, _ptr],
    "sra_attack_xie_f32": [_ptr, _i64, _i64, _ptr, _i32, _dbl, _i64, _ptr, _ptr],
    "sra_attack_xie_f64": [_ptr, _i64, _i64, _ptr, _i32, _dbl, _i64, _ptr, _ptr],
    "sra_params_flatten_f32": [_ptr, _ptr, _i32, _i64, _ptr, _ptr],
    "sra_record_delta_f32": [_ptr, _ptr, _i32, _i64, _ptr, _ptr, _ptr],
    "sra_record_momentum_f64": [_ptr, _ptr, _i32, _i64, _ptr, ctypes.c_float, _dbl, _ptr, _ptr],
    "sra_apply_update_f32": [_ptr, _ptr, _i32, _i64, _ptr, _ptr],
    "sra_apply_update_f64": [_ptr, _ptr, _i32, _i64, _ptr, _ptr],
    "sra_order_stat_f32": [_ptr, _i64, _i64, _i64, _i32, _ptr, _ptr],
    "sra_rows_sum_div_f32": [_ptr, _i64, _i64, _i64, ctypes.c_float, _ptr, _ptr],
    "sra_weighted_sum_f32": [_ptr, _i64, _i64, _i64, _ptr, _ptr, _ptr],
    "sra_clip_scale_running_f32": [_ptr, _i64, _i64, _i64, _ptr, ctypes.POINTER(_i64), _i32, _dbl, _ptr, _ptr, _ptr,
                                   _sz, _ptr],
    "sra_bulyan_dba_f32": [_ptr, _i64, _i64, _i64, _i32, _i32, _ptr, _ptr, _ptr, _ptr, _sz, _ptr],
}
_RESTYPES = {"sra_last_error": ctypes.c_char_p}

_lock = threading.Lock()
_lib = None


def header_symbols(path=HEADER):
    """Every ``sra_*`` function declared in include/sra.h."""
    with open(path) as fh:
        text = fh.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sra_[a-z0-9_]+)\s*\(", text)))


def load(path=None):
    """Load libsra.so once (thread-safe).  torch is imported first so that the
    library binds to the HIP runtime torch already has loaded (same soname)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        try:
            import torch  # noqa: F401  (binds libamdhip64 before dlopen)
        except Exception:
            pass
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise SraLibraryError(
                "libsra.so not found at %s: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(make -C secure-robust-federated-learning_amd/csrc); there is no CPU fallback" % p)
        try:
            lib = ctypes.CDLL(p)
        except OSError as e:
            raise SraLibraryError("failed to load %s: %s" % (p, e))
        for name, args in _SIGS.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = _RESTYPES.get(name, ctypes.c_int)
        if path is None:
            _lib = lib
        return lib


def last_error():
    return load().sra_last_error().decode(errors="replace")


def query_bytes(name, *args):
    """Call a ``*_workspace_bytes`` query and return the size."""
    out = _sz(0)
    call(name, *args, ctypes.byref(out))
    return int(out.value)


def call(name, *args):
    """Call ``name`` and raise the mapped exception on a non-zero status."""
    fn = getattr(load(), name)
    rc = fn(*args)
    if rc != SRA_OK:
        exc = _EXC.get(rc, SraRuntimeError)
        raise exc("%s: %s (status %d)" % (name, last_error(), rc))
    return rc
