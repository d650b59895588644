"""ctypes binding of libkcc.so (include/kcc.h).

The product path is the HIP library: if libkcc.so is missing or cannot be loaded
this module raises immediately — there is no Python or CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libkcc.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "kcc.h")

KCC_OK = 0
KCC_EINVAL = -1
KCC_ENOMEM = -2
KCC_EHIP = -3
KCC_ENODEV = -4
KCC_ERCCL = -5
KCC_EFAULT = -6
ERROR_NAMES = {
    KCC_EINVAL: "KCC_EINVAL", KCC_ENOMEM: "KCC_ENOMEM", KCC_EHIP: "KCC_EHIP",
    KCC_ENODEV: "KCC_ENODEV", KCC_ERCCL: "KCC_ERCCL", KCC_EFAULT: "KCC_EFAULT",
}
# spec_err values (include/kcc.h KCC_SPEC_*)
KCC_SPEC_OK = 0
KCC_SPEC_DIVZERO = 1
KCC_SPEC_FAULT = 2

_i64, _i32, _int, _vp, _dbl = C.c_int64, C.c_int32, C.c_int, C.c_void_p, C.c_double

# symbol -> (restype, argtypes); pointers are passed as c_void_p
SIGNATURES = {
    "kcc_abi_version": (_int, []),
    "kcc_set_allreduce_verify": (_int, [_vp, _int]),
    "kcc_build_info": (C.c_char_p, []),
    "kcc_create": (_int, [C.POINTER(_vp), _int, _int]),
    "kcc_destroy": (None, [_vp]),
    "kcc_last_error": (C.c_char_p, [_vp]),
    "kcc_create_error": (C.c_char_p, []),
    "kcc_reserve": (_int, [_vp, _i64, _i64, _i64]),
    "kcc_reduce_requests": (_int, [_vp, _i64, _i64] + [_vp] * 9),
    "kcc_reduce_requests_async": (_int, [_vp, _i64, _i64] + [_vp] * 10),
    "kcc_fit": (_int, [_vp, _i64] + [_vp] * 6 + [_i64] + [_vp] * 4),
    "kcc_capacity": (_int, [_vp, _i64, _i64] + [_vp] * 7 + [_i64] + [_vp] * 4),
    "kcc_fit_partial_async": (_int, [_vp, _i64] + [_vp] * 6 + [_i64] + [_vp] * 4),
    "kcc_fit_prepare_async": (_int, [_vp, _i64] + [_vp] * 6 + [_i64] + [_vp] * 4),
    "kcc_fit_run_async": (_int, [_vp, _i64, _i64, _vp, _vp]),
    "kcc_fit_finalize_async": (_int, [_vp, _i64, _vp, _vp, _vp, _vp]),
    "kcc_fit_async": (_int, [_vp, _i64] + [_vp] * 6 + [_i64] + [_vp] * 5),
    "kcc_capacity_partial_async": (_int, [_vp, _i64, _i64] + [_vp] * 10 + [_i64] + [_vp] * 3
                                   + [_int, _vp]),
    "kcc_capacity_async": (_int, [_vp, _i64, _i64] + [_vp] * 10 + [_i64] + [_vp] * 5),
    "kcc_set_node_shards": (_int, [_vp, _int]),
    "kcc_set_fit_dense": (_int, [_vp, _int]),
    "kcc_set_clamp_in_fit": (_int, [_vp, _int]),
    "kcc_clamp_in_fit_used": (_int, [_vp, C.POINTER(C.c_int)]),
    "kcc_fit_stream_rows": (_int, [_vp, C.POINTER(_i64)]),
    "kcc_reduce_faults": (_int, [_vp, C.POINTER(_i64)]),
    "kcc_clear_faults": (_int, [_vp]),
    "kcc_comm_unique_id": (_int, [_vp]),
    "kcc_comm_init": (_int, [_vp, _vp, _int, _int]),
    "kcc_allreduce_partial_async": (_int, [_vp, _i64, _vp, _vp]),
    "kcc_p2p_export": (_int, [_vp, _int, _i64, _vp]),
    "kcc_p2p_open": (_int, [_vp, _int, _vp]),
    "kcc_exchange_finalize_async": (_int, [_vp, _i64, _vp, _vp, _vp, _vp]),
    "kcc_p2p_faults": (_int, [_vp, C.POINTER(_i64)]),
    "kcc_profile_enable": (_int, [_vp, _int]),
    "kcc_profile_read": (_int, [_vp] + [C.POINTER(_dbl), C.POINTER(_i64)] * 2),
    "kcc_last_slow_fraction": (_dbl, [_vp]),
    "kcc_fit_slow_pairs": (_int, [_vp, C.POINTER(_i64), C.POINTER(_i64)]),
    "kcc_parse_cpu_millis": (_int, [_vp, _i64, _vp, _i64, _vp, _vp, _vp]),
    "kcc_parse_bytes": (_int, [_vp, _i64, _vp, _i64, _vp, _vp, _vp]),
    "kcc_parse_quantity": (_int, [_vp, _i64, _vp, _i64, _vp, _vp, _vp]),
    "kcc_parse_quantity_async": (_int, [_vp, _i64, _vp, _i64, _vp, _vp, _vp, _vp]),
    "kcc_parse_cpu_millis_async": (_int, [_vp, _i64, _vp, _i64, _vp, _vp, _vp, _vp]),
    "kcc_parse_bytes_async": (_int, [_vp, _i64, _vp, _i64, _vp, _vp, _vp, _vp]),
    "kcc_reduce_requests_keyed": (_int, [_vp, _i64, _i64] + [_vp] * 9),
    "kcc_reduce_requests_keyed_async": (_int, [_vp, _i64, _i64] + [_vp] * 10),
    "kcc_count_by_key": (_int, [_vp, _i64, _i64, _vp, _vp]),
    "kcc_count_by_key_async": (_int, [_vp, _i64, _i64, _vp, _vp, _vp]),
    "kcc_fit_rows": (_int, [_vp, _i64] + [_vp] * 6 + [C.c_uint64, _i64, _vp, _vp]),
    "kcc_pod_requests": (_int, [_vp, _i64, _i64, _i64] + [_vp] * 11),
    "kcc_pod_requests_async": (_int, [_vp, _i64, _i64, _i64] + [_vp] * 12),
    "kcc_reduce_requests_pods": (_int, [_vp, _i64, _i64, _i64, _i64] + [_vp] * 12),
}

# per-string status of kcc_parse_* (include/kcc.h)
KCC_PARSE_OK = 1
KCC_PARSE_ERR = 0
KCC_PARSE_UNSUPPORTED = -1
KCC_PARSE_BADOFF = -2


def header_symbols(path: str = HEADER_PATH) -> list[str]:
    """Every function the C-ABI header declares."""
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(kcc_[a-z0-9_]+)\s*\(", text)))


def header_arities(path: str = HEADER_PATH) -> dict[str, int]:
    """Number of parameters of every function the C-ABI header declares."""
    text = re.sub(r"/\*.*?\*/", "", open(path).read(), flags=re.S)
    out = {}
    for m in re.finditer(r"\b(kcc_[a-z0-9_]+)\s*\(([^;{]*?)\)\s*;", text, flags=re.S):
        params = m.group(2).strip()
        out[m.group(1)] = 0 if params in ("", "void") else params.count(",") + 1
    return out


def load(path: str = LIB_PATH) -> C.CDLL:
    if not os.path.exists(path):
        raise ImportError(
            f"libkcc.so not found at {path}: build it with "
            "`make -C kubernetesclustercapacity_amd/csrc` (or __graft_entry__.build()). "
            "There is no CPU fallback.")
    lib = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


_LIBS: dict[str, C.CDLL] = {}


def lib(path: str | None = None) -> C.CDLL:
    """The release libkcc.so, or (path) another build of it — the fault-path test build
    (libkcc_faultdiag.so) — each loaded once."""
    p = os.path.abspath(path or LIB_PATH)
    if p not in _LIBS:
        _LIBS[p] = load(p)
    return _LIBS[p]
