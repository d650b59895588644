"""ctypes binding of the C oracle (oracle/_build/libkcc_oracle.so).

TEST INFRASTRUCTURE ONLY — loaded by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the checker; never by the product package.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# KCC_ORACLE_LIB: another build of the same oracle (the sanitizer build, oracle/Makefile asan)
LIB_PATH = os.environ.get("KCC_ORACLE_LIB") or os.path.join(_HERE, "_build", "libkcc_oracle.so")
_LIB = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        vp, i64 = C.c_void_p, C.c_int64
        L.kcco_reduce_requests.argtypes = [i64] + [vp] * 9
        L.kcco_reduce_requests.restype = None
        L.kcco_fit.argtypes = [i64] + [vp] * 6 + [i64] + [vp] * 4 + [C.c_int]
        L.kcco_fit.restype = None
        L.kcco_fit_one.argtypes = [C.c_uint64, i64, i64, i64, C.c_uint64, i64, C.c_uint64, i64,
                                   C.POINTER(C.c_int)]
        L.kcco_fit_one.restype = i64
        L.kcco_find_min.argtypes = [i64, i64]
        L.kcco_find_min.restype = i64
        L.kcco_convert_cpu_to_milis.argtypes = [C.c_char_p, C.POINTER(C.c_int)]
        L.kcco_convert_cpu_to_milis.restype = C.c_uint64
        L.kcco_to_bytes.argtypes = [C.c_char_p, C.POINTER(i64)]
        L.kcco_to_bytes.restype = C.c_int
        L.kcco_parse_cpu_millis.argtypes = [i64, vp, vp, vp, vp, C.c_int]
        L.kcco_parse_cpu_millis.restype = None
        L.kcco_parse_bytes.argtypes = [i64, vp, vp, vp, vp, C.c_int]
        L.kcco_parse_bytes.restype = None
        L.kcco_pod_requests.argtypes = [i64] + [vp] * 11
        L.kcco_pod_requests.restype = None
        _LIB = L
    return _LIB


def _p(a):
    return None if a is None else C.c_void_p(a.ctypes.data)


def reduce_requests(node_ptr, cpu_req, mem_req, cpu_lim=None, mem_lim=None):
    node_ptr = np.ascontiguousarray(node_ptr, np.int64)
    n = node_ptr.size - 1
    cpu_req = np.ascontiguousarray(cpu_req, np.uint64)
    mem_req = np.ascontiguousarray(mem_req, np.int64)
    lim = cpu_lim is not None
    cl = np.ascontiguousarray(cpu_lim, np.uint64) if lim else None
    ml = np.ascontiguousarray(mem_lim, np.int64) if lim else None
    uc, um = np.zeros(n, np.uint64), np.zeros(n, np.int64)
    lc = np.zeros(n, np.uint64) if lim else None
    lm = np.zeros(n, np.int64) if lim else None
    lib().kcco_reduce_requests(n, _p(node_ptr), _p(cpu_req), _p(mem_req), _p(cl), _p(ml),
                               _p(uc), _p(um), _p(lc), _p(lm))
    return uc, um, lc, lm


def fit(alloc_cpu, alloc_mem, alloc_pods, pod_count, used_cpu, used_mem, spec_cpu, spec_mem,
        n_threads=1):
    a = [np.ascontiguousarray(alloc_cpu, np.uint64), np.ascontiguousarray(alloc_mem, np.int64),
         np.ascontiguousarray(alloc_pods, np.int64), np.ascontiguousarray(pod_count, np.int64),
         np.ascontiguousarray(used_cpu, np.uint64), np.ascontiguousarray(used_mem, np.int64)]
    sc = np.ascontiguousarray(spec_cpu, np.uint64)
    sm = np.ascontiguousarray(spec_mem, np.int64)
    tot = np.zeros(sc.size, np.int64)
    err = np.zeros(sc.size, np.int32)
    lib().kcco_fit(a[0].size, *[_p(x) for x in a], sc.size, _p(sc), _p(sm), _p(tot), _p(err),
                   int(n_threads))
    return tot, err


def fit_one(alloc_cpu, alloc_mem, alloc_pods, pod_count, used_cpu, used_mem, spec_cpu, spec_mem):
    z = C.c_int(0)
    q = lib().kcco_fit_one(alloc_cpu, alloc_mem, alloc_pods, pod_count, used_cpu, used_mem,
                           spec_cpu, spec_mem, C.byref(z))
    return q, z.value


def convert_cpu_to_milis(s: str):
    ok = C.c_int(0)
    v = lib().kcco_convert_cpu_to_milis(s.encode(), C.byref(ok))
    return v, bool(ok.value)


def to_bytes(s: str):
    out = C.c_int64(0)
    rc = lib().kcco_to_bytes(s.encode(), C.byref(out))
    return out.value, rc == 0


def parse_cpu_millis(buf, off, n_threads=1):
    """Batch convertCPUToMilis over packed strings -> (uint64 values, int8 status)."""
    buf = np.ascontiguousarray(buf, np.uint8)
    off = np.ascontiguousarray(off, np.int64)
    n = off.size - 1
    out, st = np.zeros(n, np.uint64), np.zeros(n, np.int8)
    lib().kcco_parse_cpu_millis(n, _p(buf), _p(off), _p(out), _p(st), int(n_threads))
    return out, st


def parse_bytes(buf, off, n_threads=1):
    """Batch bytefmt.ToBytes over packed strings -> (int64 values, int8 status)."""
    buf = np.ascontiguousarray(buf, np.uint8)
    off = np.ascontiguousarray(off, np.int64)
    n = off.size - 1
    out, st = np.zeros(n, np.int64), np.zeros(n, np.int8)
    lib().kcco_parse_bytes(n, _p(buf), _p(off), _p(out), _p(st), int(n_threads))
    return out, st


def pod_requests(pod_ptr, cpu_req, mem_req, init_ptr=None, init_cpu=None, init_mem=None,
                 restartable=None, ovh_cpu=None, ovh_mem=None):
    """SURVEY §8f row 4 (opt-in scheduler request model, not the reference): per-pod
    effective requests, see kcc_oracle.h kcco_pod_requests."""
    pod_ptr = np.ascontiguousarray(pod_ptr, np.int64)
    n = pod_ptr.size - 1
    a = [np.ascontiguousarray(cpu_req, np.uint64), np.ascontiguousarray(mem_req, np.int64)]
    opt = [(init_ptr, np.int64), (init_cpu, np.uint64), (init_mem, np.int64),
           (restartable, np.uint8), (ovh_cpu, np.uint64), (ovh_mem, np.int64)]
    b = [None if x is None else np.ascontiguousarray(x, t) for x, t in opt]
    pc, pm = np.zeros(n, np.uint64), np.zeros(n, np.int64)
    lib().kcco_pod_requests(n, _p(pod_ptr), *[_p(x) for x in a], *[_p(x) for x in b],
                            _p(pc), _p(pm))
    return pc, pm
