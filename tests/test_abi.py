"""The C-ABI library builds, loads and exports every symbol include/kcc.h declares.

No compute call is made here (there is no GPU in the CPU suite); creating a
context without a gfx950 device must fail loudly — there is no CPU backend.
"""
import ctypes as C
import os
import subprocess

import pytest

from conftest import have_gpu
from kubernetesclustercapacity_amd import _lib


def test_header_declares_the_hot_path():
    syms = _lib.header_symbols()
    for s in ("kcc_create", "kcc_destroy", "kcc_reduce_requests", "kcc_reduce_requests_async",
              "kcc_fit", "kcc_capacity", "kcc_fit_partial_async", "kcc_fit_finalize_async",
              "kcc_fit_prepare_async", "kcc_fit_run_async", "kcc_fit_async", "kcc_last_error"):
        assert s in syms


def test_library_exports_every_header_symbol():
    assert os.path.exists(_lib.LIB_PATH), "build libkcc.so first (make -C .../csrc)"
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = [s for s in _lib.header_symbols() if s not in exported]
    assert not missing, f"declared but not exported: {missing}"


def test_binding_covers_every_header_symbol():
    assert set(_lib.header_symbols()) == set(_lib.SIGNATURES)


def test_binding_arities_match_header():
    arity = _lib.header_arities()
    assert set(arity) == set(_lib.SIGNATURES)
    wrong = {k: (arity[k], len(v[1])) for k, v in _lib.SIGNATURES.items() if arity[k] != len(v[1])}
    assert not wrong, f"header vs ctypes parameter counts: {wrong}"


def test_library_loads_and_reports_version():
    lib = _lib.load()
    assert lib.kcc_abi_version() == 2


def test_library_is_gfx950_code():
    # the .hip_fatbin bundle carries exactly one device code object, for gfx950
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"hipv4-amdgcn-amd-amdhsa--gfx950" in data
    for other in (b"--gfx942", b"--gfx90a", b"--gfx1100"):
        assert other not in data


def test_create_rejects_cpu_backend():
    lib = _lib.load()
    h = C.c_void_p()
    assert lib.kcc_create(C.byref(h), 0, 0) == _lib.KCC_EINVAL
    assert b"no CPU backend" in lib.kcc_create_error()
    assert lib.kcc_create(None, 0, 1) == _lib.KCC_EINVAL


@pytest.mark.skipif(have_gpu(), reason="a GPU is visible")
def test_create_without_gpu_fails_loudly():
    from kubernetesclustercapacity_amd import CapacityEngine, KccError
    with pytest.raises(KccError):
        CapacityEngine(0, 1)


def test_null_context_is_einval():
    lib = _lib.load()
    assert lib.kcc_reserve(None, 1, 1, 1) == _lib.KCC_EINVAL
    assert lib.kcc_fit_run_async(None, 1, 1, None, None) == _lib.KCC_EINVAL
    assert lib.kcc_last_error(None) == b"NULL context"


def test_release_library_reports_release_build():
    # the product library is built with the default knobs only (csrc/Makefile refuses EXTRA
    # outside `make variant`); an experiment build would report "variant: <flags>"
    assert _lib.load().kcc_build_info() == b"release"


def test_makefile_refuses_knobs_for_the_release_library():
    csrc = os.path.join(os.path.dirname(_lib.LIB_PATH), "csrc")
    r = subprocess.run(["make", "-n", "-C", csrc, "EXTRA=-DKCC_DIAG_RED_NOSTORE"],
                       capture_output=True, text=True)
    assert r.returncode != 0 and "make variant" in (r.stdout + r.stderr)


def test_every_diagnostic_knob_is_fenced():
    # a result-breaking diagnostic knob compiles only into a variant build: every such name
    # used in the sources appears in kcc_internal.h's #error guard
    import glob
    import re
    csrc = os.path.join(os.path.dirname(_lib.LIB_PATH), "csrc")
    used = set()
    for f in glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.cpp")):
        used |= set(re.findall(r"\b(KCC_(?:DIAG|FIT_DIAG)\w*|KCC_TIMELINE)\b", open(f).read()))
    hdr = open(os.path.join(csrc, "kcc_internal.h")).read()
    guard = hdr[hdr.index("#if !defined(KCC_VARIANT_BUILD)"):hdr.index("#error")]
    missing = sorted(k for k in used if f"defined({k})" not in guard)
    assert used and not missing, f"diagnostic knobs outside the release guard: {missing}"
