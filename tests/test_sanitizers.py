"""CPU sanitizer run (race detection / sanitizers): the C oracle and the C++ host
code built with AddressSanitizer + UndefinedBehaviorSanitizer (oracle/Makefile and
host/Makefile `asan`, every finding fatal), and the CPU suite's oracle and host tests run
against those builds in a child pytest with libasan preloaded:

  - tests/test_oracle_kat.py, tests/test_oracle_cross.py, tests/test_parse.py (CPU part):
    the oracle's fit / reduce / parsers on the KATs, the golden fixtures and seeded
    clusters (KCC_ORACLE_LIB = oracle/_build/libkcc_oracle_asan.so);
  - tests/test_host.py (CPU part): the host parsers and the CLI's flag / error paths
    (KCC_HOST_LIB = host/libkcc_host_asan.so, KCC_HOST_CLI = host/cluster_capacity_asan).

Leak detection is off (the CPython interpreter itself holds its allocations at exit);
GPU code is not sanitized (not available on this pool) — the device path is covered by
the -m gpu parity tests.
"""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _libasan():
    p = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True)
    path = p.stdout.strip()
    return path if p.returncode == 0 and os.path.isabs(path) and os.path.exists(path) else None


@pytest.mark.skipif(shutil.which("gcc") is None or _libasan() is None,
                    reason="gcc with libasan needed")
def test_oracle_and_host_under_asan_ubsan(tmp_path):
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], check=True)
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "host"), "asan"], check=True)
    env = dict(os.environ)
    env.update(
        LD_PRELOAD=_libasan(),
        ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1",
        UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
        KCC_ORACLE_LIB=os.path.join(ROOT, "oracle", "_build", "libkcc_oracle_asan.so"),
        KCC_HOST_LIB=os.path.join(ROOT, "host", "libkcc_host_asan.so"),
        KCC_HOST_CLI=os.path.join(ROOT, "host", "cluster_capacity_asan"),
        PYTHONDONTWRITEBYTECODE="1",
    )
    # the child really loads the sanitized builds (and the sanitizer runtimes)
    probe = ("import sys; sys.path.insert(0, %r); from oracle import coracle; coracle.lib(); "
             "import ctypes, os; ctypes.CDLL(os.environ['KCC_HOST_LIB']); "
             "print(open('/proc/self/maps').read())" % ROOT)
    maps = subprocess.run([sys.executable, "-c", probe], env=env, capture_output=True, text=True,
                          timeout=120)
    assert maps.returncode == 0, maps.stderr[-2000:]
    for lib in ("libkcc_oracle_asan.so", "libkcc_host_asan.so", "libasan", "libubsan"):
        assert lib in maps.stdout, lib
    tests = [os.path.join(ROOT, "tests", t) for t in
             ("test_oracle_kat.py", "test_oracle_cross.py", "test_parse.py", "test_host.py")]
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-m", "not gpu", "-p",
                        "no:cacheprovider", "-p", "no:xdist", *tests],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "runtime error" not in out and "ERROR: AddressSanitizer" not in out, out[-4000:]
    assert " passed" in out
