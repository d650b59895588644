"""Static ISA checks of the gfx950 kernels (CPU: hipcc cross-compiles).

  - the fit kernel's fast loop, one 8-node FitGroup per iteration: 48 dwords of scalar
    loads (fc, fm, Pb), two uniform 16-B buffer loads (cl), no 64-bit integer division,
    no conversion, and exactly bench.FIT_VALU_PER_NODE_WAVE VALU instructions per node
    (the VALU-roofline accounting of bench.py);
  - the loop runs inside the round-toward--inf window of the f64 mode (our two
    s_setreg writes), and the compiler inserts no mode switch of its own;
  - no kernel spills to scratch.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "kubernetesclustercapacity_amd", "csrc", "kcc_kernels.hip")

pytestmark = pytest.mark.skipif(shutil.which("hipcc") is None, reason="hipcc not available")


@pytest.fixture(scope="module")
def asm(tmp_path_factory):
    out = tmp_path_factory.mktemp("isa") / "kcc.s"
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-S",
                    "--cuda-device-only", SRC, "-o", str(out)], check=True,
                   capture_output=True)
    return out.read_text()


def kernel_body(asm, name):
    m = re.search(rf"^(_ZN3kcc12_GLOBAL__N_1\d+{name}\w*):\s*;", asm, re.M)
    assert m, name
    start = m.end()
    return asm[start:asm.index("s_endpgm", start)]


def test_fit_fast_loop(asm):
    import bench
    body = kernel_body(asm, "fit_kernel")
    i = body.index("v_fma_f64")
    loop = body[body.rfind(".LBB", 0, i):body.index("s_cbranch", i)]
    lines = [ln.strip() for ln in loop.splitlines()
             if ln.strip() and not ln.strip().startswith(";")]
    valu = [ln for ln in lines if ln.startswith("v_")]
    group = 8  # nodes per FitGroup = per loop iteration
    width = {"s_load_dword": 1, "s_load_dwordx2": 2, "s_load_dwordx4": 4, "s_load_dwordx8": 8,
             "s_load_dwordx16": 16}
    dwords = sum(width[ln.split()[0]] for ln in lines if ln.startswith("s_load_dword"))
    assert dwords == group * 6  # fc, fm, Pb (f64) of each node
    vmem = [ln for ln in lines if ln.startswith(("global_load", "flat_load", "buffer_load"))]
    assert len(vmem) == 2 and all(ln.startswith("buffer_load_dwordx4") and ", off," in ln
                                  for ln in vmem)  # cl: uniform address, no VGPR offset
    assert len(valu) / group == pytest.approx(bench.FIT_VALU_PER_NODE_WAVE, abs=1e-9), \
        f"{len(valu)} VALU / {group} nodes: update bench.FIT_VALU_PER_NODE_WAVE"
    ops = [ln.split()[0] for ln in valu]
    assert ops.count("v_fma_f64") == 2 * group and ops.count("v_min_f64") == group
    assert sum(o.startswith("v_cmp_") and "_f64" in o for o in ops) == group
    assert sum(o.startswith("v_cndmask_b32") for o in ops) == group
    assert ops.count("v_add3_u32") == group // 2
    assert not any(o.startswith(("v_mad", "v_cvt", "v_mul", "v_max")) for o in ops)


def test_fit_round_mode_window(asm):
    body = kernel_body(asm, "fit_kernel")
    sets = [(m.start(), m.group(1)) for m in
            re.finditer(r"s_setreg\w*\s+hwreg\(HW_REG_MODE[^)]*\),\s*(\S+)", body)]
    assert [v for _, v in sets] == ["2", "0"], sets  # round down, then back to nearest
    fmas = [m.start() for m in re.finditer(r"v_fma_f64", body)]
    assert fmas and all(sets[0][0] < f < sets[1][0] for f in fmas)
    assert "hwreg(HW_REG_MODE, 2, 2)" in body


def test_no_scratch(asm):
    for m in re.finditer(r"\.private_segment_fixed_size:\s*(\d+)", asm):
        assert int(m.group(1)) == 0
