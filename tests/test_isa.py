"""Static ISA checks of the gfx950 kernels (CPU: hipcc cross-compiles).

  - the fit kernel's fast loop, one 8-node FitGroup per iteration: 40 dwords of scalar
    loads (fc, fm, P), two uniform 16-B buffer loads (cl), no 64-bit integer division,
    no correction multiply, and exactly bench.FIT_VALU_PER_NODE_WAVE VALU instructions
    per node (the VALU-roofline accounting of bench.py);
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
    i = body.index(";;#ASMSTART")
    loop = body[body.rfind(".LBB", 0, i):body.index("s_cbranch", i)]
    lines = [ln.strip() for ln in loop.splitlines()
             if ln.strip() and not ln.strip().startswith(";")]
    valu = [ln for ln in lines if ln.startswith("v_")]
    group = 8  # nodes per FitGroup = per loop iteration
    width = {"s_load_dword": 1, "s_load_dwordx2": 2, "s_load_dwordx4": 4, "s_load_dwordx8": 8,
             "s_load_dwordx16": 16}
    dwords = sum(width[ln.split()[0]] for ln in lines if ln.startswith("s_load_dword"))
    assert dwords == group * 5  # fc (f64), fm (f64), P (i32) of each node
    vmem = [ln for ln in lines if ln.startswith(("global_load", "flat_load", "buffer_load"))]
    assert len(vmem) == 2 and all(ln.startswith("buffer_load_dwordx4") and ", off," in ln
                                  for ln in vmem)  # cl: uniform address, no VGPR offset
    assert len(valu) / group == pytest.approx(bench.FIT_VALU_PER_NODE_WAVE, abs=1e-9), \
        f"{len(valu)} VALU / {group} nodes: update bench.FIT_VALU_PER_NODE_WAVE"
    ops = [ln.split()[0] for ln in valu]
    assert ops.count("v_mul_f64") == 2 * group and ops.count("v_min_f64") == group
    assert ops.count("v_cvt_i32_f64") == group and ops.count("v_add3_u32") == group // 2
    assert not any(o.startswith(("v_mad", "v_fma", "v_mul_lo", "v_mul_hi")) for o in ops)


def test_no_scratch(asm):
    for m in re.finditer(r"\.private_segment_fixed_size:\s*(\d+)", asm):
        assert int(m.group(1)) == 0
