"""Static ISA checks of the gfx950 kernels (CPU: hipcc cross-compiles).

  - the fit kernel's class-A loop, one 8-node FitGroupA per iteration: 32 dwords of
    scalar loads (fm, fc, P) and no vector memory access, exactly
    bench.FIT_VALU_PER_NODE_WAVE VALU instructions per node (the VALU-roofline
    accounting of bench.py): packed f32 and f64 multiplies, min3, add — no division,
    no conversion, no correction step, no compare/select (the clamp is the clamp
    correction's job);
  - the class-B loop: biased f64 FMAs, 4.5 VALU instructions per node;
  - both loops run inside a round-toward--inf window of the MODE register (our two
    s_setreg writes each), and the compiler inserts no mode switch of its own;
  - f32 and f64 denormals are enabled in the kernel descriptor (class A reads
    integers as denormals);
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


def loop_of(body, marker, i=None):
    i = body.index(marker) if i is None else i
    loop = body[body.rfind(".LBB", 0, i):body.index("s_cbranch", i)]
    return [ln.strip() for ln in loop.splitlines() if ln.strip() and not ln.strip().startswith(";")]


def loops_with(body, marker):
    """Every loop body holding `marker` (once each)."""
    out, seen = [], set()
    for m in re.finditer(re.escape(marker), body):
        start = body.rfind(".LBB", 0, m.start())
        if start not in seen:
            seen.add(start)
            out.append(loop_of(body, marker, m.start()))
    return out


# fit_kernel<false>: the clamp-correction layout; fit_kernel<true>: the clamp in the fit
FIT = "fit_kernelILb0E"
FIT_NC = "fit_kernelILb1E"


WIDTH = {"s_load_dword": 1, "s_load_dwordx2": 2, "s_load_dwordx4": 4, "s_load_dwordx8": 8,
         "s_load_dwordx16": 16}
GROUP = 8  # nodes per FitGroup = per loop iteration


def check_loads(lines, dwords):
    assert sum(WIDTH[ln.split()[0]] for ln in lines if ln.startswith("s_load_dword")) == dwords
    assert not [ln for ln in lines if ln.startswith(("global_", "flat_", "buffer_", "ds_"))]


def block_before(body, marker):
    """The instructions of the basic block that ends at `marker` (an asm comment the kernel
    puts at the end of a loop body)."""
    j = body.index(marker)
    st = max(body.rfind(".LBB", 0, j), body.rfind("; %bb.", 0, j))
    return [ln.strip() for ln in body[st:j].splitlines()[1:]
            if ln.strip() and not ln.strip().startswith(";")]


FULL = "; fit: full"


def test_fit_class_a_loop(asm):
    """Class A, per 8-node group (bench.FIT_VALU_PER_NODE_WAVE = 3 VALU per node: packed f32
    and f64 multiplies, min3, add) — no division, conversion, correction, compare or select;
    no vector memory in the body."""
    import bench
    body = kernel_body(asm, FIT)
    full = block_before(body, FULL)
    assert not [ln for ln in full if ln.startswith(("global_", "flat_", "buffer_", "ds_"))]
    check_loads(loop_of(body, FULL), GROUP * 4)  # fm (f64), fc, P (u32) per node
    valu = [ln.split()[0] for ln in full if ln.startswith("v_")]
    assert len(valu) / GROUP == pytest.approx(bench.FIT_VALU_PER_NODE_WAVE, abs=1e-9), \
        f"{len(valu)} VALU / {GROUP} nodes: update bench.FIT_VALU_PER_NODE_WAVE"
    assert valu.count("v_pk_mul_f32") == GROUP // 2 and valu.count("v_mul_f64") == GROUP
    assert valu.count("v_min3_u32") == GROUP and valu.count("v_add3_u32") == GROUP // 2
    assert not any(o.startswith(("v_mad", "v_cvt", "v_fma", "v_rcp", "v_div", "v_cmp",
                                 "v_cndmask")) for o in valu)


def test_fit_class_b_loop(asm):
    (lines,) = loops_with(kernel_body(asm, FIT), "v_fma_f64")
    check_loads(lines, GROUP * 6)  # fc, fm, Pb (f64) per node
    valu = [ln for ln in lines if ln.startswith("v_")]
    assert len(valu) / GROUP == 4.5
    ops = [ln.split()[0] for ln in valu]
    assert ops.count("v_fma_f64") == 2 * GROUP and ops.count("v_min_f64") == 2 * GROUP
    assert ops.count("v_add3_u32") == GROUP // 2
    assert not any(o.startswith(("v_cvt", "v_max", "v_mul", "v_cmp", "v_cndmask")) for o in ops)


def test_fit_clamp_in_fit_loops(asm):
    """The clamp-in-fit variants (kcc_set_clamp_in_fit): class A takes each group's 8 clamp
    values by two 16-B vector loads (uniform address) so the select reads them as VGPRs:
    5.0 VALU per node (min, compare, select in place of min3); class B (scalar loads) 6.5:
    fmin, compare, a move of the clamp value into a VGPR (a gfx9 select reads one scalar
    operand at most, vcc included), select in place of two min_f64."""
    import bench
    body = kernel_body(asm, FIT_NC)
    full = block_before(body, FULL)
    assert any(ln.startswith("v_cndmask") for ln in full)
    va = [ln for ln in full if ln.startswith("v_")]
    assert len(va) / GROUP == bench.FIT_NC_VALU_PER_NODE_WAVE, f"{len(va)} VALU / {GROUP} nodes"
    (b,) = loops_with(body, "v_fma_f64")
    assert any(ln.startswith("v_cndmask") for ln in b)
    check_loads(b, GROUP * 7)
    vb = [ln for ln in b if ln.startswith("v_")]
    assert len(vb) / GROUP <= 6.5, f"{len(vb)} VALU / {GROUP} nodes"


@pytest.mark.parametrize("name", [FIT, FIT_NC])
def test_fit_round_mode_windows(asm, name):
    body = kernel_body(asm, name)
    sets = [(m.start(), m.group(1)) for m in
            re.finditer(r"s_setreg\w*\s+hwreg\(HW_REG_MODE[^)]*\),\s*(\S+)", body)]
    # (round down, back to nearest) around each of the two fast loops, nothing else
    assert [v for _, v in sets] == ["10", "0", "10", "0"], sets
    assert all("hwreg(HW_REG_MODE, 0, 4)" in body[p:p + 60] for p, _ in sets)
    windows = [(sets[0][0], sets[1][0]), (sets[2][0], sets[3][0])]
    for op in ("v_pk_mul_f32", "v_mul_f64", "v_fma_f64"):
        pos = [m.start() for m in re.finditer(op, body)]
        assert pos and all(any(a < p < b for a, b in windows) for p in pos), op


@pytest.mark.parametrize("name", [FIT, FIT_NC])
def test_denormals_enabled(asm, name):
    m = re.search(rf"^(_ZN3kcc12_GLOBAL__N_1\d+{name}\w*):", asm, re.M)
    desc = asm[asm.index(".amdhsa_kernel " + m.group(1)):]
    desc = desc[:desc.index(".end_amdhsa_kernel")]
    assert re.search(r"\.amdhsa_float_denorm_mode_32 3", desc)
    assert re.search(r"\.amdhsa_float_denorm_mode_16_64 3", desc)


# node_prep's 4096-row passes (SUB = 4: four one-row sub-steps, held to the pass's end)
# spill a few loop-invariant values, reloaded once per pass; every other kernel is
# spill-free
SCRATCH_ALLOWED = {r"node_prep_kernelILi\dELi4E": 128}


def test_no_scratch(asm):
    checked = 0
    for m in re.finditer(r"\.amdhsa_kernel (\S+)(.*?)\.end_amdhsa_kernel", asm, re.S):
        name, desc = m.group(1), m.group(2)
        size = int(re.search(r"\.amdhsa_private_segment_fixed_size (\d+)", desc).group(1))
        cap = next((c for pat, c in SCRATCH_ALLOWED.items() if re.search(pat, name)), 0)
        assert size <= cap, (name, size)
        checked += 1
    assert checked >= 10  # every kernel's descriptor was found


def test_reduce_occupancy(asm):
    """reduce_kernel<2, *> (which also carries the spec ranks' workgroups, and with node prep
    behind it its workgroups too) keeps <= 128 VGPRs: 4 waves per SIMD, the occupancy its
    8-items-per-lane tiles were measured at."""
    found = re.findall(r"\.name:\s+_ZN3kcc12_GLOBAL__N_1\d+reduce_kernelILi2ELb[01]EE\w*\n(?:.*?)\.vgpr_count:\s+(\d+)",
                       asm, re.S)
    assert len(found) == 2, found
    assert all(int(v) <= 128 for v in found), found


def _vregs(line):
    """VGPR numbers a line names (v7, v[16:19]), operands only (no comment)."""
    ops = line.split(";")[0]
    regs = set()
    for a, b in re.findall(r"\bv\[(\d+):(\d+)\]", ops):
        regs.update(range(int(a), int(b) + 1))
    regs.update(int(x) for x in re.findall(r"\bv(\d+)\b", ops))
    return regs


def test_fit_claim_result_untouched_until_drained(asm):
    """The fit's queue claim is a returning atomic issued in inline asm, so the compiler
    does not wait for it where it is issued; it believes the destination VGPR is written
    at issue.  No instruction may read or write that register between the atomic and the
    s_waitcnt vmcnt(0) that drains it: a copy would read it early, a reuse would be
    overwritten when the claim returns (advisor, round 2)."""
    lines = [ln.strip() for nm in (FIT, FIT_NC) for ln in kernel_body(asm, nm).splitlines()]
    found = 0
    for i, ln in enumerate(lines):
        m = re.match(r"global_atomic_add\s+v(\d+),.*\bsc0\b", ln)
        if not m:
            continue
        found += 1
        reg = int(m.group(1))
        for ln2 in lines[i + 1:]:
            if ln2.startswith("s_waitcnt") and "vmcnt(0)" in ln2:
                break
            if not ln2 or ln2.startswith((";", ".")):
                continue
            assert reg not in _vregs(ln2), f"v{reg} of `{ln}` touched by `{ln2}` before its wait"
        else:
            raise AssertionError(f"no s_waitcnt vmcnt(0) after `{ln}`")
    assert found >= 4  # the first claim and the loop's, in both instantiations


def test_reduce_lookback_tagged_words(asm):
    """The reduce's look-back (tagged words): each 32-bit half of a
    carried sum travels in its own 64-bit word under a tag in the high half, so a word is
    complete when its tag is there — no ready flag, no fence. Pinned: the poll loop (the one
    with s_sleep) reads the 2 x NA = 4 words as single 64-bit agent-coherent loads
    (global_load_dwordx2 ... sc1, never split into dwords); the publish and the
    clean-on-consume are 64-bit sc1 stores; the kernel has no cache invalidate / write-back
    (the acquire / release variant measured 2.3x slower and was deleted)."""
    m = re.search(r"^(_ZN3kcc12_GLOBAL__N_1\d+reduce_kernelILi2E\w*):\s*;", asm, re.M)
    body = asm[m.end():asm.index(".Lfunc_end", m.end())]  # the whole function (several exits)
    polls = []
    labels = [m.start() for m in re.finditer(r"^\.LBB\w+:", body, re.M)]
    for m in re.finditer("s_sleep", body):  # (the fused spec ranks wait too)
        loop = body[max(x for x in labels if x < m.start()):m.start()]
        loads = [ln.strip() for ln in loop.splitlines()
                 if "load" in ln and not ln.strip().startswith(";")]
        if any("dwordx2" in ln for ln in loads):
            polls.append(loads)
    assert len(polls) == 1, polls
    (loads,) = polls
    assert len(loads) == 4, loads
    assert all(ln.startswith("global_load_dwordx2") and ln.endswith("sc1") for ln in loads), loads
    assert "buffer_inv" not in body and "buffer_wbl2" not in body
    stores = [ln.strip() for ln in body.splitlines()
              if ln.strip().startswith("global_store_dwordx2") and ln.strip().endswith("sc1")]
    assert len(stores) >= 5, stores  # one publish + the four frees


# ---- node prep inside the reduce launch (reduce_kernel<2, true>) --------
# Node prep's row workgroups read the reduce's per-node sums with no release / acquire: the
# hand-off is (1) every store of a node sum (out[], the used_* arrays) at agent scope (sc1,
# through to the shared L2 and past this CU's L1), (2) an `s_waitcnt vmcnt(0)` before the
# wave's flag store, so the flag cannot become visible before the sums, and (3) node prep
# reading used_* and the flags at agent scope (sc1).  The release asm carries no source
# positions, so the checks run on the same file built with line tables (-gline-tables-only
# does not change the instructions: pinned below) and map every instruction to its
# kcc_kernels.hip line.
NPM = "reduce_kernelILi2ELb1E"
VMEM = ("global_", "buffer_", "flat_")


def _src_lines(pattern, within=None):
    src = open(SRC).read().splitlines()
    lo, hi = within if within else (0, len(src))
    if within:  # (function names -> the lines from its definition to the next top-level `}`)
        lo = next(i for i, ln in enumerate(src) if re.search(within[0], ln))
        hi = next(i for i in range(lo + 1, len(src)) if src[i].startswith("}"))
    return {i + 1 for i in range(lo, hi) if re.search(pattern, src[i])}


def _asm_with_lines(tmp_path_factory, *defines):
    out = tmp_path_factory.mktemp("isa_g") / "kcc_g.s"
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-S",
                    "--cuda-device-only", "-gline-tables-only", *defines, SRC, "-o", str(out)],
                   check=True, capture_output=True)
    return out.read_text()


@pytest.fixture(scope="module")
def asm_g(tmp_path_factory):
    return _asm_with_lines(tmp_path_factory)


def _function(asm, name):
    m = re.search(rf"^(_ZN3kcc12_GLOBAL__N_1\d+{name}\w*):\s*;", asm, re.M)
    assert m, name
    return asm[m.end():asm.index(".Lfunc_end", m.end())]


def _kernels_file_ids(asm):
    """The .file numbers of kcc_kernels.hip in a line-table build."""
    return {int(m.group(1)) for m in
            re.finditer(r'^\s*\.file\s+(\d+)\s+"[^"]*"\s+"[^"]*kcc_kernels\.hip"', asm, re.M)}


def _instrs_with_lines(body, fids=frozenset()):
    """[(source line in kcc_kernels.hip or None, instruction text)] in program order."""
    out, cur = [], None
    for ln in body.splitlines():
        s = ln.strip()
        m = re.match(r"\.loc\s+(\d+)\s+(\d+)", s)
        if m:
            cur = int(m.group(2)) if int(m.group(1)) in fids else None
            continue
        if not s or s.startswith((";", ".", "@")) or s.endswith(":"):
            continue
        out.append((cur, s.split(";")[0].strip()))
    return out


def npm_ordering_problems(asm_g):
    """What breaks node prep's hand-off in reduce_kernel<2, true>'s ISA (empty: none)."""
    fids = _kernels_file_ids(asm_g)
    assert fids, "no .file entry for kcc_kernels.hip"
    ins = _instrs_with_lines(_function(asm_g, NPM), fids)
    red = (r"void reduce_kernel\(", None)
    # (1) the node sums' stores: both branches of each store site (agent-scope atomic store /
    # plain store) and the pending block's buffer store
    store_lines = (_src_lines(r"__hip_atomic_store\(out\[k\]|^\s*else out\[k\]\[", red) |
                   _src_lines(r"raw_buffer_store_b64\(.*resF\[k\]", red))
    stores = [(l, s) for l, s in ins if l in store_lines and s.startswith(VMEM) and "store" in s]
    problems = [f"node-sum store without sc1 (line {l}): {s}" for l, s in stores
                if not s.endswith("sc1")]
    if len([s for _, s in stores if s.startswith("buffer_store_dwordx2")]) < 2 or \
            len([s for _, s in stores if s.startswith("global_store_dwordx2")]) < 3:
        problems.append(f"node-sum stores not found: {stores}")
    # (2) the per-wave flag: an s_waitcnt vmcnt(0) after the wave's last vector memory access
    flag_lines = _src_lines(r"__hip_atomic_store\(np\.sync \+ NP_FLAGS \+ w", red)
    flags = [i for i, (l, s) in enumerate(ins) if l in flag_lines and s.startswith(VMEM)]
    if not flags:
        problems.append("flag store not found")
    for i in flags:
        if not ins[i][1].startswith("global_store_dword ") or not ins[i][1].endswith("sc1"):
            problems.append(f"flag store is not a 32-bit sc1 store: {ins[i][1]}")
        for _, s in reversed(ins[:i]):
            if s.startswith("s_waitcnt") and "vmcnt(0)" in s:
                break
            if s.startswith(VMEM):
                problems.append(f"vector memory access `{s}` between the last vmcnt(0) and "
                                f"the flag store `{ins[i][1]}`")
                break
    # (3) node prep reads the sums (np_rows) and polls the flags (np_wait_rows) at agent scope
    rows = (r"void np_rows\(", None)
    used_lines = _src_lines(r"np\.used_(cpu|mem) \+ i", rows)
    loads = [s for l, s in ins if l in used_lines and s.startswith(VMEM) and "load" in s]
    if len(loads) < 2:
        problems.append(f"np_rows' used_* loads not found: {loads}")
    problems += [f"np_rows used_* load without sc1: {s}" for s in loads if not s.endswith("sc1")]
    poll_lines = _src_lines(r"np\.sync \+ NP_FLAGS \+ wi", (r"void np_wait_rows\(", None))
    polls = [s for l, s in ins if l in poll_lines and s.startswith(VMEM) and "load" in s]
    if not polls:
        problems.append("np_wait_rows' flag polls not found")
    problems += [f"flag poll without sc1: {s}" for s in polls if not s.endswith("sc1")]
    return problems


def test_npm_line_tables_same_instructions(asm, asm_g):
    """The line-table build used below has exactly the release instructions."""
    strip = lambda b: [s for _, s in _instrs_with_lines(b)]  # noqa: E731
    assert strip(_function(asm, NPM)) == strip(_function(asm_g, NPM))


def test_npm_node_sums_hand_off(asm_g):
    """Node prep inside the reduce launch: every node-sum store is sc1, every
    per-wave flag store follows an s_waitcnt vmcnt(0) with no vector memory access between,
    and node prep's used_* loads and flag polls are sc1."""
    assert npm_ordering_problems(asm_g) == []


def test_npm_hand_off_check_catches_plain_stores(tmp_path_factory):
    """The check above fails on the KCC_DIAG_NP_NOSC1 diagnostic build (node sums stored
    plainly): it reads the ISA, not the source."""
    bad = _asm_with_lines(tmp_path_factory, "-DKCC_VARIANT_BUILD", "-DKCC_DIAG_NP_NOSC1")
    problems = npm_ordering_problems(bad)
    assert any("node-sum store without sc1" in p for p in problems), problems
