"""Quantity-string conversion: convertCPUToMilis (CC:301-319) and
bytefmt.ToBytes (BF:75-105) over packed string batches.

CPU tests pin the device algorithm (tests/parse_model.py, a step-by-step restatement of
kcc_parse.hip) to the C oracle and to exact rational rounding; GPU tests call the
kernels through the C-ABI (kcc_parse_*) and require bit-exact values and statuses.
"""
import os
from fractions import Fraction

import numpy as np
import pytest

from kubernetesclustercapacity_amd import quantity
from oracle import coracle
from tests import parse_model as pm

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "parse.npz")

CPU_KATS = [b"200m", b"2", b"250m", b"0", b"+3", b"0.5", b"2k", b"500u", b"", b"m", b"-100m",
            b"9223372036854775807m", b"9223372036854775808m", b"-9223372036854775808m",
            b"-9223372036854775809m", b"9223372036854775807", b"9223372036854776", b"1mm",
            b"1 m", b" 1", b"00000000000000000000000000000250m", b"-0", b"+", b"-m", b"1_000",
            b"12345678901234567890", b"\x00", b"1\x00m"]
BYTES_KATS = [b"250mb", b"500mb", b"100mb", b"16331524Ki", b"16Gi", b"1Ti", b"1", b"1.5G",
              b"1GIB", b"  2 KB ", b"  2KB ", b"0.5B", b"0mb", b"-1mb", b"1e3MB", b"100M",
              b"7b", b"1.0000000001K", b".5K", b"5.K", b"99999999999T", b".", b"+.5k",
              b"1.2.3k", b"\t64Mi\n", b"1kib", b"1KIB ", b"3mi", b"3gi", b"1BB", b"1Mx",
              b"0.000000000000000000001T", b"1" + b"0" * 308 + b"B", b"1" + b"0" * 309 + b"B",
              b"1" + b"0" * 307 + b"B", b"0." + b"0" * 322 + b"1B", b"0." + b"0" * 323 + b"1B",
              b"0." + b"0" * 321 + b"1B", b"1234567890123456789012345B",
              b"1.234567890123456789012345B", b"12345678901234567890000000.000B",
              b"9007199254740993B", b"9007199254740993.5B", b"0.1B", b"0.3K",
              b"18446744073709551615B", b"9223372036854775807B", b"9223372036854775808B",
              b"8589934591.9999999999K", b"1.00000000000000000000000000000000000000001K",
              b"123456789012345678.9K", b"0.00000000000000000000000000000000000001T",
              b"0.000000000000000000000000000000000000001T"]


def fuzz_corpus(n, seed):
    rng = np.random.default_rng(seed)
    alpha = np.frombuffer(b"0123456789012345678901234567890123456789..+-mMkKgGiIbBtTeE  \t_x",
                          np.uint8)
    out = []
    for _ in range(n):
        L = int(rng.integers(0, 24))
        out.append(bytes(rng.choice(alpha, L)))
    return out


def decimal_corpus(n, seed):
    """Structured decimals: 0-25 integer digits, optional point and 0-45 fraction digits,
    leading zeros, a valid or near-valid multiple."""
    rng = np.random.default_rng(seed)
    sufs = [b"B", b"K", b"KB", b"KI", b"KIB", b"M", b"MB", b"MI", b"MIB", b"G", b"GB", b"GIB",
            b"T", b"TB", b"TIB", b"m", b"mb", b"ki", b"Mi", b"Gi", b"k"]
    out = []
    for _ in range(n):
        ni = int(rng.integers(0, 26))
        nf = int(rng.integers(0, 46)) if rng.random() < 0.7 else 0
        ip = "".join(str(int(d)) for d in rng.integers(0, 10, ni))
        if rng.random() < 0.2:
            ip = "0" * int(rng.integers(1, 5)) + ip
        fp = "".join(str(int(d)) for d in rng.integers(0, 10, nf))
        if rng.random() < 0.3 and nf:
            fp = "0" * int(rng.integers(1, 30)) + fp
        s = ip + ("." + fp if nf or rng.random() < 0.1 else "")
        if rng.random() < 0.05:
            s = "-" + s
        out.append(s.encode() + sufs[int(rng.integers(0, len(sufs)))])
    return out


def cpu_corpus():
    rng = np.random.default_rng(5)
    vals = rng.integers(0, 1 << 63, 2000, dtype=np.int64)
    extra = [str(int(v)).encode() + (b"m" if i % 2 else b"") for i, v in enumerate(vals)]
    return CPU_KATS + fuzz_corpus(3000, 11) + extra


def bytes_corpus():
    return BYTES_KATS + fuzz_corpus(3000, 12) + decimal_corpus(6000, 13)


# ---- CPU: the algorithm against the oracle ---------------------------------------
def test_model_cpu_millis_matches_oracle():
    strs = cpu_corpus()
    buf, off = quantity.pack_strings(strs)
    ov, os_ = coracle.parse_cpu_millis(buf, off)
    for s, v, st in zip(strs, ov, os_):
        mv, mst = pm.cpu_millis(s)
        assert (mv, mst) == (int(v), int(st)), s


def test_model_to_bytes_matches_oracle():
    strs = bytes_corpus()
    buf, off = quantity.pack_strings(strs)
    ov, os_ = coracle.parse_bytes(buf, off)
    unsupported = 0
    for s, v, st in zip(strs, ov, os_):
        mv, mst = pm.to_bytes(s)
        if mst == pm.UNSUPPORTED:
            unsupported += 1
            continue
        assert (mv, mst) == (int(v), int(st)), s
    # the exact device domain covers all but the designed edge cases
    assert unsupported < 0.01 * len(strs)


def test_model_unsupported_only_at_designed_edges():
    assert pm.to_bytes(b"1" + b"0" * 308 + b"B")[1] == pm.UNSUPPORTED      # 10^308: < MaxFloat64?
    assert pm.to_bytes(b"0." + b"0" * 323 + b"1B")[1] == pm.UNSUPPORTED    # 1e-324 vs 2^-1075
    assert pm.to_bytes(b"0." + b"0" * 322 + b"1B") == (0, pm.OK)           # 1e-323 > 2^-1075
    assert pm.to_bytes(b"1.234567890123456789012345B") == (1, pm.OK)  # > 19 digits, decided
    # > 19 significant digits straddling a rounding boundary: 2^-1 + 2^-54 (a tie) + 1e-30
    tie = Fraction(1, 2) + Fraction(1, 2 ** 54)
    digits = str(tie.numerator * 10 ** 60 // tie.denominator)  # 0.5000...0555 x 10^60
    assert pm.to_bytes(("0." + digits + "1B").encode())[1] == pm.UNSUPPORTED
    assert pm.to_bytes(b"1234567890123456789012345B") == (pm.I64_MIN, pm.OK)
    assert pm.to_bytes(b"1.00000000000000000000B") == (1, pm.OK)  # trailing zeros are exact


def test_div_pow10_correctly_rounded():
    rng = np.random.default_rng(3)
    for _ in range(4000):
        D = int(rng.integers(1, 10 ** 18)) * int(rng.integers(1, 10))
        k = int(rng.integers(1, 39))
        assert pm.div_pow10_rn(D, k) == float(Fraction(D, 10 ** k)), (D, k)
    # halfway-adjacent cases: D / 10^k within a few ulp of a tie
    for k in (23, 25, 30, 38):
        for m in range(1, 200):
            x = Fraction(m * 2 + 1, 2 ** 60)  # exact binary ties scaled
            D = int(x * 10 ** k)
            if 0 < D < 10 ** 19:
                assert pm.div_pow10_rn(D, k) == float(Fraction(D, 10 ** k))


def test_oracle_batch_equals_single():
    strs = [s for s in BYTES_KATS if b"\x00" not in s]
    buf, off = quantity.pack_strings(strs)
    ov, os_ = coracle.parse_bytes(buf, off)
    for s, v, st in zip(strs, ov, os_):
        assert coracle.to_bytes(s.decode("latin-1")) == (int(v), bool(st))
    strs = [s for s in CPU_KATS if b"\x00" not in s]
    buf, off = quantity.pack_strings(strs)
    cv, cs = coracle.parse_cpu_millis(buf, off)
    for s, v, st in zip(strs, cv, cs):
        assert coracle.convert_cpu_to_milis(s.decode("latin-1")) == (int(v), bool(st))


def test_quantity_string_format():
    rng = np.random.default_rng(8)
    m = np.concatenate([rng.integers(0, 10 ** 7, 5000), [0, 1000, 1500, 2000, 999, 10 ** 18]])
    buf, off = quantity.cpu_quantity_strings(m.astype(np.uint64))
    got = quantity.unpack_strings(buf, off)
    want = [(str(v // 1000) if v % 1000 == 0 else f"{v}m").encode() for v in m.tolist()]
    assert got == want
    b = np.concatenate([rng.integers(0, 1 << 45, 3000) * 1024, rng.integers(0, 1 << 40, 3000),
                        [0, 1024, 1 << 30, 16 << 30, 5 << 40, 3 << 60]]).astype(np.uint64)
    buf, off = quantity.memory_quantity_strings(b)
    got = quantity.unpack_strings(buf, off)
    sufs = ["", "Ki", "Mi", "Gi", "Ti", "Pi", "Ei"]
    for v, g in zip(b.tolist(), got):
        k = 0
        while v and k < 6 and v % (1 << (10 * (k + 1))) == 0:
            k += 1
        assert g == f"{v >> (10 * k)}{sufs[k]}".encode()


def test_golden_parse_fixture():
    """tests/golden/parse.npz (made by tests/golden/gen_golden.py from the hand KATs and
    seeded corpora) against the oracle."""
    z = np.load(GOLDEN)
    v, s = coracle.parse_cpu_millis(z["cpu_buf"], z["cpu_off"])
    assert np.array_equal(v, z["cpu_val"]) and np.array_equal(s, z["cpu_st"])
    v, s = coracle.parse_bytes(z["mem_buf"], z["mem_off"])
    assert np.array_equal(v, z["mem_val"]) and np.array_equal(s, z["mem_st"])


# ---- GPU: the kernels through the C-ABI ---------------------------------------------
@pytest.fixture(scope="module")
def eng():
    from tests.conftest import init_torch_first
    init_torch_first()
    from kubernetesclustercapacity_amd import CapacityEngine
    with CapacityEngine(0, 1) as e:
        yield e


@pytest.mark.gpu
def test_gpu_cpu_millis_bit_exact(eng):
    strs = cpu_corpus()
    buf, off = quantity.pack_strings(strs)
    gv, gs = eng.convert_cpu_to_milis((buf, off))
    ov, os_ = coracle.parse_cpu_millis(buf, off)
    assert np.array_equal(gs, os_)
    assert np.array_equal(gv, ov)


@pytest.mark.gpu
def test_gpu_to_bytes_bit_exact(eng):
    strs = bytes_corpus()
    buf, off = quantity.pack_strings(strs)
    gv, gs = eng.to_bytes((buf, off))
    ov, os_ = coracle.parse_bytes(buf, off)
    model = [pm.to_bytes(s) for s in strs]
    assert [int(x) for x in gs] == [m[1] for m in model]
    assert [int(x) for x in gv] == [m[0] for m in model]
    sup = gs != pm.UNSUPPORTED
    assert np.array_equal(gs[sup], os_[sup]) and np.array_equal(gv[sup], ov[sup])


@pytest.mark.gpu
def test_gpu_golden_fixture(eng):
    z = np.load(GOLDEN)
    v, s = eng.convert_cpu_to_milis((z["cpu_buf"], z["cpu_off"]))
    assert np.array_equal(v, z["cpu_val"]) and np.array_equal(s, z["cpu_st"])
    v, s = eng.to_bytes((z["mem_buf"], z["mem_off"]))
    sup = s != pm.UNSUPPORTED
    assert np.array_equal(v[sup], z["mem_val"][sup]) and np.array_equal(s[sup], z["mem_st"][sup])


@pytest.mark.gpu
def test_gpu_long_strings_global_path(eng):
    """Workgroups whose character span exceeds the LDS stage read global memory."""
    rng = np.random.default_rng(21)
    strs = []
    for i in range(5000):
        if i % 7 == 0:
            strs.append(b"0" * int(rng.integers(100, 3000)) + b"250m")
        else:
            strs.append(str(int(rng.integers(0, 10 ** 6))).encode() + b"m")
    buf, off = quantity.pack_strings(strs)
    gv, gs = eng.convert_cpu_to_milis((buf, off))
    ov, os_ = coracle.parse_cpu_millis(buf, off)
    assert np.array_equal(gs, os_) and np.array_equal(gv, ov)
    mstrs = [b" " * int(rng.integers(0, 4000)) + b"16331524Ki" if i % 5 == 0 else b"64Mi"
             for i in range(3000)]
    buf, off = quantity.pack_strings(mstrs)
    gv, gs = eng.to_bytes((buf, off))
    ov, os_ = coracle.parse_bytes(buf, off)
    assert np.array_equal(gs, os_) and np.array_equal(gv, ov)


@pytest.mark.gpu
def test_gpu_edge_sizes(eng):
    for n in (0, 1, 1023, 1024, 1025, 4097):
        strs = [f"{i}m".encode() for i in range(n)]
        buf, off = quantity.pack_strings(strs)
        gv, gs = eng.convert_cpu_to_milis((buf, off))
        assert gv.size == n and np.array_equal(gv, np.arange(n, dtype=np.uint64))
        assert (gs == 1).all()
    # unaligned tail: total bytes not a multiple of 4, no padding handed over
    buf, off = quantity.pack_strings([b"1", b"22", b"333m"])
    gv, gs = eng.convert_cpu_to_milis((buf[:int(off[-1])].copy(), off))
    assert gv.tolist() == [1000, 22000, 333] and (gs == 1).all()


@pytest.mark.gpu
def test_gpu_async_bad_offsets(eng):
    import torch
    buf, off = quantity.pack_strings([b"1", b"2", b"3"])
    off = off.copy()
    off[2] = 1000  # past n_bytes
    d_buf = torch.from_numpy(buf).cuda()
    d_off = torch.from_numpy(off).cuda()
    out = torch.zeros(3, dtype=torch.int64, device="cuda")
    st = torch.zeros(3, dtype=torch.int8, device="cuda")
    eng.parse_cpu_millis_async(d_buf, d_off, out, st)
    torch.cuda.synchronize()
    assert st.cpu().tolist() == [1, -2, -2]
    assert out.cpu().tolist() == [1000, 0, 0]


@pytest.mark.gpu
def test_gpu_c4_round_trip():
    """C4 scale (1M nodes, 20M pods): every container's canonical cpu string parses back
    to its request (size-independent property), node memory strings to ToBytes'
    values (Ki/Mi multiples exact, Gi/Ti multiples 0 — the reference's quirk)."""
    from kubernetesclustercapacity_amd import CapacityEngine, synth
    c = synth.make_cluster(1_000_000, 20_000_000, seed=20261019)
    buf, off = quantity.cpu_quantity_strings(c.cpu_req)
    with CapacityEngine(0, 1) as e:
        v, s = e.convert_cpu_to_milis((buf, off))
        assert (s == 1).all() and np.array_equal(v, c.cpu_req)
        mb, mo = quantity.memory_quantity_strings(c.alloc_mem.astype(np.uint64))
        v, s = e.to_bytes((mb, mo))
    ov, os_ = coracle.parse_bytes(mb, mo)
    assert np.array_equal(v, ov) and np.array_equal(s, os_)


# ---- resource.Quantity.Value() (CC:285-286; parity unpinned) --------------------------
from tests import quantity_model as qm  # noqa: E402

QTY_KATS = [("128Mi", 134217728), ("1G", 10 ** 9), ("1.5Gi", 1610612736), ("100m", 1),
            ("0.1Ki", 103), ("-100m", -1), ("1e3", 1000), ("1E3", 1000), ("1E", 10 ** 18),
            ("0", 0), ("-", 0), ("000", 0), ("9223372036854775807", (1 << 63) - 1),
            ("1.G", 10 ** 9), (".5", 1), ("1.5", 2), ("+1", 1), ("-1.5", -2),
            ("-922337203685477580", -922337203685477580), ("-1Gi", -(1 << 30)),
            ("-0.0", 0), ("9.223372036854775807E", (1 << 63) - 1),
            ("1e-3", 1), ("12Ti", 12 << 40), ("0.5E", 5 * 10 ** 17), ("1e4294967296", 1),
            ("16331524Ki", 16723480576), ("250M", 250_000_000), ("1n", 1), ("2u", 1),
            ("3Ei", 3 << 60), ("8Ei", (1 << 63) - 1), ("0.0001Ki", 1), ("1.0e+2", 100)]
# ParseQuantity caps only binary amounts; decimal ones beyond 2^63 - 1 wrap in k8s, and a
# negative amount off its int64 fast path has an unpinned rounding: the engine reports both
# as KCC_PARSE_UNSUPPORTED
QTY_UNSUP = ["10E", "9223372036854775808", "1e19", "-1e19", "9223372036854775807.5",
             "100000000000000000000", "-1.5Ki", "-0.0000000001", "-9223372036854775807",
             "-10Ei", "9300P", "-1.0000000000000000001"]
QTY_ERRS = ["", "5e", "1ki", "1mi", "1Gib", "abc", "1.2.3", "1 Mi", "1e99999999999999999999",
            "1e", "--1", "1Mi2", "0x10"]


def qty_corpus():
    rng = np.random.default_rng(17)
    sufs = ["", "Ki", "Mi", "Gi", "Ti", "Pi", "Ei", "n", "u", "m", "k", "M", "G", "T", "P", "E",
            "e3", "E-2", "e+5", "e0", "e-12", "e18", "x", "ki", "iB"]
    out = [k for k, _ in QTY_KATS] + QTY_ERRS + QTY_UNSUP
    for _ in range(6000):
        ni = int(rng.integers(0, 22))
        nf = int(rng.integers(0, 25)) if rng.random() < 0.5 else 0
        ip = "".join(str(int(d)) for d in rng.integers(0, 10, ni))
        fp = "".join(str(int(d)) for d in rng.integers(0, 10, nf))
        sgn = rng.choice(["", "", "", "-", "+"])
        out.append(sgn + ip + ("." + fp if nf else "") + sufs[int(rng.integers(0, len(sufs)))])
    return out


def test_quantity_model_kats():
    for s, want in QTY_KATS:
        assert qm.value(s) == (want, qm.OK), s
    for s in QTY_ERRS:
        assert qm.value(s)[1] == qm.ERR, s
    for s in QTY_UNSUP:
        assert qm.value(s) == (0, qm.UNSUP), s


@pytest.mark.gpu
def test_gpu_quantity_value(eng):
    strs = qty_corpus()
    gv, gs = eng.quantity_value(strs)
    unsupported = 0
    for s, v, st in zip(strs, gv, gs):
        want = qm.value(s)
        if st == -1 and want[1] != qm.UNSUP:  # binary fraction beyond 19 significant digits
            unsupported += 1
            assert s.endswith("i") and "." in s, s
            continue
        assert (int(v), int(st)) == want, s
    assert unsupported < 0.1 * len(strs)  # the corpus is rich in 20+ digit binary fractions


def qty_fast_corpus():
    """The register fast path of parse_quantity_kernel: 1-14 plain digits (leading zeros
    included) with no suffix or an integral one, at every byte alignment, the 2^63 - 1 cap
    boundaries, and near-misses that must fall back to the general parser."""
    rng = np.random.default_rng(23)
    sufs = ["", "k", "M", "G", "T", "P", "E", "Ki", "Mi", "Gi", "Ti", "Pi", "Ei"]
    out = []
    for d in range(1, 15):
        for s in sufs:
            for _ in range(6):
                digs = "".join(str(int(x)) for x in rng.integers(0, 10, d))
                out.append(digs + s)
            out.append("9" * d + s)
            out.append("0" * d + s)
    out += ["7Ei", "8Ei", "8191Pi", "8192Pi", "9223372036854", "9223372036854k",
            "9223372E", "9223373T", "10E", "9224P", "9223372036854T", "1K", "1ki", "1Ei0", "Ki", "k", "1.5Gi", "+1Gi", "-1Gi",
            "1e3", "1m", "1 ", " 1", "1Kib", "12345678901234",
            # characters beside '0'..'9' in the byte table, inside the digits and last
            "12:4Mi", "1/2G", "99a", "1:", "/1", "9\x7f9", "12345678:1", "1234567890/23",
            "123456789012Ki", "1234567890123Ki", "123456789012M", "1234567890123", "0Ki", "0E"]
    return out


@pytest.mark.gpu
def test_gpu_quantity_fast_path(eng):
    strs = qty_fast_corpus()
    for shift in range(4):  # every start alignment of the first string
        batch = ["x" * shift] + strs
        gv, gs = eng.quantity_value(batch)
        for s, v, st in zip(batch[1:], gv[1:], gs[1:]):
            assert (int(v), int(st)) == qm.value(s), (shift, s)


def _qty_class(ch):
    """kcc_parse.hip qty_class: bit 7 digit, bits 0-2 k M G T P E, bits 3-5 K M G T P E, bit 6 'i'."""
    if 48 <= ch <= 57:
        return 0x80
    return {ord("i"): 0x40, ord("k"): 1, ord("K"): 1 << 3, ord("M"): 2 | 2 << 3,
            ord("G"): 3 | 3 << 3, ord("T"): 4 | 4 << 3, ord("P"): 5 | 5 << 3,
            ord("E"): 6 | 6 << 3}.get(ch, 0)


def qty_fast2_model(s: bytes, tail: bytes):
    """Bit-level restatement of the kernel's register path (kcc_parse.hip qty_fast2) on the
    16 bytes a lane holds (the string, then `tail`: whatever follows it in the buffer):
    -> (accepted, value, status).  Rejected strings go to the general parser."""
    M64, MAXV = (1 << 64) - 1, (1 << 63) - 1
    L = len(s)
    A = int.from_bytes((s + tail)[:16].ljust(16, b"\0"), "little")
    a = [(A >> (32 * j)) & 0xffffffff for j in range(4)]
    p = L - 2 if L >= 2 else 0
    pair = (A >> (8 * p)) & 0xffff
    z = (pair >> 8) & 0xff if L >= 2 else pair & 0xff
    y = pair & 0xff if L >= 2 else 0
    zc, yc = _qty_class(z), _qty_class(y)
    binary = bool(zc & 0x40) and bool(yc & 0x38)
    zd = zc & 7
    dec = not binary and zd != 0
    dig = bool(zc & 0x80)
    d = L - (2 if binary else (1 if dec else 0))
    ZZ = 0x3030303030303030
    l64, h64 = ((a[1] << 32) | a[0]) ^ ZZ, ((a[3] << 32) | a[2]) ^ ZZ
    sh = (128 - 8 * d) & 0xffffffff  # v_lshlrev_b64 takes the low 6 bits of the amount
    xl = (l64 << (sh & 63)) & M64
    big = sh >= 64
    th = xl if big else (((h64 << (sh & 63)) & M64) | (l64 >> ((64 - sh) & 63)))
    tl = 0 if big else xl
    t = [tl & 0xffffffff, tl >> 32, th & 0xffffffff, th >> 32]
    bad = 0
    for x in t:
        bad |= ((x + 0x76767676) & 0xffffffff) | x
    bad &= 0x80808080

    def dot4(x, w):  # v_dot4_u32_u8
        return sum(((x >> (8 * i)) & 0xff) * ((w >> (8 * i)) & 0xff) for i in range(4))

    def quad(x):
        return dot4(x, 0x010a0000) + 100 * dot4(x, 0x0000010a)

    q01 = quad(t[0]) * 10000 + quad(t[1])
    q23 = quad(t[2]) * 10000 + quad(t[3])
    D = (q01 * 100000000 + q23) & M64
    ok = (binary or dec or dig) and d >= 1 and bad == 0
    bexp = 10 * ((yc >> 3) & 7) if binary else 0
    mag = MAXV if D > (MAXV >> bexp) else (D << bexp) & M64
    st = qm.OK
    if dec:
        p10 = 1000 ** zd
        over = D > MAXV // p10
        mag, st = (0, qm.UNSUP) if over else ((D * p10) & M64, qm.OK)
    return ok, mag, st


def test_qty_fast2_model_equals_quantity_model():
    """The register path's arithmetic (one 128-bit shift right-aligning the digits, dot4
    quads, the class table) against the exact-rational Quantity model, on every string it
    accepts: 1-13 digits x every suffix x near-misses, random neighbouring bytes after the
    string (they must never change a result)."""
    rng = np.random.default_rng(41)
    sufs = ["", "k", "M", "G", "T", "P", "E", "Ki", "Mi", "Gi", "Ti", "Pi", "Ei",
            "K", "m", "i", "ki", "x", "e3", ".5", "Mi0"]
    accepted = 0
    for _ in range(40000):
        nd = int(rng.integers(0, 14))
        digs = "".join(str(int(x)) for x in rng.integers(0, 10, nd))
        if nd and rng.random() < 0.05:  # a stray character inside the digits
            k = int(rng.integers(0, nd))
            digs = digs[:k] + "a:/+-. "[int(rng.integers(0, 7))] + digs[k + 1:]
        s = (digs + sufs[int(rng.integers(0, len(sufs)))]).encode()
        if not 1 <= len(s) <= 13:
            continue
        tail = bytes(rng.integers(0, 256, 16 - len(s), dtype=np.uint8))
        ok, v, st = qty_fast2_model(s, tail)
        if not ok:
            continue
        accepted += 1
        want = qm.value(s.decode())
        assert ((v - (1 << 64)) if v >> 63 else v, st) == want, s
    assert accepted > 15000
    # the cap boundaries and the longest accepted forms
    for s in ["8191Pi", "8192Pi", "7Ei", "8Ei", "9223372036854", "9223372E", "9223373T",
              "1234567890123", "12345678901Ki", "0Ki", "0E", "1"]:  # (<= 13 characters)
        ok, v, st = qty_fast2_model(s.encode(), b"9" * 16)
        assert ok, s
        assert ((v - (1 << 64)) if v >> 63 else v, st) == qm.value(s), s
