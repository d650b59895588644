"""CPU model of the fit kernel's fast paths (kcc_kernels.hip `fit_kernel`).

Class A (the bench's specs) reads the node integers as IEEE denormals in
round-toward--inf: qc = floor(fc * rcf) with rcf = smallest f32 >= 1/c (fc < 2^23),
qm = floor(fm * rm) (fm < 2^50), both from ONE rounding of the exact product onto the
denormal grid; `fast_qc_a` / `fast_qm` replay that and `test_class_a_*` check them.
Class B (below) uses biased FMAs.

The kernel computes floor(fc / c) and floor(fm / m) (CC:123, CC:129) without any
integer division, conversion or correction step: one fused multiply-add per quotient
with the f64 rounding mode set to round toward -inf,

    qc' = RD64(fc * rc + 2^52) = 2^52 + floor(fc * rc),  rc = smallest f64 >= 1/c
    qm' = RD64(fm * rm + 2^52) = 2^52 + floor(fm * rm),  rm = smallest f64 >= 1/m
    (fc, fm < 2^50; 1 <= c, m < 2^51)

where fc * rc is the EXACT real product (the FMA rounds once, after the add, and in
[2^52, 2^53) the ulp is 1, so rounding down is floor).  `floor_prod` replays that on
the CPU — floor of the exact product from Dekker's error-free two-product, checked
against Python's exact rationals — and the tests compare it with exact integer floor
division where the argument is tightest: exact multiples, +-1 around them, the
largest operands allowed on the fast path, powers of two and their neighbours.
"""
import numpy as np
import pytest

FC_MAX, C_MAX = 1 << 50, 1 << 51
FM_MAX, M_MAX = 1 << 50, 1 << 51


def recip_up_f64(m):
    md = np.asarray(m, np.int64).astype(np.float64)
    r = 1.0 / md
    # r*m - 1 exactly: split r*m with Dekker's product (no fma in numpy)
    low = _exact_prod_minus_one_negative(r, md)
    return np.where(low, np.nextafter(r, np.inf), r)


def _exact_prod_minus_one_negative(r, md):
    """sign(r*md - 1) < 0, exactly (Veltkamp/Dekker two-product)."""
    def split(a):
        t = a * 134217729.0  # 2^27 + 1
        hi = t - (t - a)
        return hi, a - hi
    p = r * md
    rh, rl = split(r)
    mh, ml = split(md)
    e = ((rh * mh - p) + rh * ml + rl * mh) + rl * ml  # r*md = p + e exactly
    return (p < 1.0) | ((p == 1.0) & (e < 0.0))


def _two_prod(a, b):
    """p = RN(a*b) and e with a*b = p + e exactly (Dekker; no fma in numpy)."""
    def split(x):
        t = x * 134217729.0  # 2^27 + 1
        hi = t - (t - x)
        return hi, x - hi
    p = a * b
    ah, al = split(a)
    bh, bl = split(b)
    e = ((ah * bh - p) + ah * bl + al * bh) + al * bl
    return p, e


def floor_prod(a, r):
    """floor(a * r) of the exact real product = RD64(a * r + 2^52) - 2^52, the kernel's
    v_fma_f64 in round-toward--inf mode (a < 2^50 integer-valued, r > 0)."""
    a = np.asarray(a).astype(np.float64)
    p, e = _two_prod(a, np.asarray(r, np.float64))
    fp = np.floor(p)
    # p < 2^51: a non-integer p is >= ulp(p) away from every integer and |e| <= ulp/2
    return np.where((p == fp) & (e < 0.0), fp - 1.0, fp).astype(np.int64)


def fast_qc(fc, c):
    return floor_prod(fc, recip_up_f64(c))


def fast_qm(fm, m):
    return floor_prod(fm, recip_up_f64(m))


def test_floor_prod_model_vs_rationals():
    """The numpy model of the RD FMA against exact rational arithmetic."""
    from fractions import Fraction
    rng = np.random.default_rng(5)
    a = np.concatenate([rng.integers(0, FC_MAX, 3000), rng.integers(0, 1 << 20, 3000)])
    b = np.concatenate([rng.integers(1, C_MAX, 3000), rng.integers(1, 1 << 12, 3000)])
    a = np.concatenate([a, (a[:2000] // b[:2000]) * b[:2000]])  # exact multiples
    b = np.concatenate([b, b[:2000]])
    r = recip_up_f64(b)
    got = floor_prod(a, r)
    want = [int(Fraction(int(x)) * Fraction(float(y)) // 1) for x, y in zip(a, r)]
    np.testing.assert_array_equal(got, np.array(want, np.int64))


def test_round_mode_matters():
    """With the default round-to-nearest the same biased FMA rounds the quotient to the
    NEAREST integer: the kernel's s_setreg to round-toward--inf is load-bearing."""
    fc = np.arange(1, 1 << 14, dtype=np.int64)
    c = 3
    p, e = _two_prod(fc.astype(np.float64), recip_up_f64(np.full(fc.size, c)))
    nearest = np.rint(p + e).astype(np.int64)
    assert np.count_nonzero(nearest != fc // c) > fc.size // 4
    np.testing.assert_array_equal(fast_qc(fc, np.full(fc.size, c)), fc // c)


FC_A_MAX = 1 << 23


def recip_up_f32(c):
    """Smallest f32 >= 1/c, as spec_prep computes it (via f64, then one fix-up)."""
    from fractions import Fraction
    c = np.asarray(c, np.int64)
    shape = c.shape
    c = c.ravel()
    r = (1.0 / c.astype(np.float64)).astype(np.float32)
    # exact test r*c >= 1 (c < 2^29: the f64 product is exact; above, rationals)
    small = c < (1 << 29)
    low = np.zeros(c.size, bool)
    low[small] = r[small].astype(np.float64) * c[small] < 1.0
    big = np.flatnonzero(~small)
    low[big] = [Fraction(float(r[i])) * int(c[i]) < 1 for i in big]
    return np.where(low, np.nextafter(r, np.float32(np.inf)), r).reshape(shape)


def fast_qc_a(fc, c):
    """Class A CPU quotient: RD32(fc * 2^-149 * rcf) read as an integer = floor(fc * rcf)
    (fc < 2^23 and rcf have 23 + 24 significant bits: the product is exact in f64)."""
    rcf = recip_up_f32(c).astype(np.float64)
    return np.floor(np.asarray(fc).astype(np.float64) * rcf).astype(np.int64)


def test_class_a_recip_is_smallest_upper_bound():
    from fractions import Fraction
    rng = np.random.default_rng(8)
    c = np.concatenate([np.arange(1, 3000), rng.integers(1, C_MAX, 3000),
                        [C_MAX - 1, (1 << 24) + 1, (1 << 23) - 1, 3, 6, 12]]).astype(np.int64)
    r = recip_up_f32(c)
    for x, y in zip(r, c):
        assert Fraction(float(x)) * int(y) >= 1
        assert Fraction(float(np.nextafter(x, np.float32(0)))) * int(y) < 1


def test_class_a_cpu_quotient_exact():
    rng = np.random.default_rng(11)
    cs = np.concatenate([np.arange(1, 1025), rng.integers(1, 8001, 2000),
                         rng.integers(1, C_MAX, 500),
                         np.array([(1 << k) + d for k in range(1, 24) for d in (-1, 0, 1)])])
    fcs, cc = [], []
    for c in cs:
        nmax = (FC_A_MAX - 1) // c
        n = np.unique(np.concatenate([[0, 1, nmax], rng.integers(0, nmax + 1, 16)]))
        for d in (-1, 0, 1):
            fcs.append(n * c + d)
            cc.append(np.full(n.size, c))
    fc = np.concatenate(fcs + [np.arange(FC_A_MAX - 4096, FC_A_MAX)])
    c = np.concatenate(cc + [np.full(4096, 3)])
    ok = (fc >= 0) & (fc < FC_A_MAX)
    fc, c = fc[ok], c[ok]
    assert fc.size > 100_000
    np.testing.assert_array_equal(fast_qc_a(fc, c), fc // c)


def test_class_a_bound_is_tight():
    """Past fc < 2^23 the f32 quotient fails: the node bound is load-bearing."""
    fc = np.arange(1 << 26, (1 << 26) + 20_000, dtype=np.int64)
    c = np.full(fc.size, 3)
    assert np.any(fast_qc_a(fc, c) != fc // c)


def _cpu_pairs(rng):
    cs = np.concatenate([
        np.arange(1, 4097),
        rng.integers(1, C_MAX, 20_000),
        rng.integers(1, 1 << 23, 20_000),
        [C_MAX - 1, C_MAX - 2, C_MAX - 3, (1 << 21) - 1, 1 << 21, (1 << 21) + 1],
        np.array([(1 << k) + d for k in range(1, 51) for d in (-1, 0, 1)]),
    ]).astype(np.int64)
    cs = cs[(cs >= 1) & (cs < C_MAX)]
    fcs, cc = [], []
    for c in (cs,):
        nmax = (FC_MAX - 1) // c
        for frac in (None, 0.0, 1.0):
            if frac is None:
                n = rng.integers(0, nmax + 1)
            else:
                n = (nmax * frac).astype(np.int64)
            for d in (-1, 0, 1):
                fcs.append(n * c + d)
                cc.append(c)
    fc = np.concatenate(fcs)
    c = np.concatenate(cc)
    edge = np.array([FC_MAX - 1, FC_MAX - 2, 0, 1, 2], np.int64)
    fc = np.concatenate([fc, np.repeat(edge, cs.size)])
    c = np.concatenate([c, np.tile(cs, edge.size)])
    ok = (fc >= 0) & (fc < FC_MAX)
    return fc[ok], c[ok]


def test_cpu_quotient_exact():
    rng = np.random.default_rng(2026)
    fc, c = _cpu_pairs(rng)
    assert fc.size > 200_000
    np.testing.assert_array_equal(fast_qc(fc, c), fc // c)


def test_cpu_quotient_exhaustive_small():
    # every fc < 2^12 against every c < 2^10, and the top of the fc range
    fc = np.arange(0, 1 << 12, dtype=np.int64)
    for c in range(1, 1 << 10):
        np.testing.assert_array_equal(fast_qc(fc, c), fc // c)
    fc = np.arange(FC_MAX - (1 << 14), FC_MAX, dtype=np.int64)
    for c in list(range(1, 300)) + [C_MAX - 1, 1 << 21, 3, 7, 1000, 999_999, (1 << 49) + 1]:
        np.testing.assert_array_equal(fast_qc(fc, c), fc // c)


def _mem_pairs(rng):
    ms = np.concatenate([
        rng.integers(1, M_MAX, 20_000),
        rng.integers(1, 1 << 20, 5_000),
        np.array([104_857_600, 262_144_000, 1 << 30, 3 << 30, 100_000_000, 999_999_937,
                  M_MAX - 1, M_MAX - 3, FM_MAX - 1, FM_MAX + 1]),
        np.array([(1 << k) + d for k in range(1, 51) for d in (-1, 0, 1)]),
    ]).astype(np.int64)
    ms = ms[(ms >= 1) & (ms < M_MAX)]
    nmax = (FM_MAX - 1) // ms
    fms = []
    mm = []
    for n in (rng.integers(0, nmax + 1), nmax, np.minimum(nmax, rng.integers(0, 300, ms.size)),
              np.ones_like(ms)):
        for d in (-1, 0, 1):
            fms.append(n * ms + d)
            mm.append(ms)
    fm = np.concatenate(fms)
    m = np.concatenate(mm)
    ok = (fm >= 0) & (fm < FM_MAX)
    return fm[ok], m[ok]


def test_mem_quotient_exact():
    rng = np.random.default_rng(2027)
    fm, m = _mem_pairs(rng)
    assert fm.size > 200_000
    np.testing.assert_array_equal(fast_qm(fm, m), fm // m)


def test_recips_are_smallest_upper_bounds():
    rng = np.random.default_rng(1)
    m = np.concatenate([np.arange(1, 5000), rng.integers(1, M_MAX, 50_000)]).astype(np.int64)
    rm = recip_up_f64(m)
    assert not np.any(_exact_prod_minus_one_negative(rm, m.astype(np.float64)))
    assert np.all(_exact_prod_minus_one_negative(np.nextafter(rm, 0.0), m.astype(np.float64)))


@pytest.mark.parametrize("seed", [0, 1])
def test_class_a_contribution_matches_oracle(seed):
    """Class A: min3(qc, qm, P), m3 == P ? cl : m3, summed — vs the C oracle."""
    from oracle import coracle
    rng = np.random.default_rng(100 + seed)
    n, s = 3_000, 40
    sc = np.concatenate([rng.integers(1, 9000, s // 2), rng.integers(1, 1 << 20, s // 2)])
    sm = np.concatenate([rng.integers(1 << 18, 1 << 37, s // 2), rng.integers(1 << 18, M_MAX, s // 2)])
    k = rng.integers(0, 300, n)
    j = rng.integers(0, s, n)
    fc = np.minimum(k * sc[j] + rng.integers(-1, 2, n), FC_A_MAX - 1).clip(0)
    fm = np.minimum(k * sm[j] + rng.integers(-1, 2, n), FM_MAX - 1).clip(0)
    P = k + rng.integers(-2, 3, n)
    pc = rng.integers(0, 300, n)
    qc = fast_qc_a(fc[:, None], sc[None, :])
    qm = fast_qm(fm[:, None], sm[None, :])
    assert qm.max() < 2**32                                  # the low dword is all of qm
    Penc = np.maximum(P, 0)[:, None]                         # node_prep: P <= 0 -> 0
    m3 = np.minimum(np.minimum(qc, qm), Penc)               # v_min3_u32
    contrib = np.where(m3 == Penc, (P - pc)[:, None], m3)   # v_cmp_eq + v_cndmask
    zero = np.zeros(n, np.int64)
    ot, oe = coracle.fit(fc.astype(np.uint64), fm, P, pc, zero.astype(np.uint64), zero,
                         sc.astype(np.uint64), sm.astype(np.int64))
    assert not oe.any()
    np.testing.assert_array_equal(contrib.sum(axis=0), ot)


@pytest.mark.parametrize("seed", [0, 1])
def test_fast_contribution_matches_oracle(seed):
    """Whole fast-path contribution (min, pod clamp, sum) vs the C oracle."""
    from oracle import coracle
    rng = np.random.default_rng(seed)
    n, s = 3_000, 40
    sc = np.concatenate([rng.integers(1, 1 << 23, s // 2), rng.integers(1, 9000, s // 2)])
    sm = np.concatenate([rng.integers(1, 1 << 37, s // 2), rng.integers(1, M_MAX, s // 2)])
    k = rng.integers(0, 300, n)
    j = rng.integers(0, s, n)
    fc = np.minimum(k * sc[j] + rng.integers(-1, 2, n), FC_MAX - 1).clip(0)
    fm = np.minimum(k * sm[j] + rng.integers(-1, 2, n), FM_MAX - 1).clip(0)
    P = k + rng.integers(-2, 3, n)
    pc = rng.integers(0, 300, n)
    qc = fast_qc(fc[:, None], sc[None, :])          # x' - 2^52 of the kernel, exact
    qm = fast_qm(fm[:, None], sm[None, :])
    x = np.minimum(qc, qm)                          # v_min_f64 of the biased values
    low32 = (x & 0xFFFFFFFF).astype(np.uint32).view(np.int32).astype(np.int64)
    contrib = np.where(x >= P[:, None], (P - pc)[:, None], low32)  # v_cmp_f64 + v_cndmask
    tot = contrib.sum(axis=0)
    zero = np.zeros(n, np.int64)
    ot, oe = coracle.fit(fc.astype(np.uint64), fm, P, pc, zero.astype(np.uint64), zero,
                         sc.astype(np.uint64), sm.astype(np.int64))
    assert not oe.any()
    np.testing.assert_array_equal(tot, ot)
