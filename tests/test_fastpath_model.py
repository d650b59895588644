"""CPU model of the fit kernel's fast path (kcc_kernels.hip `fit_kernel`).

The kernel computes floor(fc / c) and floor(fm / m) (CC:123, CC:129) without any
integer division or correction step:

    qc = trunc(RN64(fc * rc)),  rc = smallest f64 >= 1/c     (fc < 2^50, 1 <= c < 2^51)
    qm = trunc(RN64(fm * rm)),  rm = smallest f64 >= 1/m     (fm < 2^50, 1 <= m < 2^51)

numpy's float64 products are IEEE round-to-nearest-even, exactly what v_mul_f64
does, so these tests replay the kernel's arithmetic on the
CPU and compare it with exact integer floor division — on the quotients where the
argument is tightest: exact multiples, +-1 around them, the largest operands allowed
on the fast path, powers of two and their neighbours.
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


def fast_qc(fc, c):
    return np.trunc(np.asarray(fc).astype(np.float64) * recip_up_f64(c)).astype(np.int64)


def fast_qm(fm, m):
    return np.trunc(np.asarray(fm).astype(np.float64) * recip_up_f64(m)).astype(np.int64)


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
    qc = fast_qc(fc[:, None], sc[None, :])
    qm = np.minimum(fast_qm(fm[:, None], sm[None, :]), 2**31 - 1)
    x = np.minimum(qc, qm)
    contrib = np.where(x >= P[:, None], (P - pc)[:, None], x)
    tot = contrib.sum(axis=0)
    zero = np.zeros(n, np.int64)
    ot, oe = coracle.fit(fc.astype(np.uint64), fm, P, pc, zero.astype(np.uint64), zero,
                         sc.astype(np.uint64), sm.astype(np.int64))
    assert not oe.any()
    np.testing.assert_array_equal(tot, ot)
