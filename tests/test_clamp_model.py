"""CPU model of the fit's clamp correction (kcc_internal.h `ClampWork`).

The fast loops sum min(findMin(qc, qm), P) per (node, spec); the reference's
contribution (CC:133-136) is `x >= P ? P - podCount : x`, i.e. that minus
w = P - cl (= podCount) wherever x >= P.  The correction subtracts, per spec,

    D_s = Σ_i w_i [x_is >= P_i]

computed as a 2-D dominance sum: x >= P <=> c_s <= U_i = fc_i // P_i and
m_s <= V_i = fm_i // P_i (P_i >= 1; P_i <= 0 rows are clamped for every spec).  With
the normal specs ranked by (c, index) -> x_s and by (m, index) -> y_s (permutations of
0..nN-1), node i dominates exactly the specs with x_s < L_i and y_s < b_i (L_i = #{c <=
U_i}, b_i = #{m <= V_i}).  Both axes are cut into blocks of 64 ranks (T blocks):
  - coarse table C[L_i >> 6][b_i >> 6] ((T+2)^2; P <= 0 rows in the extra last cell),
    read through its 2-D suffix sums at (x_s >> 6) + 1, (y_s >> 6) + 1;
  - x-group table H2[g][r][k] (T x 65 x 65) for the rows with L_i >> 6 == g (r = L_i & 63,
    k = #{specs of x-group g with y < b_i}), read at (x_s & 63) + 1, kpos_s + 1 (kpos_s =
    #{specs of s's x-group with y < y_s});
  - y-block table H3[Y][r][j] for the rows with b_i >> 6 == Y (r = b_i & 63, j = #{specs of
    y-block Y whose x-group < L_i >> 6}), read at (y_s & 63) + 1, jpos_s + 1 (jpos_s =
    #{specs of s's y-block with x < x_s}).
All three are linear in S (the earlier (T+1) x (nN+1) table grew as S^2/64).  This module
restates that algorithm in numpy and checks it against the direct definition, then the
whole per-spec total against the C oracle.
"""
import numpy as np
import pytest

# uint64 sums wrap on purpose (Go's int64 arithmetic)
pytestmark = pytest.mark.filterwarnings("ignore:overflow encountered:RuntimeWarning")


def suffix2(a):
    """2-D suffix sums over the last two axes (wrapping uint64)."""
    a = a[..., ::-1, :].cumsum(axis=-2, dtype=np.uint64)[..., ::-1, :]
    return a[..., ::-1].cumsum(axis=-1, dtype=np.uint64)[..., ::-1]


def clamp_correction(U, V, w, always, c, m):
    """D_s for every spec by the kernels' algorithm (numpy, exact int64 wrap)."""
    nN = c.size
    T = (nN + 63) // 64
    idx = np.arange(nN)
    order_c = np.lexsort((idx, c))                    # x-rank -> spec
    order_m = np.lexsort((idx, m))                    # y-rank -> spec
    x = np.empty(nN, np.int64)
    x[order_c] = idx
    y = np.empty(nN, np.int64)
    y[order_m] = idx
    cs, ms = c[order_c], m[order_m]
    y_by_x = y[order_c]                               # spec_place: mr_c
    x_by_y = x[order_m]                               # spec_place: cr_m
    C = np.zeros((T + 2, T + 2), np.uint64)
    H2 = np.zeros((T, 65, 65), np.uint64)             # [g][r][k]
    H3 = np.zeros((T, 65, 65), np.uint64)             # [Y][r][j]
    for Ui, Vi, wi, al in zip(U, V, w, always):
        wi = np.uint64(np.int64(wi).view(np.uint64))
        if al:
            C[T + 1, T + 1] += wi
            continue
        L = int(np.searchsorted(cs, Ui, side="right"))
        b = int(np.searchsorted(ms, Vi, side="right"))
        if L == 0 or b == 0:
            continue
        GX, rx, GY, ry = L >> 6, L & 63, b >> 6, b & 63
        C[GX, GY] += wi
        if rx:                                        # node_prep: count over the x-group
            k = int((y_by_x[64 * GX: 64 * GX + 64] < b).sum())
            if k:
                H2[GX, rx, k] += wi
        if ry and GX:                                 # count over the y-block
            j = int(((x_by_y[64 * GY: 64 * GY + 64] >> 6) < GX).sum())
            if j:
                H3[GY, ry, j] += wi
    Cs = suffix2(C)
    S2, S3 = suffix2(H2), suffix2(H3)
    D = np.zeros(nN, np.uint64)
    for s in range(nN):
        xs, ys = int(x[s]), int(y[s])
        gx, gy = xs >> 6, ys >> 6
        kpos = int((y_by_x[64 * gx: 64 * gx + 64] < ys).sum())
        jpos = int((x_by_y[64 * gy: 64 * gy + 64] < xs).sum())
        D[s] = Cs[gx + 1, gy + 1] + S2[gx, (xs & 63) + 1, kpos + 1] + S3[gy, (ys & 63) + 1, jpos + 1]
    return D.view(np.int64)


def direct(U, V, w, always, c, m):
    hit = always[:, None] | ((U[:, None] >= c[None, :]) & (V[:, None] >= m[None, :]))
    return (hit * w[:, None]).sum(axis=0)


@pytest.mark.parametrize("seed,n,s", [(0, 3000, 1), (1, 2000, 63), (2, 2000, 64), (3, 2500, 130),
                                      (4, 1500, 257), (5, 1200, 640), (6, 800, 1031)])
def test_dominance_matches_definition(seed, n, s):
    rng = np.random.default_rng(seed)
    c = rng.integers(1, 300, s)
    m = rng.integers(1, 300, s)
    c[: s // 3] = c[0]                       # ties
    m[s // 4: s // 2] = m[-1]
    U = rng.integers(0, 320, n)
    V = rng.integers(0, 320, n)
    U[: n // 5] = rng.choice(c, n // 5)      # exactly on spec values
    V[n // 5: 2 * n // 5] = rng.choice(m, n // 5)
    w = rng.integers(-(1 << 21), 1 << 21, n)
    always = rng.random(n) < 0.05
    np.testing.assert_array_equal(clamp_correction(U, V, w, always, c, m),
                                  direct(U, V, w, always, c, m))


def test_total_equals_oracle():
    """Σ min(x, P) - D over fast rows == the reference fit (C oracle), rows incl. P <= 0."""
    from oracle import coracle
    rng = np.random.default_rng(9)
    n, s = 3000, 150
    sc = rng.integers(1, 400, s)
    sm = rng.integers(1 << 18, 1 << 30, s)
    fc = rng.integers(0, 90_000, n)
    fm = rng.integers(0, 1 << 38, n)
    P = rng.integers(-3, 250, n)
    pc = rng.integers(0, 300, n)
    cl = P - pc
    x = np.minimum(fc[:, None] // sc[None, :], fm[:, None] // sm[None, :])
    Penc = np.maximum(P, 0)
    base = np.minimum(x, Penc[:, None]).sum(axis=0)
    pos = P > 0
    U = np.where(pos, fc // np.where(pos, P, 1), 0)
    V = np.where(pos, fm // np.where(pos, P, 1), 0)
    D = clamp_correction(U, V, Penc - cl, P <= 0, sc, sm)
    zero = np.zeros(n, np.int64)
    ot, oe = coracle.fit(fc.astype(np.uint64), fm, P, pc, zero.astype(np.uint64), zero,
                         sc.astype(np.uint64), sm.astype(np.int64))
    assert not oe.any()
    np.testing.assert_array_equal(base - D, ot)
