"""CPU model of the fit's clamp correction (kcc_internal.h `ClampWork`).

The fast loops sum min(findMin(qc, qm), P) per (node, spec); the reference's
contribution (CC:133-136) is `x >= P ? P - podCount : x`, i.e. that minus
w = P - cl (= podCount) wherever x >= P.  The correction subtracts, per spec,

    D_s = Σ_i w_i [x_is >= P_i]

computed as a 2-D dominance count: x >= P <=> c_s <= U_i = fc_i // P_i and
m_s <= V_i = fm_i // P_i (P_i >= 1; P_i <= 0 rows are clamped for every spec).  This
module restates the kernels' algorithm in numpy — c-ranks in groups of 64, the
(T+1) x (nN+1) table H of fully covered groups read through its row suffix sums R
(clamp_rows_kernel), and per group the 64 x 65 table H2 of partially covered groups
indexed by (r, k), k = #{group specs with m_less < b}, read through its 2-D suffix sums
(clamp_groups_kernel) — and checks it against the direct definition, then the whole
per-spec total against the C oracle.
"""
import numpy as np
import pytest

# uint64 sums wrap on purpose (Go's int64 arithmetic)
pytestmark = pytest.mark.filterwarnings("ignore:overflow encountered:RuntimeWarning")

INF32 = 0xFFFFFFFF


def group_orders(mlq, nN):
    """spec_prep_kernel / clamp_group_kernel: per group of 64 c-ranks, each spec's
    position in the group's m_less order (ties by lane) and the ascending m_less list."""
    T = (nN + 63) // 64
    kpos = np.zeros(nN, np.int64)
    gml = np.full(64 * T, INF32, np.int64)
    for g in range(T):
        v = np.full(64, INF32, np.int64)
        n = min(64, nN - 64 * g)
        v[:n] = mlq[64 * g: 64 * g + n]
        pos = np.empty(64, np.int64)
        pos[np.lexsort((np.arange(64), v))] = np.arange(64)
        kpos[64 * g: 64 * g + n] = pos[:n]
        gml[64 * g + pos] = v
    return kpos, gml


def suffix2(a):
    """2-D suffix sums over the last two axes (wrapping uint64)."""
    a = a[..., ::-1, :].cumsum(axis=-2, dtype=np.uint64)[..., ::-1, :]
    return a[..., ::-1].cumsum(axis=-1, dtype=np.uint64)[..., ::-1]


def clamp_correction(U, V, w, always, c, m):
    """D_s for every spec by the kernels' algorithm (numpy, exact int64 wrap)."""
    nN = c.size
    T = (nN + 63) // 64
    order_c = np.lexsort((np.arange(nN), c))          # c-rank -> spec (ties by position)
    cs = c[order_c]
    ms = np.sort(m, kind="stable")
    mlq = np.searchsorted(ms, m, side="left")[order_c]  # by c-rank: #specs with a smaller m
    kpos, gml = group_orders(mlq, nN)
    H = np.zeros((T + 1, nN + 1), np.uint64)
    H2 = np.zeros((T, 65, 65), np.uint64)             # [G][r][k], rows r = 0 and 64 empty
    for Ui, Vi, wi, al in zip(U, V, w, always):
        wi = np.uint64(np.int64(wi).view(np.uint64))
        if al:
            H[T, nN] += wi
            continue
        L = int(np.searchsorted(cs, Ui, side="right"))
        b = int(np.searchsorted(ms, Vi, side="right"))
        if L == 0 or b == 0:
            continue
        G, r = L >> 6, L & 63
        if G:
            H[G, b] += wi
        if r:
            k = int((gml[64 * G: 64 * G + 64] < b).sum())
            if k:
                H2[G, r, k] += wi
    R = H[:, ::-1].cumsum(axis=1, dtype=np.uint64)[:, ::-1]   # clamp_rows_kernel
    S2 = suffix2(H2)                                          # clamp_groups_kernel
    D = np.zeros(nN, np.uint64)
    for q in range(nN):
        s = order_c[q]
        g, lane = q >> 6, q & 63
        b1 = mlq[q] + 1
        d = np.uint64(0)
        if b1 <= nN:
            d += R[g + 1:, b1].sum(dtype=np.uint64)
        d += S2[g, lane + 1, kpos[q] + 1]
        D[s] = d
    return D.view(np.int64)


def direct(U, V, w, always, c, m):
    hit = always[:, None] | ((U[:, None] >= c[None, :]) & (V[:, None] >= m[None, :]))
    return (hit * w[:, None]).sum(axis=0)


@pytest.mark.parametrize("seed,n,s", [(0, 3000, 1), (1, 2000, 63), (2, 2000, 64), (3, 2500, 130),
                                      (4, 1500, 257)])
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
