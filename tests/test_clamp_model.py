"""CPU model of the fit's clamp correction (kcc_internal.h `ClampWork`).

The fast loops sum min(findMin(qc, qm), P) per (node, spec); the reference's
contribution (CC:133-136) is `x >= P ? P - podCount : x`, i.e. that minus
w = P - cl (= podCount) wherever x >= P.  The correction subtracts, per spec,

    D_s = Σ_i w_i [x_is >= P_i]

computed as a 2-D dominance count: x >= P <=> c_s <= U_i = fc_i // P_i and
m_s <= V_i = fm_i // P_i (P_i >= 1; P_i <= 0 rows are clamped for every spec).  This
module restates the kernels' algorithm in numpy — c-ranks in groups of 64, the
(T+1) x (nN+1) table H of fully covered groups with its 2-D suffix sums, and the plist
of partially covered groups — and checks it against the direct definition, then the
whole per-spec total against the C oracle.
"""
import numpy as np
import pytest

# uint64 sums wrap on purpose (Go's int64 arithmetic)
pytestmark = pytest.mark.filterwarnings("ignore:overflow encountered:RuntimeWarning")


def clamp_correction(U, V, w, always, c, m):
    """D_s for every spec by the kernels' algorithm (numpy, exact int64 wrap)."""
    nN = c.size
    T = (nN + 63) // 64
    order_c = np.lexsort((np.arange(nN), c))          # c-rank -> spec (ties by position)
    cs = c[order_c]
    ms = np.sort(m, kind="stable")
    m_less = np.searchsorted(ms, m, side="left")      # #specs with a smaller m
    H = np.zeros((T + 1, nN + 1), np.uint64)
    plist = []
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
            plist.append((G, r, b, wi))
    HS = H[::-1].cumsum(axis=0, dtype=np.uint64)[::-1]            # suffix over G
    HS = HS[:, ::-1].cumsum(axis=1, dtype=np.uint64)[:, ::-1]     # suffix over b
    D = np.zeros(nN, np.uint64)
    for q in range(nN):                                            # full groups
        s = order_c[q]
        g1, b1 = (q >> 6) + 1, m_less[s] + 1
        if g1 <= T and b1 <= nN:
            D[s] += HS[g1, b1]
    for G, r, b, wi in plist:                                      # partial groups
        for lane in range(r):
            s = order_c[64 * G + lane]
            if m_less[s] < b:
                D[s] += wi
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
