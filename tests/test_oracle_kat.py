"""Known-answer tests pinning the CPU oracles to the reference.

The reference ships no tests or golden vectors, so these values are
derived by hand from the cited lines of ClusterCapacity.go (CC) and bytes.go (BF).
Both restatements — the C oracle and the independent Python big-int one — must
reproduce every value.
"""
import pytest

from oracle import coracle, pyoracle

U64 = 1 << 64
BOTH = [coracle, pyoracle]


def fit_one(mod, *args):
    if mod is coracle:
        q, z = coracle.fit_one(*args)
        if z:
            raise ZeroDivisionError
        return q
    return pyoracle.fit_one(*args)


# ---- K1: flag parsing (CC:57-67, CC:301-319, BF:96-97) -------------------------
@pytest.mark.parametrize("mod", BOTH)
@pytest.mark.parametrize("s,want,ok", [
    ("200m", 200, True), ("400m", 400, True), ("100m", 100, True), ("200m", 200, True),
    ("2", 2000, True), ("250m", 250, True), ("0", 0, True), ("+3", 3000, True),
    ("0.5", 0, False), ("2k", 0, False), ("500u", 0, False), ("", 0, False), ("m", 0, False),
    ("-100m", U64 - 100, True),                      # K8: negative wraps (CC:318)
    ("9223372036854775807m", (1 << 63) - 1, True),
    ("9223372036854775808m", 0, False),              # Atoi range error
    ("9223372036854775807", ((1 << 63) - 1) * 1000 % U64, True),  # int multiply wraps
    ("1mm", 0, False), ("1 m", 0, False),
])
def test_convert_cpu_to_milis(mod, s, want, ok):
    v, good = mod.convert_cpu_to_milis(s)
    assert (v, good) == (want, ok)


@pytest.mark.parametrize("mod", BOTH)
@pytest.mark.parametrize("s,want,ok", [
    ("250mb", 262_144_000, True), ("500mb", 524_288_000, True),
    ("100mb", 104_857_600, True), ("200mb", 209_715_200, True),
    ("16331524Ki", 16_723_480_576, True),            # node allocatable memory
    ("16Gi", 0, False),                              # GI not accepted (BF:94)
    ("1Ti", 0, False), ("1", 0, False),              # no letter -> error (BF:81-83)
    ("1.5G", 1_610_612_736, True), ("1GIB", 1 << 30, True), ("  2 KB ", 0, False),
    ("  2KB ", 2048, True), ("0.5B", 0, True),       # int64(0.5) == 0, nil error
    ("0mb", 0, False), ("-1mb", 0, False),           # bytes <= 0 rejected
    ("1e3MB", 0, False), ("100M", 104_857_600, True), ("7b", 7, True),
    ("1.0000000001K", 1024, True), (".5K", 512, True), ("5.K", 5120, True),
    ("99999999999T", -(1 << 63), True),              # amd64 float->int64 overflow value
])
def test_to_bytes(mod, s, want, ok):
    v, good = mod.to_bytes(s)
    assert (v, good) == (want, ok)


# ---- K2-K6: fit arithmetic (CC:119-136) ------------------------------------------
@pytest.mark.parametrize("mod", BOTH)
def test_k2_ordinary_fit(mod):
    assert fit_one(mod, 4000, 16_723_480_576, 110, 12, 1850, 3_221_225_472,
                   200, 262_144_000) == 10


@pytest.mark.parametrize("mod", BOTH)
def test_k3_clamp(mod):
    assert fit_one(mod, 64000, 274_877_906_944, 110, 30, 0, 0, 100, 104_857_600) == 80


@pytest.mark.parametrize("mod", BOTH)
def test_k4_negative_clamp(mod):
    assert fit_one(mod, 64000, 274_877_906_944, 110, 130, 0, 0, 100, 104_857_600) == -20


@pytest.mark.parametrize("mod", BOTH)
def test_k5_equality_is_full(mod):
    # `<=` at CC:119/125: alloc == used leaves no room
    assert fit_one(mod, 4000, 1 << 30, 110, 5, 4000, 1 << 30, 100, 1 << 20) == 0
    assert fit_one(mod, 4000, 1 << 30, 110, 5, 4000, 0, 100, 1 << 20) == 0
    assert fit_one(mod, 4000, 1 << 30, 110, 5, 0, 1 << 30, 100, 1 << 20) == 0


@pytest.mark.parametrize("mod", BOTH)
def test_k6_zero_row(mod):
    # unhealthy node keeps its zero value (CC:221-226); podCount("") = 3
    assert fit_one(mod, 0, 0, 0, 3, 0, 0, 200, 262_144_000) == -3


# ---- K7: divide by zero (Go panics) -------------------------------------------------
@pytest.mark.parametrize("mod", BOTH)
def test_k7_div0(mod):
    with pytest.raises(ZeroDivisionError):
        fit_one(mod, 4000, 1 << 30, 110, 0, 0, 0, 0, 1 << 20)
    with pytest.raises(ZeroDivisionError):
        fit_one(mod, 4000, 1 << 30, 110, 0, 0, 0, 100, 0)
    # no free row: no division happens, the clamp still applies
    assert fit_one(mod, 4000, 1 << 30, 110, 7, 4000, 1 << 30, 0, 0) == 0
    assert fit_one(mod, 0, 0, 0, 7, 0, 0, 0, 0) == -7


def test_k7_totals_and_flags():
    nodes = dict(alloc_cpu=[4000, 0], alloc_mem=[1 << 30, 0], alloc_pods=[110, 0],
                 pod_count=[0, 2], used_cpu=[4000, 0], used_mem=[1 << 30, 0])
    args = [nodes[k] for k in ("alloc_cpu", "alloc_mem", "alloc_pods", "pod_count",
                               "used_cpu", "used_mem")]
    t, e = coracle.fit(*args, [0, 100], [0, 1 << 20])
    assert list(t) == [-2, -2] and list(e) == [0, 0]   # no free row: sum of clamps
    t2, e2 = pyoracle.fit(*args, [0, 100], [0, 1 << 20])
    assert t2 == [-2, -2] and e2 == [0, 0]
    args[4] = [0, 0]                                    # now node 0 has free CPU
    t, e = coracle.fit(*args, [0, 100], [0, 1 << 20])
    assert list(e) == [1, 0] and t[0] == 0


# ---- K8: negative CPU request wraps and makes the node "full" -----------------------
@pytest.mark.parametrize("mod", BOTH)
def test_k8_negative_request(mod):
    used = (U64 - 100) % U64                            # one container with "-100m"
    assert fit_one(mod, 4000, 1 << 34, 110, 1, used, 0, 100, 1 << 20) == 0
    uc, um, _, _ = coracle.reduce_requests([0, 2], [U64 - 100, 300], [5, -7])
    assert int(uc[0]) == 200 and int(um[0]) == -2      # wrapping sums (CC:290-292)


# ---- findMin, Go division corner cases -------------------------------------------------
def test_find_min():
    assert pyoracle.find_min(3, 3) == 3
    assert coracle.lib().kcco_find_min(-5, 2) == -5


@pytest.mark.parametrize("mod", BOTH)
def test_go_int64_division_corners(mod):
    big = (1 << 63) - 1
    # memory: alloc - used overflows to MinInt64, divided by -1 stays MinInt64
    assert fit_one(mod, 0, big, 1 << 62, 0, 0, -1, 1, -1) == -(1 << 63)
    # negative quotient (spec mem < 0) truncates toward zero
    assert fit_one(mod, 0, 10, 1 << 40, 0, 0, 0, 1, -3) == -3
    assert fit_one(mod, 1 << 20, 10, 1 << 40, 0, 0, 0, 1, -3) == -3
    # int(uint64) reinterprets: quotient >= 2^63 is negative
    assert fit_one(mod, U64 - 1, 1 << 40, 1 << 40, 0, 0, 0, 1, 1) == -1
