"""Host-side check of the node-prep wait window (kcc_kernels.hip np_wait_rows): node prep
inside the reduce launch (kcc::NpArgs) waits, for rows [i0, i1), on the flags of reduce
waves [(ptr[i0] - c0) / range - 1, (ptr[i1] - c0) / range] (clamped to the launch's
waves).  The reduce's store rule, restated from reduce_kernel: wave w covers containers
[wb, wb + len); node0 is 0 for wave 0, else the last node with ptr[j] <= wb; the wave
stores every node j >= node0 whose end ptr[j + 1] <= wb + len (node0 by its look-back when
it began in an earlier range).  Every node must have exactly one storing wave, inside
its row workgroup's window."""
import numpy as np
import pytest

NP_ROWS_PER_WG = 1024


def storing_waves(ptr, c0, c_end, rng_len):
    n = ptr.size - 1
    waves = (c_end - c0 + rng_len - 1) // rng_len
    owner = np.full(n, -1, np.int64)
    for w in range(waves):
        wb = c0 + w * rng_len
        end = min(wb + rng_len, c_end)
        node0 = 0 if w == 0 else int(np.searchsorted(ptr[:n], wb, "right")) - 1
        last = int(np.searchsorted(ptr[1:], end, "right"))  # nodes j < last end by `end`
        js = np.arange(node0, last)
        assert np.all(owner[js] == -1), "a node stored by two waves"
        owner[js] = w
    return owner, waves


def window(ptr, c0, rng_len, waves, i0, i1):
    wlo = max((int(ptr[i0]) - c0) // rng_len - 1, 0)
    whi = min((int(ptr[i1]) - c0) // rng_len, waves - 1)
    return wlo, whi


def make_ptr(rng, n, total, rng_len, empties_at_bounds, giant):
    cuts = list(rng.integers(0, total + 1, n - 1))
    if empties_at_bounds:
        b = list(range(rng_len, total, rng_len)) * 2
        cuts = b + cuts[: max(0, n - 1 - len(b))]
    if giant:
        g0 = total // 3
        cuts = [x if not (g0 < x < g0 + 5 * rng_len) else g0 for x in cuts]
    cuts = sorted(cuts)[: n - 1]
    cuts[:3] = [0, 0, 0]
    cuts[-3:] = [total] * 3
    return np.array([0] + cuts + [total], np.int64)


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("rng_len", [512, 1024, 3072])
def test_np_window_covers_storing_wave(seed, rng_len):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(3000, 9000))
    total = int(rng.integers(50_000, 400_000))
    ptr = make_ptr(rng, n, total, rng_len, seed % 2 == 0, seed % 3 == 0)
    c0 = 0
    owner, waves = storing_waves(ptr, c0, total, rng_len)
    assert np.all(owner >= 0), "a node no wave stores"
    for i0 in range(0, n, NP_ROWS_PER_WG):
        i1 = min(i0 + NP_ROWS_PER_WG, n)
        wlo, whi = window(ptr, c0, rng_len, waves, i0, i1)
        o = owner[i0:i1]
        assert o.min() >= wlo and o.max() <= whi, (i0, wlo, whi, o.min(), o.max())
