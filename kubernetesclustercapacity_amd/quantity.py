"""Resource-quantity strings in the packed layout of the kcc_parse_* entry points.

The reference converts every container's cpu request/limit with
`convertCPUToMilis(q.String())` (CC:280, CC:283) and every node's allocatable memory
with `bytefmt.ToBytes(q.String())` (CC:202-203).  `resource.Quantity.String()` prints
the canonical form (apimachinery, unpinned — SURVEY §8c): the integer value with the
largest suffix that divides it exactly.  This module builds those strings, vectorised,
as Arrow-style packed arrays (bytes + int64 offsets) for the device parser, and packs
arbitrary Python strings for tests.  Host-side formatting only: the conversion itself
is `CapacityEngine.convert_cpu_to_milis` / `.to_bytes` (gfx950 kernels).
"""
from __future__ import annotations

import numpy as np

_POW10 = np.array([10 ** k for k in range(20)], dtype=np.uint64)


def _align4(n: int) -> int:
    return (n + 3) & ~3


def pack_strings(strs) -> tuple[np.ndarray, np.ndarray]:
    """Pack a sequence of str/bytes into (uint8 bytes, int64 offsets[n+1])."""
    enc = [s.encode("latin-1") if isinstance(s, str) else bytes(s) for s in strs]
    lens = np.fromiter((len(b) for b in enc), dtype=np.int64, count=len(enc))
    off = np.zeros(len(enc) + 1, np.int64)
    np.cumsum(lens, out=off[1:])
    buf = np.zeros(_align4(int(off[-1])) or 4, np.uint8)
    joined = b"".join(enc)
    buf[:len(joined)] = np.frombuffer(joined, np.uint8)
    return buf, off


def unpack_strings(buf: np.ndarray, off: np.ndarray) -> list[bytes]:
    raw = buf.tobytes()
    return [raw[off[i]:off[i + 1]] for i in range(off.size - 1)]


def _format(values: np.ndarray, suffix_codes: np.ndarray, suffixes: list[bytes],
            chunk: int = 1 << 22) -> tuple[np.ndarray, np.ndarray]:
    """Decimal digits of non-negative `values` (< 10^19) followed by suffixes[code]."""
    values = np.ascontiguousarray(values, np.uint64)
    n = values.size
    ndig = np.maximum(np.searchsorted(_POW10, values, side="right"), 1).astype(np.int64)
    slen = np.array([len(s) for s in suffixes], np.int64)
    lens = ndig + slen[suffix_codes]
    off = np.zeros(n + 1, np.int64)
    np.cumsum(lens, out=off[1:])
    buf = np.zeros(_align4(int(off[-1])) or 4, np.uint8)
    smax = int(slen.max()) if slen.size else 0
    stab = np.zeros((len(suffixes), max(smax, 1)), np.uint8)
    for i, s in enumerate(suffixes):
        stab[i, :len(s)] = np.frombuffer(s, np.uint8) if s else []
    for c0 in range(0, n, chunk):
        v = values[c0:c0 + chunk]
        nd = ndig[c0:c0 + chunk]
        sc = suffix_codes[c0:c0 + chunk]
        start = off[c0:c0 + v.size]
        last = start + nd - 1  # position of the least significant digit
        rem = v.copy()
        for j in range(int(nd.max()) if v.size else 0):  # digits from the least significant
            live = nd > j
            buf[(last - j)[live]] = (rem[live] % np.uint64(10)).astype(np.uint8) + ord("0")
            rem //= np.uint64(10)
        for j in range(smax):
            has = slen[sc] > j
            buf[start[has] + nd[has] + j] = stab[sc[has], j]
    return buf, off


def cpu_quantity_strings(millis) -> tuple[np.ndarray, np.ndarray]:
    """Canonical Quantity.String() of DecimalSI cpu values given in millicores
    (< 10^19): whole cores print bare ("2"), the rest with "m" ("250m", "1500m")."""
    m = np.ascontiguousarray(millis, np.uint64)
    whole = (m % np.uint64(1000)) == 0
    vals = np.where(whole, m // np.uint64(1000), m)
    return _format(vals, (~whole).astype(np.int64), [b"", b"m"])


_BIN = [b"", b"Ki", b"Mi", b"Gi", b"Ti", b"Pi", b"Ei"]


def memory_quantity_strings(nbytes) -> tuple[np.ndarray, np.ndarray]:
    """Canonical Quantity.String() of BinarySI memory values in bytes (>= 0): the value
    with the largest binary suffix dividing it ("16331524Ki", "64Gi", "1000")."""
    b = np.ascontiguousarray(nbytes, np.uint64)
    code = np.zeros(b.size, np.int64)
    for k in range(1, 7):
        div = ((b % (np.uint64(1) << np.uint64(10 * k))) == 0) & (b > 0)
        code = np.where(div, k, code)
    vals = b >> (np.uint64(10) * code.astype(np.uint64))
    return _format(vals, code, _BIN)
