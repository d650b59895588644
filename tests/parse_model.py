"""Python restatement of the device parser (kubernetesclustercapacity_amd/csrc/kcc_parse.hip)
— test infrastructure.

It mirrors the kernel step by step (Atoi with the lim/10 overflow test; ToBytes with the
significant-digit scan, the domain classification and the restoring division that
rounds D / 10^k), so the CPU suite can check the kernel's algorithm against the oracle
(oracle/kcc_oracle.c, glibc strtod) before any GPU run, and the GPU tests can check that
PARSE_UNSUPPORTED appears exactly where the algorithm says.
"""
from __future__ import annotations

import math
import struct

OK, ERR, UNSUPPORTED = 1, 0, -1
I64_MIN = -(1 << 63)
U64 = 1 << 64


def _space(c):
    return c == 32 or 9 <= c <= 13


def _letter(c):
    return (ord("a") <= (c | 0x20) <= ord("z")) or c >= 0x80


def _up(c):
    return c - 32 if ord("a") <= c <= ord("z") else c


def atoi(s: bytes):
    n = len(s)
    if n == 0:
        return None
    i, neg = 0, False
    if s[0] in b"+-":
        neg, i = s[0] == ord("-"), 1
    if i == n:
        return None
    q, r = 922337203685477580, (8 if neg else 7)
    v = 0
    for c in s[i:]:
        d = c - 48
        if not 0 <= d <= 9:
            return None
        if v > q or (v == q and d > r):
            return None
        v = v * 10 + d
    return -v if neg else v


def cpu_millis(s: bytes):
    cores = True
    if s[-1:] == b"m":
        s, cores = s[:-1], False
    v = atoi(s)
    if v is None:
        return 0, ERR
    return ((v * 1000) if cores else v) % U64, OK


def div_pow10_rn(D: int, k: int) -> float:
    """Restoring division of the kernel: 57 quotient bits, round-half-even to 53."""
    V = 10 ** k
    R, q, bit, extra = 0, 0, 63, 0
    while q < (1 << 56):
        if bit >= 0:
            b = (D >> bit) & 1
            bit -= 1
        else:
            b = 0
            extra += 1
        R = (R << 1) | b
        q <<= 1
        if R >= V:
            R -= V
            q |= 1
    sticky = R != 0
    if bit >= 0:
        sticky |= (D & ((2 << bit) - 1)) != 0
        e2 = bit + 1
    else:
        e2 = -extra
    low = q & 15
    q >>= 4
    e2 += 4
    if (low & 8) and ((low & 7) or sticky or (q & 1)):
        q += 1
        if q == 1 << 53:
            q >>= 1
            e2 += 1
    return math.ldexp(float(q), e2)


def frac_rn(D: int, k: int) -> float:
    if D < (1 << 53) and k <= 22:
        return float(D) / float(10 ** k)
    return div_pow10_rn(D, k)


def _f2i_amd64(v: float) -> int:
    return I64_MIN if v >= 2.0 ** 63 else int(v)


def to_bytes(s: bytes):
    b, e = 0, len(s)
    while b < e and _space(s[b]):
        b += 1
    while e > b and _space(s[e - 1]):
        e -= 1
    i = b
    while i < e and not _letter(s[i]):
        i += 1
    if i == e:
        return 0, ERR
    mult = bytes(_up(c) for c in s[i:e])
    shifts = {b"T": 40, b"TB": 40, b"TIB": 40, b"G": 30, b"GB": 30, b"GIB": 30,
              b"M": 20, b"MB": 20, b"MIB": 20, b"MI": 20,
              b"K": 10, b"KB": 10, b"KIB": 10, b"KI": 10, b"B": 0}
    shift = shifts.get(mult, -1)
    j, neg = b, False
    if j < i and s[j] in b"+-":
        neg, j = s[j] == ord("-"), j + 1
    dot = trunc_nz = False
    digits = sig = e10 = D = 0
    for c in s[j:i]:
        d = c - 48
        if 0 <= d <= 9:
            digits += 1
            if sig == 0 and d == 0:
                if dot:
                    e10 -= 1
                continue
            if sig < 19:
                D = D * 10 + d
                sig += 1
                if dot:
                    e10 -= 1
            else:
                trunc_nz |= d != 0
                if not dot:
                    e10 += 1
        elif c == ord(".") and not dot:
            dot = True
        else:
            return 0, ERR
    if digits == 0 or D == 0 or neg or shift < 0:
        return 0, ERR
    mag = sig + e10
    if mag >= 310:
        return 0, ERR
    if mag == 309:
        return 0, UNSUPPORTED
    if mag >= 20:
        return I64_MIN, OK
    if e10 >= 0:
        x = float(D * 10 ** e10)  # correctly rounded int -> float
    else:
        k = -e10
        if k > 38:
            if mag >= -322:
                return 0, OK
            return 0, (UNSUPPORTED if mag == -323 else ERR)
        x = frac_rn(D, k)
        if trunc_nz and frac_rn(D + 1, k) != x:
            return 0, UNSUPPORTED
    return _f2i_amd64(math.ldexp(x, shift)), OK


def f64_bits(x: float) -> int:
    return struct.unpack("<Q", struct.pack("<d", x))[0]
