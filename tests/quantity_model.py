"""Independent restatement of k8s.io/apimachinery resource.ParseQuantity + Quantity.Value()
(resource/quantity.go, published algorithm; not vendored in the reference, version
unpinned -> parity unpinned) — test infrastructure for kcc_parse_quantity.

parseQuantityString: [+-], leading zeros, numerator digits, optional '.' + denominator
digits, then a suffix of "eEinumkKMGTP" letters, an optional sign and digits, to the end
(else ErrFormatWrong).  interpret: "" | Ki..Ei (2^10k) | n u m k M G T P E (10^3k) |
e/E<ParseInt64> (10^int32(exp)) (else ErrSuffix).  Value() rounds up away from zero;
binary (Ki..Ei) amounts are capped at 2^63 - 1 in magnitude (ParseQuantity caps only
BinarySI at maxAllowed).  Two cases the engine reports as UNSUP (its "outside the exact
domain" status) instead of guessing: a decimal amount beyond 2^63 - 1 (k8s wraps it, in a
way that depends on which of ParseQuantity's two representations it takes), and a
negative nonzero amount that leaves ParseQuantity's int64 fast path (<= 18 digits and a
scale >= -9 for decimal suffixes; no fraction and few enough digits for binary ones),
whose Value() rounding is not pinned.  Exact rationals throughout.
"""
from fractions import Fraction

OK, ERR, UNSUP = 1, 0, -1
MAXV = (1 << 63) - 1
_BIN = {"Ki": 10, "Mi": 20, "Gi": 30, "Ti": 40, "Pi": 50, "Ei": 60}
_DEC = {"n": -9, "u": -6, "m": -3, "": 0, "k": 3, "M": 6, "G": 9, "T": 12, "P": 15, "E": 18}


def _go_parse_int64(t: str):
    if not t or (t[0] in "+-" and len(t) == 1):
        return None
    body = t[1:] if t[0] in "+-" else t
    if not body.isdigit() or not body.isascii():
        return None
    v = int(t)
    return v if -(1 << 63) <= v <= MAXV else None


def value(s: str):
    """-> (Value() as int, status)"""
    if s == "":
        return 0, ERR
    pos, end = 0, len(s)
    neg = False
    if s[0] in "+-":
        neg, pos = s[0] == "-", 1
    while pos < end and s[pos] == "0":
        pos += 1
    if pos >= end:
        return 0, OK
    n0 = pos
    while pos < end and s[pos] in "0123456789":
        pos += 1
    num = s[n0:pos]
    den = ""
    if pos < end and s[pos] == ".":
        pos += 1
        d0 = pos
        while pos < end and s[pos] in "0123456789":
            pos += 1
        den = s[d0:pos]
    suf0 = pos
    while pos < end and s[pos] in "eEinumkKMGTP":
        pos += 1
    if pos < end and s[pos] in "+-":
        pos += 1
    while pos < end and s[pos] in "0123456789":
        pos += 1
    if pos < end:
        return 0, ERR
    suf = s[suf0:]
    x = Fraction(int(num or "0") * 10 ** len(den) + int(den or "0"), 10 ** len(den))
    binary = suf in _BIN
    if binary:
        x *= 2 ** _BIN[suf]
        fast = len(den) == 0 and len(num) <= 14 - 3 * (_BIN[suf] // 10)
    elif suf in _DEC:
        x *= Fraction(10) ** _DEC[suf]
        fast = len(num) + len(den) <= 18 and _DEC[suf] - len(den) >= -9
    elif len(suf) > 1 and suf[0] in "eE":
        e = _go_parse_int64(suf[1:])
        if e is None:
            return 0, ERR
        e = (e + (1 << 31)) % (1 << 32) - (1 << 31)  # int32(parsed)
        fast = len(num) + len(den) <= 18 and e - len(den) >= -9
        if e > 400 and x != 0:
            x = Fraction(MAXV + 1)  # beyond 2^63 - 1 anyway
        elif e < -400:
            x = Fraction(1, 10 ** 400) if x != 0 else Fraction(0)  # rounds up to 1 anyway
        else:
            x *= Fraction(10) ** e
    else:
        return 0, ERR
    if not binary and x > MAXV:
        return 0, UNSUP
    if neg and not fast and x != 0:
        return 0, UNSUP
    if x > MAXV:
        x = Fraction(MAXV)
    mag = -((-x.numerator) // x.denominator)  # ceil
    return (-mag if neg else mag), OK
