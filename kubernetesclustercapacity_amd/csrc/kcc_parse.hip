// kcc_parse.hip — batch conversion of resource-quantity strings to the int64s the hot
// path consumes (the caller side of the reduce):
//
//   MODE_CPU_MILLIS  convertCPUToMilis   CC:301-319  (container cpu request / limit
//                    strings, CC:279-283; node allocatable cpu, CC:196-197)
//   MODE_BYTES       bytefmt.ToBytes     BF:75-105   (node allocatable memory, CC:199-206)
//
// Input: Arrow-style packed strings, string i = bytes[offsets[i], offsets[i+1]).
// Output: value[i] and status[i] (PARSE_OK; PARSE_ERR where the reference reports an
// error and uses 0; PARSE_UNSUPPORTED outside the exact domain of MODE_BYTES, see
// bytes_value(); PARSE_BADOFF for offsets outside [0, n_bytes] or decreasing).
//
// Byte work, HBM-bound: a workgroup owns PS_BLOCK consecutive strings,
// stages their offsets and their character span in LDS with coalesced dword loads, and
// each lane parses PS_PER_THREAD strings out of LDS (strided by the workgroup size, so a
// wave's lanes read neighbouring strings).  A span too long for the LDS buffer is read
// straight from global memory by the same parser (same results, slower).
#include "kcc_internal.h"

namespace kcc {
namespace {

constexpr int PS_THREADS = 256;
constexpr int PS_PER_THREAD = 4;
constexpr int PS_BLOCK = PS_THREADS * PS_PER_THREAD;  // strings per workgroup
constexpr int PC_PER_THREAD = 4;  // parse_cpu_kernel: strings per lane (8: equal or slower, 86 VGPRs)
constexpr int PC_BLOCK = PS_THREADS * PC_PER_THREAD;
// parse_quantity_kernel: strings per lane (51 VGPRs at 4): 4 -> 8 took C4's 39.6M memory
// strings 0.260 -> 0.233 ms
constexpr int PQ_PER_THREAD = 8;
constexpr int PQ_BLOCK = PS_THREADS * PQ_PER_THREAD;
constexpr int PS_LDS_WORDS = 6144;                    // 24 KiB of staged characters
// a parsed value and its status (written once, read by a later launch): streaming stores
__device__ __forceinline__ void put_parsed(int64_t* out, int8_t* status, int64_t i, int64_t v, int8_t st) {
  __builtin_nontemporal_store(v, out + i);
  __builtin_nontemporal_store(st, status + i);
}

__device__ __forceinline__ bool go_space(uint32_t c) {
  // strings.TrimSpace on ASCII input: '\t', '\n', '\v', '\f', '\r', ' '
  return c == ' ' || (c >= 9 && c <= 13);
}
__device__ __forceinline__ bool go_letter(uint32_t c) {
  // unicode.IsLetter on ASCII; a byte >= 0x80 starts a non-ASCII rune and is taken as a
  // letter (as in oracle/kcc_oracle.c; Quantity.String() emits ASCII only)
  return ((c | 0x20u) - 'a') < 26u || c >= 0x80u;
}
__device__ __forceinline__ uint32_t up(uint32_t c) { return (c - 'a') < 26u ? c - 32u : c; }

// Go strconv.Atoi (64-bit int) on s[0, n): ParseInt base 10 — optional sign, at least
// one digit, no underscores (base given), range error beyond int64.
template <class P>
__device__ __forceinline__ bool go_atoi(P s, int n, int64_t& out) {
  int i = 0;
  bool neg = false;
  if (n <= 0) return false;
  const uint32_t c0 = s[0];
  if (c0 == '+' || c0 == '-') {
    neg = c0 == '-';
    i = 1;
  }
  if (i == n) return false;
  // v * 10 + d <= lim  with lim = 2^63 - 1 (or 2^63 negative): lim / 10 = 922337203685477580
  const uint64_t q = 922337203685477580ull;
  const uint32_t r = neg ? 8u : 7u;
  uint64_t v = 0;
  for (; i < n; ++i) {
    const uint32_t d = (uint32_t)s[i] - '0';
    if (d > 9u) return false;
    if (v > q || (v == q && d > r)) return false;  // ErrRange
    v = v * 10u + d;
  }
  out = neg ? (int64_t)(0ull - v) : (int64_t)v;
  return true;
}

// convertCPUToMilis (CC:301-319): one trailing 'm' means millicores, otherwise cores
// times 1000 (Go int multiply: wraps); an Atoi failure prints and yields 0.
template <class P>
__device__ __forceinline__ uint64_t cpu_millis_value(P s, int n, int8_t& st) {
  bool cores = true;
  if (n > 0 && (uint32_t)s[n - 1] == 'm') {  // HasSuffix / TrimSuffix: one 'm'
    --n;
    cores = false;
  }
  int64_t v;
  if (!go_atoi(s, n, v)) {
    st = PARSE_ERR;
    return 0;
  }
  st = PARSE_OK;
  return cores ? (uint64_t)v * 1000ull : (uint64_t)v;
}

// amd64 CVTTSD2SQ (Go's float64 -> int64 on amd64): truncation, 0x8000000000000000 when
// out of range.  v is finite and >= 0 here.
__device__ __forceinline__ int64_t f2i_amd64(double v) {
  return v >= 9223372036854775808.0 ? (int64_t)0x8000000000000000ull : (int64_t)v;
}

__device__ __forceinline__ double p10(int k) {  // exact for k <= 22
  double r = 1.0;
  double b = 10.0;
  while (k) {
    if (k & 1) r *= b;
    b *= b;
    k >>= 1;
  }
  return r;
}

// Correctly rounded D / 10^k for 1 <= k <= 38 (D >= 1): restoring division until the
// quotient holds 57 bits, then round-half-even to 53 bits with the remainder as sticky.
__device__ __noinline__ double div_pow10_rn(uint64_t D, int k) {
  unsigned __int128 V = 1;
  for (int t = 0; t < k; ++t) V *= 10u;  // < 2^127
  unsigned __int128 R = 0;
  uint64_t q = 0;
  int bit = 63;   // next bit of D to bring down
  int extra = 0;  // zero bits brought down after D's last bit
  while (q < (1ull << 56)) {
    uint32_t b = 0;
    if (bit >= 0) {
      b = (uint32_t)(D >> bit) & 1u;
      --bit;
    } else {
      ++extra;
    }
    R = (R << 1) | b;
    q <<= 1;
    if (R >= V) {
      R -= V;
      q |= 1u;
    }
  }
  // x = (q + f) * 2^e2,  f in [0, 1),  f > 0 iff sticky
  bool sticky = R != 0;
  int e2;
  if (bit >= 0) {
    sticky |= (D & ((2ull << bit) - 1u)) != 0;
    e2 = bit + 1;
  } else {
    e2 = -extra;
  }
  // q in [2^56, 2^57): drop 4 bits
  const uint32_t low = (uint32_t)(q & 15u);
  q >>= 4;
  e2 += 4;
  const bool guard = (low & 8u) != 0;
  const bool rest = (low & 7u) != 0 || sticky;
  if (guard && (rest || (q & 1u))) {
    ++q;
    if (q == (1ull << 53)) {
      q >>= 1;
      ++e2;
    }
  }
  return ldexp((double)q, e2);
}

// D / 10^k correctly rounded, 1 <= k <= 38
__device__ __forceinline__ double frac_rn(uint64_t D, int k) {
  if (D < (1ull << 53) && k <= 22) return (double)D / p10(k);  // exact operands: one rounding
  return div_pow10_rn(D, k);
}

// bytefmt.ToBytes (BF:75-105): TrimSpace, ToUpper, split at the first letter,
// ParseFloat(number, 64) > 0, multiple in {T,TB,TIB | G,GB,GIB | M,MB,MIB,MI |
// K,KB,KIB,KI | B}, int64(bytes * multiple).
//
// The number is [sign] digits [. digits] (no letters: the split is at the first one).
// Exact domain on the device: values >= 10^19 (int64() overflows to 0x8000000000000000
// whatever the rounding), < 10^-19 (the product truncates to 0), and in between any
// digit string whose first 19 significant digits D decide the rounding (all of them
// when there are at most 19; otherwise when D and D+1 round alike).  Outside it (a value
// at the float64 overflow or underflow edge, 10^308 <= x < 10^309 or 10^-324 <= x <
// 10^-323, or > 19 significant digits straddling a rounding boundary) the status is
// PARSE_UNSUPPORTED — never a silently different value.
template <class P>
__device__ __forceinline__ int64_t bytes_value(P s, int n, int8_t& st) {
  int b = 0, e = n;
  while (b < e && go_space((uint32_t)s[b])) ++b;
  while (e > b && go_space((uint32_t)s[e - 1])) --e;
  int i = b;
  while (i < e && !go_letter((uint32_t)s[i])) ++i;
  st = PARSE_ERR;
  if (i == e) return 0;  // no letter: invalidByteQuantityError (BF:81-83)
  // the multiple (BF:91-104), upper-cased
  const int ml = e - i;
  const uint32_t m0 = up(s[i]);
  const uint32_t m1 = ml > 1 ? up(s[i + 1]) : 0u;
  const uint32_t m2 = ml > 2 ? up(s[i + 2]) : 0u;
  int shift = -1;
  if (ml <= 3) {
    if (m0 == 'B') {
      shift = ml == 1 ? 0 : -1;
    } else if (m0 == 'T' || m0 == 'G' || m0 == 'M' || m0 == 'K') {
      const int sh = m0 == 'T' ? 40 : m0 == 'G' ? 30 : m0 == 'M' ? 20 : 10;
      const bool ok1 = ml == 1 || (ml == 2 && m1 == 'B') || (ml == 3 && m1 == 'I' && m2 == 'B') ||
                       (ml == 2 && m1 == 'I' && (m0 == 'M' || m0 == 'K'));
      shift = ok1 ? sh : -1;
    }
  }
  // ParseFloat(s[b:i])
  int j = b;
  bool neg = false;
  if (j < i && ((uint32_t)s[j] == '+' || (uint32_t)s[j] == '-')) {
    neg = (uint32_t)s[j] == '-';
    ++j;
  }
  bool dot = false, trunc_nz = false;
  int digits = 0, sig = 0, e10 = 0;
  uint64_t D = 0;
  for (; j < i; ++j) {
    const uint32_t c = s[j];
    const uint32_t d = c - '0';
    if (d <= 9u) {
      ++digits;
      if (sig == 0 && d == 0) {  // leading zero
        if (dot) --e10;
        continue;
      }
      if (sig < 19) {
        D = D * 10u + d;
        ++sig;
        if (dot) --e10;
      } else {  // beyond 19 significant digits
        trunc_nz |= d != 0;
        if (!dot) ++e10;
      }
    } else if (c == '.' && !dot) {
      dot = true;
    } else {
      return 0;  // syntax error
    }
  }
  if (digits == 0 || D == 0 || neg || shift < 0) return 0;  // error, or bytes <= 0
  const int mag = sig + e10;  // x in [10^(mag-1), 10^mag)
  if (mag >= 310) return 0;   // ParseFloat ErrRange (rounds to +Inf)
  if (mag == 309) {
    st = PARSE_UNSUPPORTED;
    return 0;
  }
  if (mag >= 20) {  // x >= 10^19 > 2^63: int64() overflows
    st = PARSE_OK;
    return (int64_t)0x8000000000000000ull;
  }
  double x;
  if (e10 >= 0) {
    uint64_t v = D;  // mag <= 19: the integer fits 64 bits
    for (int t = 0; t < e10; ++t) v *= 10u;
    x = (double)v;  // u64 -> f64, correctly rounded
  } else {
    const int k = -e10;
    if (k > 38) {  // x < 10^-19: the product truncates to 0; only the status depends on x
      if (mag >= -322) {
        st = PARSE_OK;  // x > 2^-1075: rounds to a positive double
      } else if (mag == -323) {
        st = PARSE_UNSUPPORTED;
      }  // mag <= -324: rounds to 0, bytes <= 0 -> error
      return 0;
    }
    x = frac_rn(D, k);
    // more than 19 significant digits: x lies in [D, D+1) x 10^-k; when both ends round
    // to the same double so does x (Go's own test for a truncated mantissa, atof.go)
    if (trunc_nz && frac_rn(D + 1u, k) != x) {
      st = PARSE_UNSUPPORTED;
      return 0;
    }
  }
  st = PARSE_OK;
  return f2i_amd64(ldexp(x, shift));  // times a power of two: exact
}

// resource.Quantity.Value() of ParseQuantity(s) (k8s.io/apimachinery resource/quantity.go;
// the reference's per-container memory, CC:285-286).  Restated from the published
// algorithm — apimachinery is not vendored and its version is unpinned (DESIGN.md §4.6:
// parity unpinned): [+-] digits [. digits] then a suffix — "", Ki..Ei (2^10k), n u m k M
// G T P E (10^3k), or e/E<int64> (10^int32(exp)); parse errors (ErrFormatWrong /
// ErrSuffix) -> PARSE_ERR.  Value() rounds up away from zero; binary amounts are capped at
// 2^63 - 1 (ParseQuantity caps only BinarySI): v = sign * min(ceil(|x|), 2^63 - 1).
// PARSE_UNSUPPORTED: a decimal amount beyond 2^63 - 1 (k8s wraps it, path-dependent), a
// negative amount off ParseQuantity's int64 fast path (rounding not pinned), and binary
// suffixes with a fraction of more than 19 significant digits.
__device__ __forceinline__ bool mul10_sat(uint64_t& v, uint32_t d) {  // v = v*10 + d, false on > 2^63-1
  const uint64_t lim = 0x7fffffffffffffffull;
  if (v > (lim - d) / 10u) return false;
  v = v * 10u + d;
  return true;
}

template <class P>
__device__ __forceinline__ int64_t quantity_value(P s, int n, int8_t& st) {
  const uint64_t MAXV = 0x7fffffffffffffffull;
  st = PARSE_ERR;
  if (n == 0) return 0;  // ErrFormatWrong
  int i = 0;
  bool neg = false;
  if ((uint32_t)s[0] == '-' || (uint32_t)s[0] == '+') {
    neg = (uint32_t)s[0] == '-';
    i = 1;
  }
  while (i < n && (uint32_t)s[i] == '0') ++i;  // leading zeros
  if (i >= n) {  // all zeros (or a bare sign): 0
    st = PARSE_OK;
    return 0;
  }
  const int num0 = i;
  while (i < n && (uint32_t)s[i] - '0' <= 9u) ++i;
  const int num1 = i;  // numerator digits [num0, num1)
  int den0 = i, den1 = i;
  if (i < n && (uint32_t)s[i] == '.') {
    ++i;
    den0 = i;
    while (i < n && (uint32_t)s[i] - '0' <= 9u) ++i;
    den1 = i;
  }
  // suffix: letters of "eEinumkKMGTP", then an optional sign, then digits, to the end
  const int suf0 = i;
  auto suffix_letter = [](uint32_t c) {
    return c == 'e' || c == 'E' || c == 'i' || c == 'n' || c == 'u' || c == 'm' || c == 'k' ||
           c == 'K' || c == 'M' || c == 'G' || c == 'T' || c == 'P';
  };
  while (i < n && suffix_letter((uint32_t)s[i])) ++i;
  if (i < n && ((uint32_t)s[i] == '+' || (uint32_t)s[i] == '-')) ++i;
  while (i < n && (uint32_t)s[i] - '0' <= 9u) ++i;
  if (i < n) return 0;  // ErrFormatWrong
  // interpret the suffix
  const int sl = n - suf0;
  const uint32_t a0 = sl > 0 ? (uint32_t)s[suf0] : 0u, a1 = sl > 1 ? (uint32_t)s[suf0 + 1] : 0u;
  bool binary = false;
  int64_t e10 = 0;
  int bexp = 0;
  if (sl == 0) {
  } else if (sl == 2 && a1 == 'i' &&
             (a0 == 'K' || a0 == 'M' || a0 == 'G' || a0 == 'T' || a0 == 'P' || a0 == 'E')) {
    binary = true;
    bexp = a0 == 'K' ? 10 : a0 == 'M' ? 20 : a0 == 'G' ? 30 : a0 == 'T' ? 40 : a0 == 'P' ? 50 : 60;
  } else if (sl == 1 && (a0 == 'n' || a0 == 'u' || a0 == 'm' || a0 == 'k' || a0 == 'M' ||
                         a0 == 'G' || a0 == 'T' || a0 == 'P' || a0 == 'E')) {
    e10 = a0 == 'n' ? -9 : a0 == 'u' ? -6 : a0 == 'm' ? -3 : a0 == 'k' ? 3 : a0 == 'M' ? 6
        : a0 == 'G' ? 9 : a0 == 'T' ? 12 : a0 == 'P' ? 15 : 18;
  } else if (sl > 1 && (a0 == 'e' || a0 == 'E')) {  // strconv.ParseInt(suffix[1:], 10, 64)
    int64_t x;
    if (!go_atoi(s + suf0 + 1, sl - 1, x)) return 0;  // ErrSuffix
    e10 = (int64_t)(int32_t)(uint32_t)(uint64_t)x;     // int32(parsed)
  } else {
    return 0;  // ErrSuffix
  }
  const int nd = (num1 - num0) + (den1 - den0);  // significant-or-not digits after the zeros
  uint64_t I = 0;
  bool over = false, frac = false;
  if (!binary) {
    // x = digits x 10^(e10 - |denom|): the first (|num| + e10) digits are the integer part
    const int64_t intlen = (int64_t)(num1 - num0) + e10;
    int64_t k = 0;
    for (int j = num0; j < den1; ++j) {
      if (j == num1) continue;  // the point
      const uint32_t d = (uint32_t)s[j] - '0';
      if (k < intlen) {
        if (!over && !mul10_sat(I, d)) over = true;
      } else {
        frac |= d != 0;
      }
      ++k;
    }
    if (!over && intlen > nd && I != 0) {  // the exponent's trailing zeros (0 stays 0)
      if (intlen - nd > 19) {
        over = true;
      } else {
        for (int64_t t = nd; t < intlen; ++t)
          if (!mul10_sat(I, 0)) {
            over = true;
            break;
          }
      }
    }
  } else {
    // x = D x 2^bexp / 10^f exactly, D the digits (<= 19 significant)
    uint64_t D = 0;
    int sig = 0, f = den1 - den0;
    bool trunc = false;
    for (int j = num0; j < den1; ++j) {
      if (j == num1) continue;
      const uint32_t d = (uint32_t)s[j] - '0';
      if (sig == 0 && d == 0) continue;
      if (sig < 19) {
        D = D * 10u + d;
        ++sig;
      } else {
        trunc |= d != 0;
        if (j < num1) {  // an integer digit beyond 19: the value is >= 10^19 > cap
          over = true;
        } else {
          --f;  // fractional zero digits past the 19th are dropped exactly
        }
      }
    }
    if (trunc && !over) {
      st = PARSE_UNSUPPORTED;
      return 0;
    }
    // (f counts fraction digits kept in D: f - (dropped zeros))
    if (!over) {
      unsigned __int128 N = (unsigned __int128)D << bexp;  // < 2^124
      unsigned __int128 Q = N;
      if (f > 0) {
        if (f > 38) {
          st = PARSE_UNSUPPORTED;
          return 0;
        }
        unsigned __int128 V = 1;
        for (int t = 0; t < f; ++t) V *= 10u;
        // restoring division N / V
        unsigned __int128 R = 0;
        Q = 0;
        for (int b = 127; b >= 0; --b) {
          R = (R << 1) | (unsigned __int128)((N >> b) & 1u);
          Q <<= 1;
          if (R >= V) {
            R -= V;
            Q |= 1u;
          }
        }
        frac = R != 0;
      }
      if (Q > (unsigned __int128)MAXV) over = true;
      else I = (uint64_t)Q;
    }
  }
  // ParseQuantity's int64 fast path: <= 18 digits at a scale >= -9 (decimal suffixes), no
  // fraction and 14 - 3k digits at most (2^10k)
  const int nnum = num1 - num0, nden = den1 - den0;
  const bool fast = binary ? (nden == 0 && nnum <= 14 - 3 * (bexp / 10))
                           : (nnum + nden <= 18 && e10 - nden >= -9);
  uint64_t mag;
  if (over) {
    if (!binary) {  // a decimal amount beyond 2^63 - 1: k8s wraps it (path-dependent)
      st = PARSE_UNSUPPORTED;
      return 0;
    }
    mag = MAXV;  // binary amounts are capped at maxAllowed
  } else {
    mag = I + (frac ? 1u : 0u);  // rounded up away from zero
    if (mag > MAXV) {
      if (!binary) {
        st = PARSE_UNSUPPORTED;
        return 0;
      }
      mag = MAXV;
    }
  }
  if (neg && !fast && mag != 0) {  // off the int64 path, negative: rounding not pinned
    st = PARSE_UNSUPPORTED;
    return 0;
  }
  st = PARSE_OK;
  return neg ? -(int64_t)mag : (int64_t)mag;
}

template <int MODE, class P>
__device__ __forceinline__ void parse_one(P s, int n, int64_t& v, int8_t& st) {
  if (MODE == PARSE_MODE_CPU_MILLIS)
    v = (int64_t)cpu_millis_value(s, n, st);
  else if (MODE == PARSE_MODE_BYTES)
    v = bytes_value(s, n, st);
  else
    v = quantity_value(s, n, st);
}

template <int MODE>
__global__ __launch_bounds__(PS_THREADS) void parse_kernel(int64_t n, const uint8_t* __restrict__ bytes,
                                                           int64_t n_bytes,
                                                           const int64_t* __restrict__ off,
                                                           int64_t* __restrict__ out,
                                                           int8_t* __restrict__ status) {
  __shared__ int64_t s_off[PS_BLOCK + 1];
  __shared__ uint32_t s_chr[PS_LDS_WORDS];
  const int64_t base = (int64_t)blockIdx.x * PS_BLOCK;
  const int cnt = (int)min((int64_t)PS_BLOCK, n - base);
  for (int t = threadIdx.x; t <= cnt; t += PS_THREADS) s_off[t] = off[base + t];
  __syncthreads();
  const int64_t b0 = max(s_off[0], (int64_t)0);
  const int64_t b1 = min(max(s_off[cnt], b0), n_bytes);
  const int64_t w0 = b0 >> 2, w1 = (b1 + 3) >> 2;
  const bool staged = w1 - w0 <= PS_LDS_WORDS;  // uniform over the workgroup
  if (staged) {
    const uint32_t* __restrict__ wp = reinterpret_cast<const uint32_t*>(bytes);
    const int64_t full = n_bytes >> 2;  // words entirely inside the buffer
    for (int64_t t = threadIdx.x; t < w1 - w0; t += PS_THREADS) {
      const int64_t w = w0 + t;
      uint32_t v = 0;
      if (w < full) {
        v = __builtin_nontemporal_load(wp + w);
      } else {
        for (int k = 0; k < 4; ++k)
          if (w * 4 + k < n_bytes) v |= (uint32_t)bytes[w * 4 + k] << (8 * k);
      }
      s_chr[t] = v;
    }
  }
  __syncthreads();
  const uint8_t* lds = reinterpret_cast<const uint8_t*>(s_chr);
#pragma unroll
  for (int r = 0; r < PS_PER_THREAD; ++r) {
    const int li = r * PS_THREADS + (int)threadIdx.x;
    if (li >= cnt) break;
    const int64_t sb = s_off[li], se = s_off[li + 1];
    int64_t v = 0;
    int8_t st = PARSE_BADOFF;
    if (sb >= 0 && se >= sb && se <= n_bytes && se - sb < ((int64_t)1 << 31)) {
      if (staged && sb >= b0 && se <= b1)
        parse_one<MODE>(lds + (sb - w0 * 4), (int)(se - sb), v, st);
      else
        parse_one<MODE>(bytes + sb, (int)(se - sb), v, st);
    }
    out[base + li] = v;
    status[base + li] = st;
  }
}

// Eight ASCII characters (the first in the low byte) -> their decimal value, when all
// eight are digits: nibble tests, then three multiply-shift steps that combine digit
// pairs, quads and the two halves (SWAR).
__device__ __forceinline__ bool swar8(uint64_t c, uint64_t& v) {
  const uint64_t hi = 0xF0F0F0F0F0F0F0F0ull, z = 0x3030303030303030ull;
  if ((c & hi) != z || ((c + 0x0606060606060606ull) & hi) != z) return false;
  c = ((c & 0x0F0F0F0F0F0F0F0Full) * 2561u) >> 8;
  c = ((c & 0x00FF00FF00FF00FFull) * 6553601u) >> 16;
  v = ((c & 0x0000FFFF0000FFFFull) * 42949672960001ull) >> 32;
  return true;
}

// convertCPUToMilis without LDS: one lane per string.  Strings of <= 9 characters (all
// canonical cpu quantities up to 99999999m / 99999999 cores) come from one aligned
// 12-byte load per lane — neighbouring lanes read neighbouring bytes, so a wave's loads
// coalesce into the few cache lines its strings span — and are parsed in registers
// (swar8); anything else takes the byte loop over global memory.  PC_PER_THREAD strings
// per lane, strided by the workgroup size, all loads issued before the first parse.
__global__ __launch_bounds__(PS_THREADS) void parse_cpu_kernel(int64_t n, const uint8_t* __restrict__ bytes,
                                                               int64_t n_bytes,
                                                               const int64_t* __restrict__ off,
                                                               int64_t* __restrict__ out,
                                                               int8_t* __restrict__ status) {
  const int64_t b0 = (int64_t)blockIdx.x * PC_BLOCK;
  const int64_t base = b0 + threadIdx.x;
  // the workgroup's character span, for one range-checked buffer descriptor: loads past
  // it (or past n_bytes) read 0 instead of faulting, so every load is unconditional
  const int64_t cnt = min((int64_t)PC_BLOCK, n - b0);
  const int64_t lo_b = max(off[b0], (int64_t)0) & ~(int64_t)3;
  const int64_t hi_b = min(off[b0 + cnt], n_bytes);
  const bool span_ok = hi_b > lo_b && hi_b - lo_b < ((int64_t)1 << 31);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(bytes + (span_ok ? lo_b : 0)), (short)0, span_ok ? (int)(hi_b - lo_b) : 0,
      0x00020000);
  int64_t sb[PC_PER_THREAD], se[PC_PER_THREAD];
  uint32_t w[PC_PER_THREAD][3];
  bool fast[PC_PER_THREAD];
#pragma unroll
  for (int r = 0; r < PC_PER_THREAD; ++r) {
    const int64_t i = min(base + r * PS_THREADS, n - 1);
    sb[r] = off[i];
    se[r] = off[i + 1];
  }
#pragma unroll
  for (int r = 0; r < PC_PER_THREAD; ++r) {
    const int64_t a = sb[r] & ~(int64_t)3;
    const int64_t L = se[r] - sb[r];
    fast[r] = span_ok && sb[r] >= lo_b && L >= 1 && L <= 9 && a + 12 <= hi_b;
    typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
    const u32x3 x = __builtin_bit_cast(
        u32x3, __builtin_amdgcn_raw_buffer_load_b96(rs, fast[r] ? (int)(a - lo_b) : 0x7ffffff0, 0, 0));
    w[r][0] = x.x;
    w[r][1] = x.y;
    w[r][2] = x.z;
  }
#pragma unroll
  for (int r = 0; r < PC_PER_THREAD; ++r) {
    const int64_t i = base + r * PS_THREADS;
    if (i >= n) break;
    int64_t v = 0;
    int8_t st = PARSE_BADOFF;
    bool done = false;
    if (fast[r]) {
      const int L = (int)(se[r] - sb[r]);
      const int sh = (int)(sb[r] & 3) * 8;
      const uint64_t lo = ((uint64_t)w[r][1] << 32) | w[r][0];
      const uint64_t hi = w[r][2];
      const uint64_t c = sh ? (lo >> sh) | (hi << (64 - sh)) : lo;  // characters 0..7
      const uint32_t last = L == 9 ? (uint32_t)(hi >> sh) & 0xffu : (uint32_t)(c >> (8 * (L - 1))) & 0xffu;
      const bool milli = last == 'm';
      const int d = L - (milli ? 1 : 0);
      const uint32_t c0 = (uint32_t)c & 0xffu;
      if (d >= 1 && d <= 8 && c0 != '+' && c0 != '-') {
        // d digits, left-padded with '0' to eight
        const uint64_t cp =
            d == 8 ? c : (c << (8 * (8 - d))) | (0x3030303030303030ull >> (8 * d));
        uint64_t x;
        if (swar8(cp, x)) {
          v = (int64_t)(milli ? x : x * 1000u);
          st = PARSE_OK;
        } else {
          st = PARSE_ERR;  // unsigned, non-digit inside: strconv.Atoi fails
        }
        done = true;
      }
    }
    if (!done && sb[r] >= 0 && se[r] >= sb[r] && se[r] <= n_bytes && se[r] - sb[r] < ((int64_t)1 << 31))
      v = (int64_t)cpu_millis_value(bytes + sb[r], (int)(se[r] - sb[r]), st);
    put_parsed(out, status, i, v, st);
  }
}

// The general parser for the strings the register path does not take, out of line (one
// copy instead of one per unrolled string; the result comes back in registers).
struct QtyResult {
  int64_t v;
  int32_t st;
};
__device__ __noinline__ QtyResult quantity_value_global(const uint8_t* s, int n) {
  int8_t st;
  const int64_t v = quantity_value(s, n, st);
  return QtyResult{v, st};
}

// Character classes for qty_fast2 (one LDS byte per character): bit 7 a digit; bits 0-2 the
// decimal suffix k M G T P E (10^3k: 1..6; 'K' alone is none); bits 3-5 the binary prefix
// K M G T P E of "Ki".."Ei" (2^10k: 1..6); bit 6 'i'.
__host__ __device__ constexpr uint32_t qty_class(uint32_t ch) {
  return (ch - '0' <= 9u) ? 0x80u
       : ch == 'i' ? 0x40u
       : ch == 'k' ? 1u
       : ch == 'K' ? (1u << 3)
       : ch == 'M' ? (2u | (2u << 3))
       : ch == 'G' ? (3u | (3u << 3))
       : ch == 'T' ? (4u | (4u << 3))
       : ch == 'P' ? (5u | (5u << 3))
       : ch == 'E' ? (6u | (6u << 3)) : 0u;
}

// The register fast path of Quantity.Value() (round 4; replaced round 2's qty_fast, whose
// contract it keeps: the same accepted strings, values and statuses, fewer VALU): the suffix
// from the character-class table; the digits right-aligned by ONE 128-bit shift left by
// 8 x (16 - d) bytes' worth of bits — the suffix and whatever follows the string fall off
// the top, zeros (leading '0' digits) come in at the bottom, so no masks and no exact
// division by 10^(16 - d); four digits per word from two v_dot4_u32_u8 (10 b0 + b1,
// 10 b2 + b3) and a 24-bit multiply-add.
[[maybe_unused]] __device__ __forceinline__ bool qty_fast2(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3,
                                          uint32_t al, int L, const uint8_t* s_cls,
                                          const uint64_t* s_p10, const uint64_t* s_lim,
                                          int64_t& v, int8_t& st) {
  const uint64_t MAXV = 0x7fffffffffffffffull;
  const uint32_t a0 = __builtin_amdgcn_alignbyte(w1, w0, al);
  const uint32_t a1 = __builtin_amdgcn_alignbyte(w2, w1, al);
  const uint32_t a2 = __builtin_amdgcn_alignbyte(w3, w2, al);
  const uint32_t a3 = __builtin_amdgcn_alignbyte(0u, w3, al);
  // the last two characters: the 16 bits at byte p = L - 2 (L = 1: at 0, shifted)
  const uint32_t p = L >= 2 ? (uint32_t)(L - 2) : 0u;
  const uint32_t q = p >> 2;  // 0..2
  const uint32_t lo = q == 0 ? a0 : (q == 1 ? a1 : a2);
  const uint32_t hi = q == 0 ? a1 : (q == 1 ? a2 : a3);
  const uint32_t pair = __builtin_amdgcn_alignbyte(hi, lo, p & 3u);
  const uint32_t z = L >= 2 ? (pair >> 8) & 0xffu : pair & 0xffu;  // last
  const uint32_t y = L >= 2 ? pair & 0xffu : 0u;                    // second last
  const uint32_t zc = s_cls[z], yc = s_cls[y];
  const bool bin = (zc & 0x40u) != 0u && (yc & 0x38u) != 0u;  // "Ki".."Ei"
  const uint32_t zd = zc & 7u;                                  // k M G T P E
  const bool dec = !bin && zd != 0u;
  const bool dig = (zc & 0x80u) != 0u;
  const int d = L - (bin ? 2 : (dec ? 1 : 0));  // the digits
  // T = (characters - '0') << (128 - 8d): the d digits end at byte 15
  const uint64_t ZZ = 0x3030303030303030ull;
  const uint64_t l64 = (((uint64_t)a1 << 32) | a0) ^ ZZ;
  const uint64_t h64 = (((uint64_t)a3 << 32) | a2) ^ ZZ;
  const uint32_t sh = (uint32_t)(128 - 8 * d);  // 24..120 on the fast path
  const uint64_t xl = l64 << (sh & 63u);
  const bool big = sh >= 64u;
  const uint64_t th = big ? xl : ((h64 << (sh & 63u)) | (l64 >> ((64u - sh) & 63u)));
  const uint64_t tl = big ? 0ull : xl;
  const uint32_t t0 = (uint32_t)tl, t1 = (uint32_t)(tl >> 32), t2 = (uint32_t)th, t3 = (uint32_t)(th >> 32);
  const uint32_t H = 0x76767676u;  // a byte > 9 sets bit 7 of t + 0x76 or of t itself
  const uint32_t bad = ((t0 + H) | t0 | (t1 + H) | t1 | (t2 + H) | t2 | (t3 + H) | t3) & 0x80808080u;
  // four digits per word (the first in the low byte): (10 b0 + b1) x 100 + 10 b2 + b3
  // (the second dot4 accumulates 100 x the first; no inline asm here: a VALU read of a
  // dot4 result needs a wait state the compiler inserts only around instructions it sees)
  auto quad = [](uint32_t t) -> uint32_t {
    const uint32_t hi2 = __builtin_amdgcn_udot4(t, 0x0000010au, 0u, false);
    return __builtin_amdgcn_udot4(t, 0x010a0000u, __umul24(hi2, 100u), false);
  };
  const uint32_t q01 = __umul24(quad(t0), 10000u) + quad(t1);
  const uint32_t q23 = __umul24(quad(t2), 10000u) + quad(t3);
  const uint64_t D = (uint64_t)q01 * 100000000u + q23;  // < 10^13
  const bool ok = (bin || dec || dig) && d >= 1 && bad == 0;
  const int bexp = bin ? 10 * (int)((yc >> 3) & 7u) : 0;
  uint64_t mag = D > (MAXV >> bexp) ? MAXV : D << bexp;
  st = PARSE_OK;
  if (dec) {
    const bool over = D > s_lim[zd];
    mag = over ? 0 : D * s_p10[zd];
    st = over ? PARSE_UNSUPPORTED : PARSE_OK;
  }
  v = (int64_t)mag;
  return ok;
}

// Quantity.Value() without LDS, as parse_cpu_kernel: one lane per string, strings of
// <= 13 characters from one aligned 16-byte buffer load per lane, parsed in registers
// (qty_fast2) when they are plain digits (<= 13) and an optional integral suffix — k M G
// T P E (10^3k) or Ki Mi Gi Ti Pi Ei (2^10k) — which covers every canonical memory
// quantity of a container (Quantity.String() of a BinarySI or DecimalSI integer amount);
// the value is capped at 2^63 - 1 exactly as quantity_value does.  Anything else (a sign,
// a fraction, an exponent, m/u/n, a malformed string) takes quantity_value over global
// memory, so the results are identical by construction.
__global__ __launch_bounds__(PS_THREADS) void parse_quantity_kernel(int64_t n, const uint8_t* __restrict__ bytes,
                                                                    int64_t n_bytes,
                                                                    const int64_t* __restrict__ off,
                                                                    int64_t* __restrict__ out,
                                                                    int8_t* __restrict__ status) {
  const uint64_t MAXV = 0x7fffffffffffffffull;
  // 10^3k and (2^63 - 1) / 10^3k (k = 0..6)
  __shared__ uint64_t s_p10[8], s_lim[8];
  __shared__ uint8_t s_cls[256];  // qty_class of every byte value
  s_cls[threadIdx.x] = (uint8_t)qty_class(threadIdx.x);  // (256 threads)
  if (threadIdx.x < 8) {
    uint64_t p = 1;
    for (unsigned k = 0; k < threadIdx.x && k < 6; ++k) p *= 1000u;
    s_p10[threadIdx.x] = p;
    s_lim[threadIdx.x] = MAXV / p;
  }
  __syncthreads();
  const int64_t b0 = (int64_t)blockIdx.x * PQ_BLOCK;
  const int64_t base = b0 + threadIdx.x;
  const int64_t cnt = min((int64_t)PQ_BLOCK, n - b0);
  const int64_t lo_b = max(off[b0], (int64_t)0) & ~(int64_t)3;
  const int64_t hi_b = min(off[b0 + cnt], n_bytes);
  const bool span_ok = hi_b > lo_b && hi_b - lo_b < ((int64_t)1 << 31);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(bytes + (span_ok ? lo_b : 0)), (short)0, span_ok ? (int)(hi_b - lo_b) : 0,
      0x00020000);
  int64_t sb[PQ_PER_THREAD], se[PQ_PER_THREAD];
  uint32_t w[PQ_PER_THREAD][4];
  bool fast[PQ_PER_THREAD];
#pragma unroll
  for (int r = 0; r < PQ_PER_THREAD; ++r) {
    const int64_t i = min(base + r * PS_THREADS, n - 1);
    sb[r] = off[i];
    se[r] = off[i + 1];
  }
#pragma unroll
  for (int r = 0; r < PQ_PER_THREAD; ++r) {
    const int64_t a = sb[r] & ~(int64_t)3;
    const int64_t L = se[r] - sb[r];
    fast[r] = span_ok && sb[r] >= lo_b && L >= 1 && L <= 13 && a + 16 <= hi_b;
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 x = __builtin_bit_cast(
        u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, fast[r] ? (int)(a - lo_b) : 0x7ffffff0, 0, 0));
    w[r][0] = x.x;
    w[r][1] = x.y;
    w[r][2] = x.z;
    w[r][3] = x.w;
  }
  // the register path for every string; the ones it does not take (need) go through the
  // general parser afterwards, from one call site (four unrolled call sites shaped the
  // register allocation and branching of the whole loop)
  uint32_t need = 0;
#pragma unroll
  for (int r = 0; r < PQ_PER_THREAD; ++r) {
    const int64_t i = base + r * PS_THREADS;
    if (i >= n) break;
    int64_t v = 0;
    int8_t st = PARSE_BADOFF;
    bool done = false;
    if (fast[r])
      done = qty_fast2(w[r][0], w[r][1], w[r][2], w[r][3], (uint32_t)sb[r], (int)(se[r] - sb[r]),
                       s_cls, s_p10, s_lim, v, st);
    if (!done) {
      need |= 1u << r;  // the offsets' checks and the general parser: below
    } else {
      put_parsed(out, status, i, v, st);
    }
  }
#pragma unroll 1
  for (int r = 0; r < PQ_PER_THREAD; ++r) {
    if (!((need >> r) & 1u)) continue;
    const int64_t i = base + r * PS_THREADS;
    const int64_t b = off[i], e = off[i + 1];
    if (!(b >= 0 && e >= b && e <= n_bytes && e - b < ((int64_t)1 << 31))) {
      out[i] = 0;
      status[i] = PARSE_BADOFF;
      continue;
    }
    const QtyResult q = quantity_value_global(bytes + b, (int)(e - b));
    out[i] = q.v;
    status[i] = (int8_t)q.st;
  }
}

}  // namespace

int64_t parse_grid(int64_t n) { return (n + PS_BLOCK - 1) / PS_BLOCK; }
static int64_t parse_cpu_grid(int64_t n) { return (n + PC_BLOCK - 1) / PC_BLOCK; }
static int64_t parse_qty_grid(int64_t n) { return (n + PQ_BLOCK - 1) / PQ_BLOCK; }

hipError_t launch_parse(int mode, int64_t n, const uint8_t* bytes, int64_t n_bytes,
                        const int64_t* offsets, int64_t* out, int8_t* status, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int64_t grid = parse_grid(n);
  if (grid > 0x7fffffff) return hipErrorInvalidValue;
  if (mode == PARSE_MODE_CPU_MILLIS)
    hipLaunchKernelGGL(parse_cpu_kernel, dim3((unsigned)parse_cpu_grid(n)), dim3(PS_THREADS), 0, s,
                       n, bytes, n_bytes, offsets, out, status);
  else if (mode == PARSE_MODE_BYTES)
    hipLaunchKernelGGL(parse_kernel<PARSE_MODE_BYTES>, dim3((unsigned)grid), dim3(PS_THREADS), 0, s,
                       n, bytes, n_bytes, offsets, out, status);
  else
    hipLaunchKernelGGL(parse_quantity_kernel, dim3((unsigned)parse_qty_grid(n)), dim3(PS_THREADS), 0,
                       s, n, bytes, n_bytes, offsets, out, status);
  return hipGetLastError();
}

}  // namespace kcc
