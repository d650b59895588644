/*
 * kcc_oracle.c — plain C restatement of the reference hot path.
 * TEST INFRASTRUCTURE ONLY (see kcc_oracle.h).  Parity of this file to the Go
 * reference is pinned by the hand-derived KATs of SURVEY.md §8c (no reference
 * goldens exist) and by oracle/pyoracle.py (independent big-int restatement).
 *
 * Go semantics restated exactly:
 *   - uint64/int64 arithmetic wraps (done here in uint64_t and reinterpreted);
 *   - Go `int` is int64 on amd64; int(uint64) reinterprets;
 *   - integer division truncates toward zero; MinInt64 / -1 == MinInt64 (Go spec);
 *   - division by zero panics (reported as a per-spec error flag).
 */
#include "kcc_oracle.h"

#include <ctype.h>
#include <errno.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* CC:255-299: for each pod, for each container, CC:290-293 adds. */
void kcco_reduce_requests(int64_t n_nodes, const int64_t* node_ptr,
                          const uint64_t* cpu_req, const int64_t* mem_req,
                          const uint64_t* cpu_lim, const int64_t* mem_lim,
                          uint64_t* used_cpu, int64_t* used_mem, uint64_t* lim_cpu,
                          int64_t* lim_mem) {
  for (int64_t i = 0; i < n_nodes; ++i) {
    uint64_t cpuReq = 0, cpuLim = 0; /* CC:257-258 (uint64) */
    uint64_t memReq = 0, memLim = 0; /* CC:259-260 (int64, kept as bits) */
    for (int64_t c = node_ptr[i]; c < node_ptr[i + 1]; ++c) {
      cpuReq += cpu_req[c];            /* CC:290 */
      memReq += (uint64_t)mem_req[c];  /* CC:292 */
      if (cpu_lim) cpuLim += cpu_lim[c];            /* CC:291 */
      if (mem_lim) memLim += (uint64_t)mem_lim[c];  /* CC:293 */
    }
    used_cpu[i] = cpuReq;
    used_mem[i] = (int64_t)memReq;
    if (lim_cpu) lim_cpu[i] = cpuLim;
    if (lim_mem) lim_mem[i] = (int64_t)memLim;
  }
}

/* SURVEY §8f row 4 (opt-in, not the reference): see kcc_oracle.h. */
void kcco_pod_requests(int64_t n_pods, const int64_t* pod_ptr, const uint64_t* cpu_req,
                       const int64_t* mem_req, const int64_t* init_ptr,
                       const uint64_t* init_cpu, const int64_t* init_mem,
                       const uint8_t* restartable, const uint64_t* ovh_cpu,
                       const int64_t* ovh_mem, uint64_t* pod_cpu, int64_t* pod_mem) {
  for (int64_t p = 0; p < n_pods; ++p) {
    uint64_t ac = 0, am = 0; /* app sums (memory kept as bits) */
    for (int64_t c = pod_ptr[p]; c < pod_ptr[p + 1]; ++c) {
      ac += cpu_req[c];
      am += (uint64_t)mem_req[c];
    }
    /* sidecar sums; init max, starting at the identity of max (no init container:
     * req = app, as k8s' maxResourceList over an empty list) */
    uint64_t sc = 0, sm = 0, ic = 0;
    int64_t im = INT64_MIN;
    if (init_ptr) {
      for (int64_t k = init_ptr[p]; k < init_ptr[p + 1]; ++k) {
        if (restartable && restartable[k]) {
          ac += init_cpu[k];
          am += (uint64_t)init_mem[k];
          sc += init_cpu[k];
          sm += (uint64_t)init_mem[k];
          if (sc > ic) ic = sc;
          if ((int64_t)sm > im) im = (int64_t)sm;
        } else {
          const uint64_t tc = init_cpu[k] + sc;
          const int64_t tm = (int64_t)((uint64_t)init_mem[k] + sm);
          if (tc > ic) ic = tc;
          if (tm > im) im = tm;
        }
      }
    }
    uint64_t rc = ac > ic ? ac : ic;
    uint64_t rm = (int64_t)am > im ? am : (uint64_t)im;
    if (ovh_cpu) rc += ovh_cpu[p];
    if (ovh_mem) rm += (uint64_t)ovh_mem[p];
    pod_cpu[p] = rc;
    pod_mem[p] = (int64_t)rm;
  }
}

/* CC:159-164 */
int64_t kcco_find_min(int64_t x, int64_t y) { return x <= y ? x : y; }

/* Go int64 division (truncating; MinInt64/-1 wraps).  Caller guarantees y != 0. */
static int64_t go_div_i64(int64_t x, int64_t y) {
  if (y == -1) return (int64_t)(0u - (uint64_t)x);
  return x / y;
}

/* CC:119-136 */
int64_t kcco_fit_one(uint64_t alloc_cpu, int64_t alloc_mem, int64_t alloc_pods,
                     int64_t pod_count, uint64_t used_cpu, int64_t used_mem,
                     uint64_t spec_cpu, int64_t spec_mem, int* div0) {
  int64_t possibleMaxCPUReplicas, possibleMaxMemoryReplicas;
  if (alloc_cpu <= used_cpu) { /* CC:119 */
    possibleMaxCPUReplicas = 0;
  } else {
    if (spec_cpu == 0) { *div0 = 1; return 0; } /* Go: runtime panic */
    possibleMaxCPUReplicas = (int64_t)((alloc_cpu - used_cpu) / spec_cpu); /* CC:123 */
  }
  if (alloc_mem <= used_mem) { /* CC:125 */
    possibleMaxMemoryReplicas = 0;
  } else {
    if (spec_mem == 0) { *div0 = 1; return 0; }
    int64_t freeMem = (int64_t)((uint64_t)alloc_mem - (uint64_t)used_mem); /* wraps */
    possibleMaxMemoryReplicas = go_div_i64(freeMem, spec_mem); /* CC:129 */
  }
  int64_t maxReplicas = kcco_find_min(possibleMaxCPUReplicas, possibleMaxMemoryReplicas); /* CC:133 */
  if (maxReplicas >= alloc_pods) {                                                 /* CC:134 */
    maxReplicas = (int64_t)((uint64_t)alloc_pods - (uint64_t)pod_count);           /* CC:135 */
  }
  return maxReplicas;
}

typedef struct {
  int64_t n_nodes;
  const uint64_t* alloc_cpu;
  const int64_t* alloc_mem;
  const int64_t* alloc_pods;
  const int64_t* pod_count;
  const uint64_t* used_cpu;
  const int64_t* used_mem;
  const uint64_t* spec_cpu;
  const int64_t* spec_mem;
  int64_t* totals;
  int32_t* spec_err;
  int64_t s_begin, s_end;
} fit_job;

static void* fit_worker(void* arg) {
  fit_job* j = (fit_job*)arg;
  for (int64_t s = j->s_begin; s < j->s_end; ++s) {
    uint64_t total = 0; /* totalPossibleMaxReplicas, CC:101 (Go int, wraps) */
    int div0 = 0;
    for (int64_t i = 0; i < j->n_nodes && !div0; ++i) { /* CC:105 */
      int64_t q = kcco_fit_one(j->alloc_cpu[i], j->alloc_mem[i], j->alloc_pods[i],
                               j->pod_count[i], j->used_cpu[i], j->used_mem[i],
                               j->spec_cpu[s], j->spec_mem[s], &div0);
      total += (uint64_t)q; /* CC:138 */
    }
    j->totals[s] = div0 ? 0 : (int64_t)total;
    j->spec_err[s] = div0;
  }
  return NULL;
}

void kcco_fit(int64_t n_nodes, const uint64_t* alloc_cpu, const int64_t* alloc_mem,
              const int64_t* alloc_pods, const int64_t* pod_count,
              const uint64_t* used_cpu, const int64_t* used_mem, int64_t n_specs,
              const uint64_t* spec_cpu, const int64_t* spec_mem, int64_t* totals,
              int32_t* spec_err, int n_threads) {
  if (n_threads < 1) n_threads = 1;
  if (n_threads > 256) n_threads = 256;
  if (n_threads > n_specs) n_threads = n_specs > 0 ? (int)n_specs : 1;
  fit_job jobs[256];
  pthread_t tids[256];
  for (int t = 0; t < n_threads; ++t) {
    fit_job* j = &jobs[t];
    j->n_nodes = n_nodes;
    j->alloc_cpu = alloc_cpu; j->alloc_mem = alloc_mem;
    j->alloc_pods = alloc_pods; j->pod_count = pod_count;
    j->used_cpu = used_cpu; j->used_mem = used_mem;
    j->spec_cpu = spec_cpu; j->spec_mem = spec_mem;
    j->totals = totals; j->spec_err = spec_err;
    j->s_begin = n_specs * t / n_threads;
    j->s_end = n_specs * (t + 1) / n_threads;
  }
  if (n_threads == 1) { fit_worker(&jobs[0]); return; }
  for (int t = 0; t < n_threads; ++t) pthread_create(&tids[t], NULL, fit_worker, &jobs[t]);
  for (int t = 0; t < n_threads; ++t) pthread_join(tids[t], NULL);
}

/* Go strconv.Atoi (== ParseInt(s, 10, 0) on 64-bit): optional sign, >= 1 decimal
 * digit, nothing else, value within int64. */
static int go_atoi(const char* s, size_t n, int64_t* out) {
  size_t i = 0;
  int neg = 0;
  if (n == 0) return 0;
  if (s[0] == '+' || s[0] == '-') { neg = s[0] == '-'; i = 1; }
  if (i == n) return 0;
  uint64_t v = 0;
  const uint64_t lim = neg ? (uint64_t)1 << 63 : ((uint64_t)1 << 63) - 1;
  for (; i < n; ++i) {
    if (s[i] < '0' || s[i] > '9') return 0;
    uint64_t d = (uint64_t)(s[i] - '0');
    if (v > (lim - d) / 10) return 0; /* ErrRange */
    v = v * 10 + d;
  }
  *out = neg ? (int64_t)(0u - v) : (int64_t)v;
  return 1;
}

/* CC:301-319 */
static uint64_t cpu_to_milis_n(const char* cpu, size_t n, int* ok) {
  int flag = 1;
  if (n > 0 && cpu[n - 1] == 'm') { /* strings.HasSuffix / TrimSuffix (one 'm') */
    n -= 1;
    flag = 0;
  }
  int64_t cpuMili = 0;
  if (go_atoi(cpu, n, &cpuMili)) {
    if (flag) cpuMili = (int64_t)((uint64_t)cpuMili * 1000u); /* Go int multiply wraps */
    if (ok) *ok = 1;
  } else {
    cpuMili = 0;
    if (ok) *ok = 0; /* CC:315-316 prints an error */
  }
  return (uint64_t)cpuMili; /* CC:318 */
}

uint64_t kcco_convert_cpu_to_milis(const char* cpu, int* ok) {
  return cpu_to_milis_n(cpu, strlen(cpu), ok);
}

/* Go unicode.IsLetter restricted to the bytes a Quantity/flag string can carry:
 * ASCII letters, plus any non-ASCII byte treated as part of a letter rune start
 * (multi-byte runes are not produced by Quantity.String()). */
static int is_letter_byte(unsigned char c) { return isalpha(c) || c >= 0x80; }

/* Go strconv.ParseFloat(s, 64) restricted to inputs containing no letters
 * (ToBytes splits at the first letter, BF:79-86): [sign] digits [. digits] with at
 * least one digit.  Returns 0 on syntax/range error. */
static int go_parse_float_noletters(const char* s, size_t n, double* out) {
  size_t i = 0, digits = 0;
  char buf[512];
  if (n == 0) return 0;
  if (s[0] == '+' || s[0] == '-') i = 1;
  int seen_dot = 0;
  for (; i < n; ++i) {
    if (s[i] >= '0' && s[i] <= '9') { ++digits; continue; }
    if (s[i] == '.' && !seen_dot) { seen_dot = 1; continue; }
    return 0;
  }
  if (digits == 0) return 0;
  char* tmp = n < sizeof(buf) ? buf : (char*)malloc(n + 1);
  memcpy(tmp, s, n);
  tmp[n] = 0;
  errno = 0;
  double v = strtod(tmp, NULL); /* glibc strtod is correctly rounded, like Go */
  if (tmp != buf) free(tmp);
  if (isinf(v)) return 0; /* ErrRange on overflow */
  *out = v;
  return 1;
}

/* amd64 CVTTSD2SQ: out-of-range / NaN gives 0x8000000000000000 (Go's float->int64
 * conversion of an out-of-range value on amd64). */
static int64_t go_f64_to_i64_amd64(double v) {
  if (isnan(v) || v >= 9223372036854775808.0 || v < -9223372036854775808.0)
    return INT64_MIN;
  return (int64_t)v;
}

/* BF:75-105 */
static int to_bytes_n(const char* s_in, size_t n, int64_t* out) {
  /* strings.TrimSpace + strings.ToUpper (ASCII subset) */
  size_t b = 0, e = n;
  while (b < e && isspace((unsigned char)s_in[b])) ++b;
  while (e > b && isspace((unsigned char)s_in[e - 1])) --e;
  size_t len = e - b;
  char* s = (char*)malloc(len + 1);
  for (size_t k = 0; k < len; ++k) s[k] = (char)toupper((unsigned char)s_in[b + k]);
  s[len] = 0;
  *out = 0;
  size_t i = 0;
  while (i < len && !is_letter_byte((unsigned char)s[i])) ++i; /* IndexFunc(IsLetter) */
  if (i == len) { free(s); return -1; }                         /* BF:81-83 */
  double bytes = 0;
  if (!go_parse_float_noletters(s, i, &bytes) || bytes <= 0) { free(s); return -1; } /* BF:86-89 */
  const char* m = s + i;
  if (strlen(m) != len - i) { free(s); return -1; } /* an embedded NUL is no multiple */
  double mult;
  if (!strcmp(m, "T") || !strcmp(m, "TB") || !strcmp(m, "TIB")) mult = 1099511627776.0;
  else if (!strcmp(m, "G") || !strcmp(m, "GB") || !strcmp(m, "GIB")) mult = 1073741824.0;
  else if (!strcmp(m, "M") || !strcmp(m, "MB") || !strcmp(m, "MIB") || !strcmp(m, "MI")) mult = 1048576.0;
  else if (!strcmp(m, "K") || !strcmp(m, "KB") || !strcmp(m, "KIB") || !strcmp(m, "KI")) mult = 1024.0;
  else if (!strcmp(m, "B")) mult = 1.0;
  else { free(s); return -1; } /* BF:102-103 */
  free(s);
  *out = go_f64_to_i64_amd64(bytes * mult);
  return 0;
}

int kcco_to_bytes(const char* s_in, int64_t* out) { return to_bytes_n(s_in, strlen(s_in), out); }

/* Batch forms over Arrow-style packed strings (string i = bytes[offsets[i],
 * offsets[i+1])): the checker of kcc_parse_* and the CPU baseline of its bench leg.
 * status[i] = 1 ok, 0 error (the reference prints and uses 0). */
typedef struct {
  int mode;
  const char* bytes;
  const int64_t* off;
  int64_t* out;
  int8_t* st;
  int64_t b, e;
} parse_job;

static void* parse_worker(void* arg) {
  parse_job* j = (parse_job*)arg;
  for (int64_t i = j->b; i < j->e; ++i) {
    const char* s = j->bytes + j->off[i];
    const size_t n = (size_t)(j->off[i + 1] - j->off[i]);
    if (j->mode == 0) {
      int ok = 0;
      j->out[i] = (int64_t)cpu_to_milis_n(s, n, &ok);
      j->st[i] = (int8_t)ok;
    } else {
      int64_t v = 0;
      j->st[i] = (int8_t)(to_bytes_n(s, n, &v) == 0);
      j->out[i] = v;
    }
  }
  return NULL;
}

static void parse_batch(int mode, int64_t n, const char* bytes, const int64_t* off, int64_t* out,
                        int8_t* st, int n_threads) {
  parse_job jobs[256];
  pthread_t tids[256];
  if (n_threads < 1) n_threads = 1;
  if (n_threads > 256) n_threads = 256;
  for (int t = 0; t < n_threads; ++t) {
    parse_job* j = &jobs[t];
    j->mode = mode; j->bytes = bytes; j->off = off; j->out = out; j->st = st;
    j->b = n * t / n_threads;
    j->e = n * (t + 1) / n_threads;
  }
  if (n_threads == 1) { parse_worker(&jobs[0]); return; }
  for (int t = 0; t < n_threads; ++t) pthread_create(&tids[t], NULL, parse_worker, &jobs[t]);
  for (int t = 0; t < n_threads; ++t) pthread_join(tids[t], NULL);
}

void kcco_parse_cpu_millis(int64_t n, const char* bytes, const int64_t* offsets, uint64_t* out,
                           int8_t* status, int n_threads) {
  parse_batch(0, n, bytes, offsets, (int64_t*)out, status, n_threads);
}

void kcco_parse_bytes(int64_t n, const char* bytes, const int64_t* offsets, int64_t* out,
                      int8_t* status, int n_threads) {
  parse_batch(1, n, bytes, offsets, out, status, n_threads);
}
