/*
 * ec_oracle.c — scalar C restatement of ec-cpp (the parity oracle).
 *
 * TEST INFRASTRUCTURE ONLY (see ec_oracle.h).  Written for clarity, not speed:
 * it is the checker the HIP path is compared against, and the "port" CPU
 * baseline.  All references are to /root/reference (snapshot 2025-07-04).
 */
#include "ec_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define FIELD_SIZE 65536u
#define ONE_MASK 65535u

static uint16_t g_log[FIELD_SIZE];
static uint16_t g_exp[FIELD_SIZE];
static uint16_t g_log_walsh[FIELD_SIZE];
static uint16_t g_skew[ONE_MASK];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

/* f2e16.hpp:36-38 — the Cantor-style basis used to relabel field elements */
static const uint16_t k_base[16] = {1,     44234, 15374, 5694,  50562, 60718,
                                    37196, 16402, 27800, 4312,  27250, 47360,
                                    64952, 64308, 65336, 39198};

/* walsh.hpp:15-39: in-place Walsh-Hadamard transform over Z/65535 using
 * ones'-complement folding (fold(t) = (t & 0xffff) + (t >> 16)). */
void eco_walsh(uint16_t *d, size_t size) {
  for (size_t half = 1; half < size; half <<= 1) {
    for (size_t blk = 0; blk < size; blk += half << 1) {
      for (size_t i = blk; i < blk + half; ++i) {
        uint32_t x = d[i], y = d[i + half];
        uint32_t s = x + y;
        uint32_t t = x + ONE_MASK - y;
        d[i] = (uint16_t)((s & 0xffffu) + (s >> 16));
        d[i + half] = (uint16_t)((t & 0xffffu) + (t >> 16));
      }
    }
  }
}

/* f2e16.hpp:48-84 */
static void build_field(void) {
  /* LFSR powers of the generator (poly x^16 + x^5 + x^3 + x^2 + 1, 0x2D):
   * g_exp temporarily maps polynomial-basis element -> discrete log. */
  uint32_t state = 1;
  for (uint32_t e = 0; e < ONE_MASK; ++e) {
    g_exp[state] = (uint16_t)e;
    state <<= 1;
    if (state & 0x10000u) state = (state & 0xffffu) ^ 0x2Du;
  }
  g_exp[0] = (uint16_t)ONE_MASK;

  /* linear relabelling by k_base, then compose with the discrete log */
  g_log[0] = 0;
  for (uint32_t b = 0; b < 16; ++b)
    for (uint32_t j = 0; j < (1u << b); ++j)
      g_log[j + (1u << b)] = g_log[j] ^ k_base[b];
  for (uint32_t x = 0; x < FIELD_SIZE; ++x) g_log[x] = g_exp[g_log[x]];
  for (uint32_t x = 0; x < FIELD_SIZE; ++x) g_exp[g_log[x]] = (uint16_t)x;
  g_exp[ONE_MASK] = g_exp[0];

  memcpy(g_log_walsh, g_log, sizeof g_log);
  g_log_walsh[0] = 0;
  eco_walsh(g_log_walsh, FIELD_SIZE);
}

/* additive_fft.hpp:21-33 — x * g^log_c; log_c is a residue mod 65535 */
uint16_t eco_mul(uint16_t x, uint16_t log_c) {
  if (x == 0) return 0;
  uint32_t l = (uint32_t)g_log[x] + log_c;
  return g_exp[(l & 0xffffu) + (l >> 16)];
}

/* additive_fft.hpp:47-97 — skew factors of the subspace vanishing polys */
static void build_skews(void) {
  static uint16_t add[ONE_MASK]; /* skews in additive (element) form */
  uint16_t base[15];
  memset(add, 0, sizeof add);
  for (uint32_t i = 1; i < 16; ++i) base[i - 1] = (uint16_t)(1u << i);

  for (uint32_t m = 0; m < 15; ++m) {
    uint32_t step = 1u << (m + 1);
    add[(1u << m) - 1] = 0;
    for (uint32_t i = m; i < 15; ++i) {
      uint32_t s = 1u << (i + 1);
      for (uint32_t j = (1u << m) - 1; j < s; j += step)
        add[j + s] = add[j] ^ base[i];
    }
    /* normalise level m: base[m] <- 1/(base[m]*(base[m]^1)) in log form */
    uint16_t v = eco_mul(base[m], g_log[base[m] ^ 1]);
    base[m] = (uint16_t)(ONE_MASK - g_log[v]);
    for (uint32_t i = m + 1; i < 15; ++i) {
      uint32_t b = ((uint32_t)g_log[base[i] ^ 1] + base[m]) % ONE_MASK;
      base[i] = eco_mul(base[i], (uint16_t)b);
    }
  }
  for (uint32_t i = 0; i < ONE_MASK; ++i) g_skew[i] = g_log[add[i]];
}

static void init_once(void) {
  build_field();
  build_skews();
}
static void ensure_init(void) { pthread_once(&g_once, init_once); }

const uint16_t *eco_log_table(void) { ensure_init(); return g_log; }
const uint16_t *eco_exp_table(void) { ensure_init(); return g_exp; }
const uint16_t *eco_log_walsh_table(void) { ensure_init(); return g_log_walsh; }
const uint16_t *eco_skews(void) { ensure_init(); return g_skew; }

/* additive_fft.hpp:99-119 — inverse transform: stages d = 1, 2, 4, ... */
void eco_inverse_afft(uint16_t *x, size_t size, size_t index) {
  ensure_init();
  for (size_t d = 1; d < size; d <<= 1) {
    for (size_t j = d; j < size; j += d << 1) {
      for (size_t i = j - d; i < j; ++i) x[i + d] ^= x[i];
      uint16_t w = g_skew[j + index - 1];
      if (w != ONE_MASK)
        for (size_t i = j - d; i < j; ++i) x[i] ^= eco_mul(x[i + d], w);
    }
  }
}

/* additive_fft.hpp:121-141 — forward transform: stages d = size/2, ..., 1 */
void eco_afft(uint16_t *x, size_t size, size_t index) {
  ensure_init();
  for (size_t d = size >> 1; d > 0; d >>= 1) {
    for (size_t j = d; j < size; j += d << 1) {
      uint16_t w = g_skew[j + index - 1];
      if (w != ONE_MASK)
        for (size_t i = j - d; i < j; ++i) x[i] ^= eco_mul(x[i + d], w);
      for (size_t i = j - d; i < j; ++i) x[i + d] ^= x[i];
    }
  }
}

/* poly_encoder.hpp:195-215 (the tail loop never runs: cos.size() == size) */
void eco_formal_derivative(uint16_t *c, size_t size) {
  for (size_t i = 1; i < size; ++i) {
    size_t len = ((i ^ (i - 1)) + 1) >> 1;
    for (size_t j = i - len; j < i; ++j) c[j] ^= (j + len < size) ? c[j + len] : 0;
  }
}

/* math.hpp:25-36 */
static size_t next_high_pow2(size_t v) {
  if (v && !(v & (v - 1))) return v;
  size_t p = v == 0 ? 0 : 64 - (size_t)__builtin_clzll(v);
  return (size_t)1 << p;
}
static size_t next_low_pow2(size_t v) {
  size_t p = v <= 1 ? 0 : 64 - (size_t)__builtin_clzll(v >> 1);
  return (size_t)1 << p;
}

/* ec-cpp.cpp:15-24 */
int eco_recovery_threshold(size_t nv, size_t *thr) {
  if (nv > FIELD_SIZE) return ECO_TOO_MANY_VALIDATORS;
  if (nv <= 1) return ECO_NOT_ENOUGH_VALIDATORS;
  *thr = (nv - 1) / 3 + 1;
  return ECO_OK;
}

/* ec-cpp.cpp:26-37 + reed-solomon.hpp:24-45 */
int eco_params(size_t nv, size_t *n, size_t *k) {
  size_t thr;
  int e = eco_recovery_threshold(nv, &thr);
  if (e) return e;
  if (nv < 2) return ECO_WANTED_SHARD_COUNT_TOO_LOW;
  size_t kk = next_low_pow2(thr), nn = next_high_pow2(nv);
  if (nn > FIELD_SIZE) return ECO_WANTED_SHARD_COUNT_TOO_HIGH;
  *n = nn;
  *k = kk;
  return ECO_OK;
}

size_t eco_shard_len(size_t k, size_t len) {
  size_t syms = (len + 1) / 2;
  return (syms + k - 1) / k * 2;
}

/* reed-solomon.hpp:47-81 with poly_encoder.hpp:31-86,217-240 */
int eco_encode(size_t nv, const uint8_t *p, size_t len, uint8_t *shards,
               size_t cap) {
  size_t n, k;
  int e = eco_params(nv, &n, &k);
  if (e) return e;
  if (len == 0) return ECO_PAYLOAD_SIZE_IS_ZERO;
  size_t sl = eco_shard_len(k, len);
  if (cap < nv * sl) return ECO_WANTED_SHARD_COUNT_TOO_HIGH;
  ensure_init();
  uint16_t *cw = (uint16_t *)malloc(n * sizeof *cw);
  for (size_t off = 0, piece = 0; off < len; off += 2 * k, ++piece) {
    size_t end = off + 2 * k < len ? off + 2 * k : len;
    memset(cw, 0, n * sizeof *cw);
    for (size_t b = off, s = 0; b < end; b += 2, ++s) {
      uint16_t hi = p[b], lo = b + 1 < end ? p[b + 1] : 0; /* BE; odd tail */
      cw[s] = (uint16_t)(hi << 8 | lo);
    }
    /* encodeLow: coefficients, then one shifted forward transform per coset */
    eco_inverse_afft(cw, k, 0);
    for (size_t sh = k; sh < n; sh += k) {
      memcpy(cw + sh, cw, k * sizeof *cw);
      eco_afft(cw + sh, k, sh);
    }
    /* systematic prefix restored from the data itself */
    for (size_t b = off, s = 0; s < k; b += 2, ++s) {
      uint16_t hi = b < end ? p[b] : 0, lo = b + 1 < end ? p[b + 1] : 0;
      cw[s] = (uint16_t)(hi << 8 | lo);
    }
    for (size_t v = 0; v < nv; ++v) {
      shards[v * sl + 2 * piece] = (uint8_t)(cw[v] >> 8);
      shards[v * sl + 2 * piece + 1] = (uint8_t)cw[v];
    }
  }
  free(cw);
  return ECO_OK;
}

/* poly_encoder.hpp:90-116; the reference calls it with n = kFieldSize
 * (reed-solomon.hpp:109-110), so z = min(65536, received + gap) = code length */
void eco_error_poly(const uint8_t *erased, size_t nr, size_t n, uint16_t *out) {
  ensure_init();
  memset(out, 0, FIELD_SIZE * sizeof *out);
  for (size_t i = 0; i < n; ++i) out[i] = (i >= nr || erased[i]) ? 1 : 0;
  eco_walsh(out, FIELD_SIZE);
  for (size_t i = 0; i < FIELD_SIZE; ++i)
    out[i] = (uint16_t)(((uint32_t)out[i] * g_log_walsh[i]) % ONE_MASK);
  eco_walsh(out, FIELD_SIZE);
  for (size_t i = 0; i < n; ++i)
    if (i >= nr || erased[i]) out[i] = (uint16_t)(ONE_MASK - out[i]);
}

/* Same residues (mod 65535) for i < n in O(n log n): the input is supported on
 * [0, n), so the 65536-point WHT only depends on the low log2(n) bits; fold
 * LOG_WALSH over the high bits.  Not in the reference — checked against
 * eco_error_poly in tests/test_oracle.py. */
void eco_error_poly_folded(const uint8_t *erased, size_t nr, size_t n,
                           uint16_t *out) {
  ensure_init();
  uint16_t *w = (uint16_t *)calloc(n, sizeof *w);
  for (size_t i = 0; i < n; ++i) w[i] = (i >= nr || erased[i]) ? 1 : 0;
  eco_walsh(w, n);
  for (size_t lo = 0; lo < n; ++lo) {
    uint64_t f = 0;
    for (size_t hi = 0; hi < FIELD_SIZE / n; ++hi) f += g_log_walsh[hi * n + lo];
    w[lo] = (uint16_t)(((uint64_t)w[lo] * (f % ONE_MASK)) % ONE_MASK);
  }
  eco_walsh(w, n);
  for (size_t i = 0; i < n; ++i) {
    uint16_t v = w[i] % ONE_MASK;
    out[i] = (i >= nr || erased[i]) ? (uint16_t)((ONE_MASK - v) % ONE_MASK) : v;
  }
  free(w);
}

/* reed-solomon.hpp:83-134 with poly_encoder.hpp:118-189 */
int eco_reconstruct(size_t nv, const uint8_t *const *sh, const size_t *lens,
                    size_t nr, uint8_t *out, size_t cap, size_t *out_len) {
  size_t n, k;
  int e = eco_params(nv, &n, &k);
  if (e) return e;
  if (nr > n) nr = n; /* the reference asserts received + gap == n */
  size_t present = 0, syms = 0;
  for (size_t i = 0; i < nr; ++i) {
    if (!sh[i] || lens[i] == 0) continue;
    if (present == 0) syms = lens[i] / 2;
    else if (syms != lens[i] / 2) return ECO_INCONSISTENT_SHARD_LENGTHS;
    ++present;
  }
  if (present < k) return ECO_NEED_MORE_SHARDS;
  if (cap < syms * 2 * k) return ECO_NEED_MORE_SHARDS;
  ensure_init();

  uint8_t *erased = (uint8_t *)calloc(n, 1);
  for (size_t i = 0; i < n; ++i) erased[i] = (i >= nr || !sh[i] || lens[i] == 0);
  uint16_t *ep = (uint16_t *)malloc(FIELD_SIZE * sizeof *ep);
  eco_error_poly(erased, n, n, ep);

  uint16_t *cw = (uint16_t *)malloc(n * sizeof *cw);
  for (size_t pos = 0; pos < syms; ++pos) {
    for (size_t i = 0; i < n; ++i)
      cw[i] = erased[i] ? 0
                        : eco_mul((uint16_t)(sh[i][2 * pos] << 8 | sh[i][2 * pos + 1]), ep[i]);
    eco_inverse_afft(cw, n, 0);
    eco_formal_derivative(cw, n);
    eco_afft(cw, n, 0);
    for (size_t y = 0; y < k; ++y) {
      uint16_t s = erased[y] ? eco_mul(cw[y], ep[y])
                             : (uint16_t)(sh[y][2 * pos] << 8 | sh[y][2 * pos + 1]);
      out[2 * (pos * k + y)] = (uint8_t)(s >> 8);
      out[2 * (pos * k + y) + 1] = (uint8_t)s;
    }
  }
  *out_len = syms * 2 * k;
  free(cw);
  free(ep);
  free(erased);
  return ECO_OK;
}

/* reed-solomon.hpp:143-179 */
int eco_reconstruct_from_systematic(size_t nv, const uint8_t *const *ch,
                                    const size_t *lens, size_t count,
                                    uint8_t *out, size_t cap, size_t *out_len) {
  size_t n, k;
  int e = eco_params(nv, &n, &k);
  if (e) return e;
  if (count == 0 || count < k) return ECO_NEED_MORE_SHARDS;
  size_t syms = lens[0] / 2;
  if (syms == 0) return ECO_EMPTY_SHARD;
  for (size_t c = 0; c < count; ++c)
    if (lens[c] / 2 != syms) return ECO_INCONSISTENT_SHARD_LENGTHS;
  if (cap < syms * 2 * k) return ECO_NEED_MORE_SHARDS;
  for (size_t i = 0; i < syms; ++i)
    for (size_t y = 0; y < k; ++y) {
      out[2 * (i * k + y)] = ch[y][2 * i];
      out[2 * (i * k + y) + 1] = ch[y][2 * i + 1];
    }
  *out_len = syms * 2 * k;
  return ECO_OK;
}
