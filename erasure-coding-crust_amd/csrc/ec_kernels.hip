// ec_kernels.hip — HIP kernels for gfx950: NPB Reed-Solomon encode, erasure
// locator, reconstruct, systematic reconstruct.
//
// Generic path ("g" kernels): one workgroup owns G byte-planar groups (4 pieces
// or 4 shard positions each) and runs the additive FFT stage by stage on a
// [position][group] uint2 array in LDS (or global scratch for FFTs above
// 4096 points).  Butterflies follow additive_fft.hpp:99-141 exactly; the
// multiply is the v_perm lookup of ec_device.hpp.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "ec_device.hpp"
#include "ec_kernels.hpp"

namespace ecamd {
namespace {

constexpr int kBlock = 256;
constexpr int kLdsSlots = 4096;  // uint2 slots per buffer in LDS (32 KiB)

__device__ __forceinline__ void ld(uint2 *p, uint32_t &l, uint32_t &h) {
  const uint2 v = *p;
  l = v.x;
  h = v.y;
}

// inverse_afft (additive_fft.hpp:99-119) on S[pos * G + g], pos < 2^logsz.
// Small transforms (<= 3 stages, at most one butterfly per thread and stage:
// the per-call sizes of tiny codes, e.g. n_validators 6) request every
// stage's table up front, so the stages wait on one table latency instead of
// one each (the per-call C ABI's kernel time).
constexpr int kPreStages = 3;
__device__ void ifft_g(uint2 *S, int logG, int logsz, uint32_t index, const DevTables t) {
  const int G = 1 << logG;
  const int half = (1 << logsz) >> 1;
  if (logsz <= kPreStages && half * G <= int(blockDim.x)) {
    const int b = threadIdx.x, g = b & (G - 1), pi = b >> logG;
    const bool on = b < half * G;
    Tab T[kPreStages];
#pragma unroll
    for (int m = 0; m < kPreStages; ++m) {
      const int d = 1 << m, i = ((pi >> m) << (m + 1)) | (pi & (d - 1)), j = (i & ~(2 * d - 1)) | d;
      if (on && m < logsz) load_tab(t.mslot, j - 1 + index, T[m]);
    }
#pragma unroll
    for (int m = 0; m < kPreStages; ++m) {
      if (m >= logsz) break;
      const int d = 1 << m, i = ((pi >> m) << (m + 1)) | (pi & (d - 1));
      if (on) {
        uint32_t al, ah, bl, bh;
        ld(S + i * G + g, al, ah);
        ld(S + (i + d) * G + g, bl, bh);
        bl ^= al;
        bh ^= ah;
        mul_acc(bl, bh, T[m], al, ah);
        S[i * G + g] = make_uint2(al, ah);
        S[(i + d) * G + g] = make_uint2(bl, bh);
      }
      __syncthreads();
    }
    return;
  }
  for (int m = 0; m < logsz; ++m) {
    const int d = 1 << m;
    for (int b = threadIdx.x; b < half * G; b += blockDim.x) {
      const int g = b & (G - 1), pi = b >> logG;
      const int i = ((pi >> m) << (m + 1)) | (pi & (d - 1));
      const int j = (i & ~(2 * d - 1)) | d;
      Tab T;
      load_tab(t.mslot, j - 1 + index, T);  // (mtab[skews[..]]: no dependent load)
      uint32_t al, ah, bl, bh;
      ld(S + i * G + g, al, ah);
      ld(S + (i + d) * G + g, bl, bh);
      bl ^= al;
      bh ^= ah;
      mul_acc(bl, bh, T, al, ah);
      S[i * G + g] = make_uint2(al, ah);
      S[(i + d) * G + g] = make_uint2(bl, bh);
    }
    __syncthreads();
  }
}

// afft (additive_fft.hpp:121-141); small transforms as in ifft_g
__device__ void fft_g(uint2 *S, int logG, int logsz, uint32_t index, const DevTables t) {
  const int G = 1 << logG;
  const int half = (1 << logsz) >> 1;
  if (logsz <= kPreStages && half * G <= int(blockDim.x)) {
    const int b = threadIdx.x, g = b & (G - 1), pi = b >> logG;
    const bool on = b < half * G;
    Tab T[kPreStages];
#pragma unroll
    for (int m = 0; m < kPreStages; ++m) {
      const int d = 1 << m, i = ((pi >> m) << (m + 1)) | (pi & (d - 1)), j = (i & ~(2 * d - 1)) | d;
      if (on && m < logsz) load_tab(t.mslot, j - 1 + index, T[m]);
    }
#pragma unroll
    for (int m = kPreStages - 1; m >= 0; --m) {
      if (m >= logsz) continue;
      const int d = 1 << m, i = ((pi >> m) << (m + 1)) | (pi & (d - 1));
      if (on) {
        uint32_t al, ah, bl, bh;
        ld(S + i * G + g, al, ah);
        ld(S + (i + d) * G + g, bl, bh);
        mul_acc(bl, bh, T[m], al, ah);
        bl ^= al;
        bh ^= ah;
        S[i * G + g] = make_uint2(al, ah);
        S[(i + d) * G + g] = make_uint2(bl, bh);
      }
      __syncthreads();
    }
    return;
  }
  for (int m = logsz - 1; m >= 0; --m) {
    const int d = 1 << m;
    for (int b = threadIdx.x; b < half * G; b += blockDim.x) {
      const int g = b & (G - 1), pi = b >> logG;
      const int i = ((pi >> m) << (m + 1)) | (pi & (d - 1));
      const int j = (i & ~(2 * d - 1)) | d;
      Tab T;
      load_tab(t.mslot, j - 1 + index, T);
      uint32_t al, ah, bl, bh;
      ld(S + i * G + g, al, ah);
      ld(S + (i + d) * G + g, bl, bh);
      mul_acc(bl, bh, T, al, ah);
      bl ^= al;
      bh ^= ah;
      S[i * G + g] = make_uint2(al, ah);
      S[(i + d) * G + g] = make_uint2(bl, bh);
    }
    __syncthreads();
  }
}

// the fused completion signal (HostSig): every thread's output is made
// visible at system scope, then one lane stores v
__device__ __forceinline__ void signal_end(uint32_t *flag, uint32_t v) {
  if (!flag) return;
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// reed-solomon.hpp:47-81 + poly_encoder.hpp:31-86,217-240 for 4*G pieces
__global__ void __launch_bounds__(kBlock) encode_g(const uint8_t *__restrict__ payloads,
                                                   uint64_t plen, uint64_t pstride,
                                                   uint8_t *__restrict__ shards, uint64_t slen,
                                                   uint64_t sstride, int nv, int logn, int logk,
                                                   int logG, uint32_t batch, DevTables t,
                                                   uint2 *scratch, uint32_t *sig_flag, uint32_t sig_v) {
  extern __shared__ __attribute__((aligned(16))) uint2 smem[];
  const int k = 1 << logk, n = 1 << logn, G = 1 << logG;
  const uint64_t npieces = slen / 2;
  const uint64_t piece0 = uint64_t(blockIdx.x) * 4 * G;
  uint2 *S = smem, *Cf = smem + size_t(k) * G;
  if (scratch) {  // one buffer per block, reused by its payloads in turn
    S = scratch + (uint64_t(blockIdx.y) * gridDim.x + blockIdx.x) * 2 * uint64_t(k) * G;
    Cf = S + size_t(k) * G;
  }
  for (uint32_t b = blockIdx.y; b < batch; b += gridDim.y) {  // batch may exceed gridDim.y's limit
  const uint8_t *P = payloads + uint64_t(b) * pstride;
  uint8_t *SH = shards + uint64_t(b) * nv * sstride;
  // BE-unpack 4 pieces per group, zero-padded (poly_encoder.hpp:53-76); the
  // systematic shards are the data symbols themselves (poly_encoder.hpp:239)
  for (int e = threadIdx.x; e < k * G; e += blockDim.x) {
    const int g = e & (G - 1), i = e >> logG;
    uint32_t xl = 0, xh = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint64_t p = piece0 + 4 * g + q;
      const uint64_t off = p * 2 * uint64_t(k) + 2 * uint64_t(i);
      const uint32_t hi = off < plen ? P[off] : 0;
      const uint32_t lo = off + 1 < plen ? P[off + 1] : 0;
      xl |= lo << (8 * q);
      xh |= hi << (8 * q);
      if (p < npieces) {
        SH[uint64_t(i) * sstride + 2 * p] = uint8_t(hi);
        SH[uint64_t(i) * sstride + 2 * p + 1] = uint8_t(lo);
      }
    }
    S[e] = make_uint2(xl, xh);
  }
  __syncthreads();
  ifft_g(S, logG, logk, 0, t);
  for (int e = threadIdx.x; e < k * G; e += blockDim.x) Cf[e] = S[e];
  __syncthreads();
  for (int s = k; s < n && s < nv; s += k) {
    if (s > k) {
      for (int e = threadIdx.x; e < k * G; e += blockDim.x) S[e] = Cf[e];
      __syncthreads();
    }
    fft_g(S, logG, logk, uint32_t(s), t);
    for (int e = threadIdx.x; e < k * G; e += blockDim.x) {
      const int g = e & (G - 1), v = s + (e >> logG);
      if (v >= nv) continue;
      const uint2 x = S[e];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint64_t p = piece0 + 4 * g + q;
        if (p < npieces) {
          SH[uint64_t(v) * sstride + 2 * p] = uint8_t(x.y >> (8 * q));
          SH[uint64_t(v) * sstride + 2 * p + 1] = uint8_t(x.x >> (8 * q));
        }
      }
    }
    __syncthreads();
  }
  }
  signal_end(sig_flag, sig_v);  // (single-workgroup launches only)
}

// poly_encoder.hpp:90-116 in the folded n-point form: one
// workgroup per erasure pattern.  W lives in LDS (n <= 65536 -> 128 KiB) or
// in global scratch.
__global__ void __launch_bounds__(kBlock) error_locator_g(const uint8_t *__restrict__ present,
                                                          int nv, int logn,
                                                          const uint16_t *__restrict__ fold,
                                                          const uint32_t *__restrict__ pattern,
                                                          uint16_t *__restrict__ elog,
                                                          uint16_t *scratch) {
  extern __shared__ __attribute__((aligned(16))) uint16_t w16[];
  const int n = 1 << logn;
  if (pattern && pattern[blockIdx.x] != blockIdx.x) return;  // computed by its pattern's leader
  const uint8_t *pr = present + uint64_t(blockIdx.x) * n;
  uint16_t *W = scratch ? scratch + uint64_t(blockIdx.x) * n : w16;
  for (int i = threadIdx.x; i < n; i += blockDim.x) W[i] = (i < nv && pr[i]) ? 0 : 1;
  __syncthreads();
  for (int pass = 0; pass < 2; ++pass) {
    for (int h = 1; h < n; h <<= 1) {  // walsh.hpp:15-39
      for (int b = threadIdx.x; b < n / 2; b += blockDim.x) {
        const int i = (b / h) * 2 * h + (b % h);
        const uint32_t x = W[i], y = W[i + h];
        const uint32_t s = x + y, u = x + 65535u - y;
        W[i] = uint16_t((s & 0xffff) + (s >> 16));
        W[i + h] = uint16_t((u & 0xffff) + (u >> 16));
      }
      __syncthreads();
    }
    if (pass == 0) {
      for (int i = threadIdx.x; i < n; i += blockDim.x)
        W[i] = uint16_t((uint32_t(W[i]) * fold[i]) % 65535u);
      __syncthreads();
    }
  }
  uint16_t *E = elog + uint64_t(blockIdx.x) * n;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const bool erased = !(i < nv && pr[i]);
    E[i] = erased ? uint16_t(65535u - W[i]) : W[i];
  }
}

// The same folded locator with one WAVE per erasure pattern, for 64 <= n <= 4096
// (round 3): V = n / 64 positions per lane (position lane * V + r), the Walsh
// stages over register bits in registers and over the six lane bits by
// __shfl_xor; no LDS, no barrier, four patterns per 256-thread workgroup.  The
// workgroup form above spends ~20 barriers per pattern; at 4096 distinct
// patterns (n = 1024) it took 43 us, this form ~5 us, which also makes the
// pattern dedup (~35 us of hash / insert / resolve / broadcast kernels) cost
// more than it can save for n <= 4096: ECCR_AMD_error_locator computes every
// row directly there.  Results are congruent mod 65535 to the reference's
// (the workgroup form's arithmetic, term for term).
__device__ __forceinline__ uint32_t fold16(uint32_t s) { return (s & 0xffffu) + (s >> 16); }

template <int V>
__device__ __forceinline__ void walsh_wave(uint32_t (&w)[V], uint32_t lane) {
#pragma unroll
  for (int h = 1; h < V; h <<= 1)  // register bits
#pragma unroll
    for (int r = 0; r < V; ++r)
      if (!(r & h)) {
        const uint32_t x = w[r], y = w[r + h];
        w[r] = fold16(x + y);
        w[r + h] = fold16(x + 65535u - y);
      }
#pragma unroll
  for (int m = 0; m < 6; ++m) {  // lane bits: the partner is lane ^ 2^m
    const bool upper = (lane >> m) & 1;
#pragma unroll
    for (int r = 0; r < V; ++r) {
      const uint32_t o = uint32_t(__shfl_xor(int(w[r]), 1 << m));
      w[r] = upper ? fold16(o + 65535u - w[r]) : fold16(w[r] + o);
    }
  }
}

template <int V>
__global__ void __launch_bounds__(256) error_locator_w(const uint8_t *__restrict__ present, int nv,
                                                       uint32_t rows,
                                                       const uint16_t *__restrict__ fold,
                                                       const uint32_t *__restrict__ pattern,
                                                       uint16_t *__restrict__ elog) {
  constexpr uint32_t n = 64 * V;
  const uint32_t b = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (b >= rows) return;                             // whole waves
  if (pattern && pattern[b] != b) return;            // computed by its pattern's leader
  const uint8_t *pr = present + uint64_t(b) * n + lane * V;
  const uint16_t *F = fold + lane * V;
  uint32_t w[V];
  uint64_t erased = 0;
#pragma unroll
  for (int r = 0; r < V; ++r) {
    const bool e = !(int(lane * V + r) < nv && pr[r]);
    erased |= uint64_t(e) << r;
    w[r] = e;
  }
  walsh_wave<V>(w, lane);
#pragma unroll
  for (int r = 0; r < V; ++r) w[r] = fold16(fold16(w[r] * uint32_t(F[r])));  // W * F mod 65535
  walsh_wave<V>(w, lane);
  uint16_t *E = elog + uint64_t(b) * n + lane * V;
#pragma unroll
  for (int r = 0; r < V; ++r) E[r] = uint16_t(((erased >> r) & 1) ? 65535u - w[r] : w[r]);
}

// ---- erasure-pattern dedup: payloads whose erasure
// patterns are equal share one locator.  The locator depends only on the
// flags (present[i] != 0) of positions i < nv, and so do the hash and the
// equality test below.
__device__ __forceinline__ uint64_t mix64(uint64_t x) {  // splitmix64 finaliser
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// block per row: H = sum over present positions i of mix64(i) (order-free, so
// a block-wide sum); never 0 (0 marks an empty hash slot)
__global__ void __launch_bounds__(kBlock) pattern_hash(const uint8_t *__restrict__ present, int nv,
                                                       int n, uint64_t *__restrict__ hash) {
  __shared__ uint64_t part[kBlock / 64];
  const uint8_t *pr = present + uint64_t(blockIdx.x) * n;
  uint64_t h = 0;
  for (int i = threadIdx.x; i < nv; i += kBlock)
    if (pr[i]) h += mix64(uint64_t(i));
  for (int o = 32; o > 0; o >>= 1) h += __shfl_xor(h, o);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = h;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t t = 0;
    for (int w = 0; w < kBlock / 64; ++w) t += part[w];
    hash[blockIdx.x] = t ? t : 1;
  }
}

// thread per row: open-addressing insert, each slot keeps the smallest row
// index with its hash
__global__ void __launch_bounds__(kBlock) pattern_insert(const uint64_t *__restrict__ hash,
                                                         uint32_t batch, unsigned long long *keys,
                                                         uint32_t *vals, uint32_t cap) {
  const uint32_t b = blockIdx.x * kBlock + threadIdx.x;
  if (b >= batch) return;
  const uint64_t h = hash[b];
  for (uint32_t slot = uint32_t(h % cap), probe = 0; probe < cap; ++probe, slot = (slot + 1) % cap) {
    const unsigned long long prev = atomicCAS(&keys[slot], 0ull, (unsigned long long)h);
    if (prev == 0ull || prev == h) {
      atomicMin(&vals[slot], b);
      return;
    }
  }
}

// block per row: pattern[b] = the leader (smallest index) of b's hash if its
// flags are identical to b's, else b itself (a hash collision: b keeps its own)
__global__ void __launch_bounds__(kBlock) pattern_resolve(const uint8_t *__restrict__ present, int nv,
                                                          int n, const uint64_t *__restrict__ hash,
                                                          const unsigned long long *__restrict__ keys,
                                                          const uint32_t *__restrict__ vals,
                                                          uint32_t cap, uint32_t *__restrict__ pattern) {
  __shared__ uint32_t leader;
  __shared__ int differ;
  const uint32_t b = blockIdx.x;
  if (threadIdx.x == 0) {
    const uint64_t h = hash[b];
    uint32_t slot = uint32_t(h % cap);
    for (uint32_t probe = 0; probe < cap && keys[slot] != h; ++probe) slot = (slot + 1) % cap;
    leader = keys[slot] == h ? vals[slot] : b;
    differ = 0;
  }
  __syncthreads();
  const uint32_t l = leader;
  if (l != b) {
    const uint8_t *pb = present + uint64_t(b) * n, *pl = present + uint64_t(l) * n;
    for (int i = threadIdx.x; i < nv; i += kBlock)
      if ((pb[i] != 0) != (pl[i] != 0)) differ = 1;
    __syncthreads();
  }
  if (threadIdx.x == 0) pattern[b] = (l != b && !differ) ? l : b;
}

// block per row: a follower's locator row = its leader's
__global__ void __launch_bounds__(kBlock) pattern_broadcast(const uint32_t *__restrict__ pattern, int n,
                                                            uint16_t *__restrict__ elog) {
  const uint32_t b = blockIdx.x, l = pattern[b];
  if (l == b) return;
  const uint16_t *src = elog + uint64_t(l) * n;
  uint16_t *dst = elog + uint64_t(b) * n;
  for (int i = threadIdx.x; i < n; i += kBlock) dst[i] = src[i];
}

__device__ __forceinline__ uint32_t mul_index(uint32_t log_c) {  // 65535 == 0 (mod 65535)
  return log_c == 65535u ? 0u : log_c;
}

// reed-solomon.hpp:83-134 + poly_encoder.hpp:118-215 for 4*G shard positions
__global__ void __launch_bounds__(kBlock) reconstruct_g(
    const uint8_t *__restrict__ shards, uint64_t slen, uint64_t sstride,
    const uint8_t *__restrict__ present, const uint16_t *__restrict__ elog,
    uint8_t *__restrict__ out, uint64_t ostride, int nv, int logn, int logk, int logG,
    uint32_t batch, const uint32_t *__restrict__ pattern, DevTables t, uint2 *scratch) {
  extern __shared__ __attribute__((aligned(16))) uint2 smem[];
  const int n = 1 << logn, k = 1 << logk, G = 1 << logG;
  const uint64_t npos = slen / 2;
  const uint64_t pos0 = uint64_t(blockIdx.x) * 4 * G;
  uint2 *S = smem, *D = smem + size_t(n) * G;
  if (scratch) {  // one buffer per block, reused by its payloads in turn
    S = scratch + (uint64_t(blockIdx.y) * gridDim.x + blockIdx.x) * 2 * uint64_t(n) * G;
    D = S + size_t(n) * G;
  }
  for (uint32_t b = blockIdx.y; b < batch; b += gridDim.y) {  // batch may exceed gridDim.y's limit
  const uint64_t pt = pattern ? pattern[b] : b;  // erasure pattern of payload b
  const uint8_t *SH = shards + uint64_t(b) * nv * sstride;
  const uint8_t *pr = present + pt * n;
  const uint16_t *E = elog + pt * n;
  uint8_t *O = out + uint64_t(b) * ostride;
  __syncthreads();  // the previous payload's readers of S / D are done
  // gather the column, multiply present symbols by the locator (decode_main:174-177)
  for (int e = threadIdx.x; e < n * G; e += blockDim.x) {
    const int g = e & (G - 1), v = e >> logG;
    uint32_t yl = 0, yh = 0;
    if (v < nv && pr[v]) {
      uint32_t xl = 0, xh = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint64_t pos = pos0 + 4 * g + q;
        if (pos < npos) {
          xh |= uint32_t(SH[uint64_t(v) * sstride + 2 * pos]) << (8 * q);
          xl |= uint32_t(SH[uint64_t(v) * sstride + 2 * pos + 1]) << (8 * q);
        }
      }
      Tab T;
      load_tab(t.mtab, mul_index(E[v]), T);
      mul_acc(xl, xh, T, yl, yh);
    }
    S[e] = make_uint2(yl, yh);
  }
  __syncthreads();
  ifft_g(S, logG, logn, 0, t);
  // formal derivative (poly_encoder.hpp:195-215), closed form:
  //   c'[j] = c[j] ^ XOR_{b : bit b of j is 0} c[j | 2^b]
  for (int e = threadIdx.x; e < n * G; e += blockDim.x) {
    const int g = e & (G - 1), j = e >> logG;
    uint2 acc = S[e];
    for (int b = 0; b < logn; ++b)
      if (!(j & (1 << b))) {
        const uint2 o = S[(j | (1 << b)) * G + g];
        acc.x ^= o.x;
        acc.y ^= o.y;
      }
    D[e] = acc;
  }
  __syncthreads();
  fft_g(D, logG, logn, 0, t);
  // erased systematic positions: * locator (decode_main:185-188); present: as received
  for (int e = threadIdx.x; e < k * G; e += blockDim.x) {
    const int g = e & (G - 1), y = e >> logG;
    const bool have = y < nv && pr[y];
    uint32_t xl = 0, xh = 0;
    if (have) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint64_t pos = pos0 + 4 * g + q;
        if (pos < npos) {
          xh |= uint32_t(SH[uint64_t(y) * sstride + 2 * pos]) << (8 * q);
          xl |= uint32_t(SH[uint64_t(y) * sstride + 2 * pos + 1]) << (8 * q);
        }
      }
    } else {
      Tab T;
      load_tab(t.mtab, mul_index(E[y]), T);
      const uint2 r = D[e];
      mul_acc(r.x, r.y, T, xl, xh);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint64_t pos = pos0 + 4 * g + q;
      if (pos < npos) {
        O[(pos * k + y) * 2] = uint8_t(xh >> (8 * q));
        O[(pos * k + y) * 2 + 1] = uint8_t(xl >> (8 * q));
      }
    }
  }
  }
}

// reed-solomon.hpp:143-179: out[2(i*k + y) ..] = shard_y[2i ..]
__global__ void __launch_bounds__(kBlock) systematic_g(const uint8_t *__restrict__ shards,
                                                       uint64_t slen, uint64_t sstride, int nv,
                                                       int logk, uint8_t *__restrict__ out,
                                                       uint64_t ostride, uint32_t batch,
                                                       uint32_t *sig_flag, uint32_t sig_v) {
  const int k = 1 << logk;
  const uint64_t npos = slen / 2;
  const uint64_t total = npos * k;
  for (uint32_t b = blockIdx.y; b < batch; b += gridDim.y) {
    const uint8_t *SH = shards + uint64_t(b) * nv * sstride;
    uint8_t *O = out + uint64_t(b) * ostride;
    for (uint64_t e = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; e < total;
         e += uint64_t(gridDim.x) * blockDim.x) {
      const uint64_t i = e >> logk;
      const int y = int(e & (k - 1));
      O[2 * e] = SH[uint64_t(y) * sstride + 2 * i];
      O[2 * e + 1] = SH[uint64_t(y) * sstride + 2 * i + 1];
    }
  }
  signal_end(sig_flag, sig_v);  // (single-workgroup launches only)
}

// completion signal of a per-call C-ABI call: after the call's work on the
// stream, one lane stores `v` to a pinned host word at system scope; the host
// spins on it (a host spin on a kernel-written flag is ~5 us faster per round
// trip than hipStreamSynchronize: scripts/micro/launch_lat.hip)
__global__ void signal_host(uint32_t *flag, uint32_t v) {
  __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

int ilog2(uint32_t v) { return 31 - __builtin_clz(v); }

// payload slots in gridDim.y (hardware limit 65535); the kernels loop over the rest
size_t grid_y(size_t batch) { return batch < 65535 ? batch : 65535; }

int groups_for(uint32_t size) {  // byte-planar groups per workgroup
  if (size >= kLdsSlots) return 1;
  uint32_t g = kLdsSlots / size;
  return int(g > 64 ? 64 : g);
}

}  // namespace

bool locator_wave_applicable(uint32_t n) { return n >= 64 && n <= 4096; }

// zeroes a dynamic schedule's tile counters in stream order.  A kernel, not
// hipMemsetAsync: a memset captured into a hipGraph did not re-zero the
// counters on replay here (the reconstruct of the second replay found its
// queue drained: tests/test_gpu_parity.py test_graph_capture_ws at nv 4096)
__global__ void zero_words(uint32_t *p, uint32_t n) {
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) p[i] = 0;
}

hipError_t launch_zero_counters(uint32_t *p, size_t bytes, hipStream_t s) {
  hipLaunchKernelGGL(zero_words, dim3(1), dim3(64), 0, s, p, uint32_t(bytes / 4));
  return hipGetLastError();
}

hipError_t launch_signal_host(uint32_t *h_flag, uint32_t v, hipStream_t s) {
  hipLaunchKernelGGL(signal_host, dim3(1), dim3(1), 0, s, h_flag, v);
  return hipGetLastError();
}

// Encode scratch that is only a tile counter (the k = 16 .. 1024 fast
// kernels): optional, the kernels fall back to a static schedule without it.
bool encode_scratch_optional(const CodeParams &p) {
  return k1024_applicable(p) || k256_applicable(p) || k512w_applicable(p) || kw_applicable(p);
}

size_t encode_scratch_bytes(const CodeParams &p, size_t plen, size_t batch) {
  if (k1024_applicable(p)) return k1024_scratch_bytes(plen, batch);
  if (k256_applicable(p)) return k256_scratch_bytes(p);
  if (k512w_applicable(p)) return k512w_scratch_bytes(p);
  if (kw_applicable(p)) return kw_scratch_bytes(p);
  if (p.k <= uint32_t(kLdsSlots)) return 0;
  const size_t pieces = shard_len(p.k, plen) / 2;
  const size_t tiles = (pieces + 3) / 4;
  return tiles * grid_y(batch) * 2 * size_t(p.k) * sizeof(uint2);
}

hipError_t launch_encode(const CodeParams &p, const DevTables &t, const uint8_t *d_payloads,
                         size_t plen, size_t pstride, size_t batch, uint8_t *d_shards,
                         size_t sstride, void *scratch, hipStream_t s, HostSig *sig) {
  if (batch == 0 || plen == 0) return hipSuccess;
  const bool aligned = (reinterpret_cast<uintptr_t>(d_payloads) % 16 == 0) &&
                       (reinterpret_cast<uintptr_t>(d_shards) % 8 == 0) &&
                       (batch == 1 || pstride % 16 == 0) && sstride % 8 == 0;
  if (k256_applicable(p) &&
      (k256_packed(plen, pstride, batch, reinterpret_cast<uintptr_t>(d_payloads),
                   reinterpret_cast<uintptr_t>(d_shards), sstride)
           ? k256_packed_ok(plen, batch, reinterpret_cast<uintptr_t>(d_shards), sstride)
           : aligned))
    return launch_encode_k256(p, t, d_payloads, plen, pstride, batch, d_shards, sstride, scratch, s);
  if (aligned && k512w_applicable(p))
    return launch_encode_k512w(p, t, d_payloads, plen, pstride, batch, d_shards, sstride, scratch, s);
  if (aligned && kw_applicable(p))
    return launch_encode_kw(p, t, d_payloads, plen, pstride, batch, d_shards, sstride, scratch, s);
  if (aligned && k1024_applicable(p))
    return launch_encode_k1024(p, t, d_payloads, plen, pstride, batch, d_shards, sstride, scratch, s);
  const size_t sl = shard_len(p.k, plen);
  const int G = groups_for(p.k);
  const size_t tiles = (sl / 2 + 4 * G - 1) / (4 * G);
  const bool lds = p.k <= uint32_t(kLdsSlots);
  const size_t shm = lds ? 2 * size_t(p.k) * G * sizeof(uint2) : 0;
  dim3 grid((unsigned)tiles, (unsigned)grid_y(batch));
  const bool fuse = sig && sig->flag && grid.x * grid.y == 1;
  if (fuse) sig->fused = true;
  hipLaunchKernelGGL(encode_g, grid, dim3(kBlock), shm, s, d_payloads, uint64_t(plen),
                     uint64_t(pstride), d_shards, uint64_t(sl), uint64_t(sstride), int(p.nv),
                     ilog2(p.n), ilog2(p.k), ilog2(uint32_t(G)), uint32_t(batch), t,
                     lds ? nullptr : static_cast<uint2 *>(scratch), fuse ? sig->flag : nullptr,
                     fuse ? sig->v : 0u);
  return hipGetLastError();
}

namespace {
size_t dedup_cap(size_t batch) {  // hash slots: a power of two >= 2 * batch (batch < 2^31)
  size_t c = 64;
  while (c < 2 * batch) c <<= 1;
  return c;
}
}  // namespace

size_t dedup_scratch_bytes(size_t batch) {
  const size_t cap = dedup_cap(batch);
  return batch * 8 + cap * 8 + cap * 4;  // hashes, keys, values
}

hipError_t launch_dedup_patterns(const CodeParams &p, const uint8_t *d_present, size_t batch,
                                 uint32_t *d_pattern, void *scratch, hipStream_t s) {
  if (batch == 0) return hipSuccess;
  if (!scratch || batch >= (size_t(1) << 31)) return hipErrorInvalidValue;
  const uint32_t cap = uint32_t(dedup_cap(batch));
  uint64_t *hash = static_cast<uint64_t *>(scratch);
  unsigned long long *keys = reinterpret_cast<unsigned long long *>(hash + batch);
  uint32_t *vals = reinterpret_cast<uint32_t *>(keys + cap);
  if (const hipError_t e = hipMemsetAsync(keys, 0, size_t(cap) * 8, s); e != hipSuccess) return e;
  if (const hipError_t e = hipMemsetAsync(vals, 0xff, size_t(cap) * 4, s); e != hipSuccess) return e;
  hipLaunchKernelGGL(pattern_hash, dim3(unsigned(batch)), dim3(kBlock), 0, s, d_present, int(p.nv),
                     int(p.n), hash);
  hipLaunchKernelGGL(pattern_insert, dim3(unsigned((batch + kBlock - 1) / kBlock)), dim3(kBlock), 0, s,
                     hash, uint32_t(batch), keys, vals, cap);
  hipLaunchKernelGGL(pattern_resolve, dim3(unsigned(batch)), dim3(kBlock), 0, s, d_present,
                     int(p.nv), int(p.n), hash, keys, vals, cap, d_pattern);
  return hipGetLastError();
}

hipError_t launch_error_locator(const CodeParams &p, const uint8_t *d_present, size_t batch,
                                const uint16_t *d_fold, const uint32_t *d_pattern,
                                uint16_t *d_err_log, hipStream_t s) {
  if (batch == 0) return hipSuccess;
  if (locator_wave_applicable(p.n)) {
    const dim3 grid(unsigned((batch + 3) / 4));
#define ECAMD_LOC_W(VV)                                                                          \
  case VV:                                                                                       \
    hipLaunchKernelGGL(error_locator_w<VV>, grid, dim3(256), 0, s, d_present, int(p.nv),         \
                       uint32_t(batch), d_fold, d_pattern, d_err_log);                           \
    break;
    switch (p.n / 64) {
      ECAMD_LOC_W(1) ECAMD_LOC_W(2) ECAMD_LOC_W(4) ECAMD_LOC_W(8) ECAMD_LOC_W(16) ECAMD_LOC_W(32)
      ECAMD_LOC_W(64)
      default: return hipErrorInvalidValue;
    }
#undef ECAMD_LOC_W
    return hipGetLastError();
  }
  const size_t shm = size_t(p.n) * sizeof(uint16_t);
  int cus = 0;
  if (const hipError_t e = prepare_kernel(reinterpret_cast<const void *>(&error_locator_g), 65536 * 2, &cus);
      e != hipSuccess)
    return e;
  hipLaunchKernelGGL(error_locator_g, dim3(unsigned(batch)), dim3(kBlock), shm, s, d_present,
                     int(p.nv), ilog2(p.n), d_fold, d_pattern, d_err_log,
                     static_cast<uint16_t *>(nullptr));
  return hipGetLastError();
}

hipError_t launch_broadcast_locators(const CodeParams &p, const uint32_t *d_pattern, size_t batch,
                                     uint16_t *d_err_log, hipStream_t s) {
  if (batch == 0) return hipSuccess;
  hipLaunchKernelGGL(pattern_broadcast, dim3(unsigned(batch)), dim3(kBlock), 0, s, d_pattern,
                     int(p.n), d_err_log);
  return hipGetLastError();
}

size_t reconstruct_scratch_bytes(const CodeParams &p, size_t slen, size_t batch) {
  if (n4096_applicable(p)) return n4096_scratch_bytes(p, batch);
  if (n1024_applicable(p)) return n1024_scratch_bytes(p, batch);
  if (decgen_applicable(p)) return gather_order_bytes(p, batch);
  if (p.n <= uint32_t(kLdsSlots)) return 0;
  const size_t tiles = (slen / 2 + 3) / 4;
  return tiles * grid_y(batch) * 2 * size_t(p.n) * sizeof(uint2);
}

hipError_t launch_reconstruct(const CodeParams &p, const DevTables &t, const uint8_t *d_shards,
                              size_t slen, size_t sstride, const uint8_t *d_present,
                              const uint16_t *d_err_log, const uint32_t *d_pattern, size_t batch,
                              uint8_t *d_out, size_t ostride, void *scratch, hipStream_t s) {
  if (batch == 0 || slen < 2) return hipSuccess;
  const bool aligned = (reinterpret_cast<uintptr_t>(d_shards) % 16 == 0) &&
                       (reinterpret_cast<uintptr_t>(d_out) % 8 == 0) && sstride % 16 == 0 &&
                       (batch == 1 || ostride % 8 == 0);
  const bool out8 = reinterpret_cast<uintptr_t>(d_out) % 8 == 0 && (batch == 1 || ostride % 8 == 0) &&
                    reinterpret_cast<uintptr_t>(d_present) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(d_err_log) % 16 == 0;  // vector loads of flag / E rows
  // ECCR_AMD_RECON_WAVES=8 (experiments): the 8-wave kernel where the 12-wave one applies
  static const bool waves8 = [] {
    const char *e = std::getenv("ECCR_AMD_RECON_WAVES");
    return e && e[0] == '8';
  }();
  const bool packed1024 = n1024_packed(slen, reinterpret_cast<uintptr_t>(d_shards), sstride);
  if (n1024_applicable(p) && !packed1024 && aligned && out8 && !waves8 && slen / 2 >= 48)
    return launch_reconstruct_n1024x(p, t, d_shards, slen, sstride, d_present, d_err_log, d_pattern, batch,
                                     d_out, ostride, scratch, s);
  if (n1024_applicable(p) &&
      (packed1024 ? out8 && reinterpret_cast<uintptr_t>(d_shards) % 2 == 0 && sstride % 2 == 0
                  : aligned && out8))
    return launch_reconstruct_n1024(p, t, d_shards, slen, sstride, d_present, d_err_log, d_pattern, batch,
                                    d_out, ostride, scratch, s);
  if (aligned && n4096_applicable(p) && reinterpret_cast<uintptr_t>(d_out) % 16 == 0 &&
      (batch == 1 || ostride % 16 == 0))
    return launch_reconstruct_n4096(p, t, d_shards, slen, sstride, d_present, d_err_log, d_pattern, batch,
                                    d_out, ostride, scratch, s);
  if (aligned && decgen_applicable(p) && reinterpret_cast<uintptr_t>(d_out) % 16 == 0 &&
      (batch == 1 || ostride % 16 == 0))
    return launch_reconstruct_gen(p, t, d_shards, slen, sstride, d_present, d_err_log, d_pattern, batch,
                                  d_out, ostride, scratch, s);
  const int G = groups_for(p.n);
  const size_t tiles = (slen / 2 + 4 * G - 1) / (4 * G);
  const bool lds = p.n <= uint32_t(kLdsSlots);
  const size_t shm = lds ? 2 * size_t(p.n) * G * sizeof(uint2) : 0;
  dim3 grid((unsigned)tiles, (unsigned)grid_y(batch));
  hipLaunchKernelGGL(reconstruct_g, grid, dim3(kBlock), shm, s, d_shards, uint64_t(slen),
                     uint64_t(sstride), d_present, d_err_log, d_out, uint64_t(ostride), int(p.nv),
                     ilog2(p.n), ilog2(p.k), ilog2(uint32_t(G)), uint32_t(batch), d_pattern, t,
                     lds ? nullptr : static_cast<uint2 *>(scratch));
  return hipGetLastError();
}

hipError_t launch_systematic(const CodeParams &p, const uint8_t *d_shards, size_t slen,
                             size_t sstride, size_t batch, uint8_t *d_out, size_t ostride,
                             hipStream_t s, HostSig *sig) {
  if (batch == 0 || slen < 2) return hipSuccess;
  const size_t total = slen / 2 * p.k;
  size_t blocks = (total + kBlock - 1) / kBlock;
  if (blocks > 4096) blocks = 4096;
  const bool fuse = sig && sig->flag && blocks * grid_y(batch) == 1;
  if (fuse) sig->fused = true;
  hipLaunchKernelGGL(systematic_g, dim3(unsigned(blocks), unsigned(grid_y(batch))), dim3(kBlock), 0,
                     s, d_shards, uint64_t(slen), uint64_t(sstride), int(p.nv), ilog2(p.k), d_out,
                     uint64_t(ostride), uint32_t(batch), fuse ? sig->flag : nullptr, fuse ? sig->v : 0u);
  return hipGetLastError();
}

}  // namespace ecamd
