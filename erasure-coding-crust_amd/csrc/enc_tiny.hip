// enc_tiny.hip — the per-call C ABI's encode for tiny codes and payloads
// (n <= 16, i.e. n_validators <= 16; payload <= kTinyBytes): the shape of the
// reference's own benchmark (`benchmark/benchmark.cpp:15`, n_validators = 6,
// 15 B .. 5 KB payloads through ECCR_Test_MeasurePerformance).
//
// A call of that size is launch latency, not work (scripts/micro/small_io.hip:
// launch + host spin on a pinned flag 7.1-7.6 us; reading the payload from
// pinned host memory +0.7-1.1 us).  So:
//  * the payload travels in the kernel arguments (no host-memory reads, no
//    host-side copy into the staging buffer);
//  * so do the code's skew tables (n - 1 <= 15 of them, mslot[0 .. n-2],
//    built on the host): no dependent device-memory round trip, no LDS;
//  * one thread per piece keeps its k <= 4 symbols (kMaxK; tiny_applicable: n <= 16) in registers through the
//    IFFT_k and each coset's FFT_k (additive_fft.hpp:99-141; encodeLow,
//    poly_encoder.hpp:217-240), and writes its 2-byte BE symbol of every shard
//    row straight to the pinned output (a wave's 64 pieces are 128 contiguous
//    bytes of a row);
//  * the same workgroup stores the completion flag (HostSig).
// The multiply is mul_acc on byte-planar words with the symbol in byte 0.
// systematic_tiny is the same for the per-call decode from all k systematic
// shards (reed-solomon.hpp:143-179): the k shards (<= kTinyBytes together) in
// the kernel arguments, the interleaved payload written to the pinned output.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstring>
#include <type_traits>

#include "ec_device.hpp"
#include "ec_kernels.hpp"

namespace ecamd {
namespace {

constexpr int kThreads = 256;
constexpr int kLogMaxK = 2;  // n <= 16: k <= 4
constexpr int kMaxK = 1 << kLogMaxK;

// PB: payload bytes carried (the argument block is copied at every launch:
// 64 / 512 / 2048 by the call's size)
template <int PB>
struct TinyArgs {
  uint32_t w[PB / 4];
};

// the code's multiply tables, mslot[0 .. n-2] (every skew of IFFT_k at 0 and
// FFT_k at the cosets below n), in the kernel arguments too; NT - 1 slots
// (NT = 8 for n <= 8, the reference benchmark's n_validators = 6: 560 B of
// arguments instead of 1,200 B to copy per launch)
template <int NT>
struct TinyTabs {
  MulTab t[NT - 1];
};

template <int PB, int NT>
__global__ void __launch_bounds__(kThreads) encode_tiny(TinyArgs<PB> pay, TinyTabs<NT> tt, uint32_t nv, uint32_t n,
                                                         uint32_t logk, uint32_t npieces,
                                                         uint8_t *__restrict__ out, uint64_t ostride,
                                                         uint32_t *sig_flag, uint32_t sig_v) {
  const uint32_t tid = threadIdx.x, k = 1u << logk;
  // the tables into LDS in one parallel round of loads from the arguments
  // (read where used instead, each multiply waited for its own load)
  __shared__ MulTab tabs[NT - 1];
  for (uint32_t i = tid; i < 5 * (n - 1); i += blockDim.x)  // (75 chunks at n = 16: more than a wave)
    reinterpret_cast<uint4 *>(tabs)[i] = reinterpret_cast<const uint4 *>(tt.t)[i];
  // piece p = symbols p*k .. p*k + k - 1, BE (poly_encoder.hpp:53-76):
  // bytes [2pk, 2pk + 2k), zero past the payload (the host pads the
  // arguments), from two unconditional word loads; the first piece's are
  // requested with the tables, before the barrier
  uint32_t q0 = 0, q1 = 0;
  const auto words = [&](uint32_t p) {
    const uint32_t w0 = 2 * p * k / 4;
    q0 = pay.w[w0 < PB / 4 ? w0 : PB / 4 - 1];
    q1 = pay.w[w0 + 1 < PB / 4 ? w0 + 1 : PB / 4 - 1];
  };
  if (tid < npieces) words(tid);
  __syncthreads();
  const auto tab = [&](uint32_t i, Tab &T) {
    const uint4 *q = reinterpret_cast<const uint4 *>(&tabs[i]);
#pragma unroll
    for (int w = 0; w < 5; ++w) {
      const uint4 v = q[w];
      T.t[4 * w] = v.x;
      T.t[4 * w + 1] = v.y;
      T.t[4 * w + 2] = v.z;
      T.t[4 * w + 3] = v.w;
    }
  };
  // row r, piece p: 2 bytes BE at 2p
  const auto put = [&](uint32_t r, uint32_t p, uint32_t lo, uint32_t hi) {
    *reinterpret_cast<uint16_t *>(out + uint64_t(r) * ostride + 2 * p) = uint16_t(hi | (lo << 8));
  };
  const uint32_t nth = blockDim.x;  // 64 .. kThreads: the pieces, rounded up to whole waves
  for (uint32_t p = tid; p < npieces; p += nth) {
    const uint32_t b0 = 2 * p * k;
    const uint64_t q = (uint64_t(q1) << 32 | q0) >> (8 * (b0 & 3));
    if (p + nth < npieces) words(p + nth);  // the next piece of this thread
    uint32_t cl[kMaxK], ch[kMaxK];
#pragma unroll
    for (int i = 0; i < kMaxK; ++i) {  // symbol in byte 0 of (l, h)
      ch[i] = uint32_t(q >> (16 * i)) & 0xFFu;
      cl[i] = uint32_t(q >> (16 * i + 8)) & 0xFFu;
      if (uint32_t(i) < k) put(i, p, cl[i], ch[i]);  // systematic rows (k <= nv)
    }
    // IFFT_k at index 0: b ^= a; a ^= b * skew  (stage m, block skew j - 1)
    // (stages and registers compile-time: no dynamic register indexing)
#pragma unroll
    for (int m = 0; m < kLogMaxK; ++m) {
      if (uint32_t(m) >= logk) break;
      const int d = 1 << m;
#pragma unroll
      for (int i = 0; i < kMaxK; ++i) {
        if (uint32_t(i) >= k || (i & d)) continue;
        const int b = i | d;
        Tab T;
        tab(uint32_t((i & ~(2 * d - 1)) + d - 1), T);
        cl[b] ^= cl[i];
        ch[b] ^= ch[i];
        mul_acc(cl[b], ch[b], T, cl[i], ch[i]);
      }
    }
    // each coset s = k, 2k, .. below n and nv: FFT_k at index s of the
    // coefficients (a ^= b * skew; b ^= a, stages from the top)
    for (uint32_t s = k; s < n && s < nv; s += k) {
      uint32_t xl[kMaxK], xh[kMaxK];
#pragma unroll
      for (int i = 0; i < kMaxK; ++i) {
        xl[i] = cl[i];
        xh[i] = ch[i];
      }
#pragma unroll
      for (int m = kLogMaxK - 1; m >= 0; --m) {
        if (uint32_t(m) >= logk) continue;
        const int d = 1 << m;
#pragma unroll
        for (int i = 0; i < kMaxK; ++i) {
          if (uint32_t(i) >= k || (i & d)) continue;
          const int b = i | d;
          Tab T;
          tab(s + uint32_t((i & ~(2 * d - 1)) + d - 1), T);
          mul_acc(xl[b], xh[b], T, xl[i], xh[i]);
          xl[b] ^= xl[i];
          xh[b] ^= xh[i];
        }
      }
#pragma unroll
      for (int i = 0; i < kMaxK; ++i)
        if (uint32_t(i) < k && s + i < nv) put(s + i, p, xl[i] & 0xFFu, xh[i] & 0xFFu);
    }
  }
  // completion flag (HostSig): every thread's rows visible at system scope first
  __threadfence_system();
  __syncthreads();
  if (tid == 0 && sig_flag) __hip_atomic_store(sig_flag, sig_v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <int PB>
__global__ void __launch_bounds__(kThreads) systematic_tiny(TinyArgs<PB> sh, uint32_t slen, uint32_t logk,
                                                             uint8_t *__restrict__ out, uint32_t *sig_flag,
                                                             uint32_t sig_v) {
  // shard y's bytes at sh[y * slen ..]; out[2 (i k + y) ..] = shard_y[2 i ..]
  const uint8_t *S = reinterpret_cast<const uint8_t *>(sh.w);
  const uint32_t k = 1u << logk, total = (slen / 2) * k;
  for (uint32_t e = threadIdx.x; e < total; e += blockDim.x) {
    const uint32_t i = e >> logk, y = e & (k - 1);
    const uint32_t a = y * slen + 2 * i;
    *reinterpret_cast<uint16_t *>(out + 2 * e) = uint16_t(S[a] | (uint32_t(S[a + 1]) << 8));
  }
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0 && sig_flag)
    __hip_atomic_store(sig_flag, sig_v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// one thread per piece (output symbol), whole waves, at most kThreads: a
// 15-B call is one wave instead of four
uint32_t block_for(uint32_t items) {
  const uint32_t w = (items + 63) / 64 * 64;
  return w < 64 ? 64 : w > uint32_t(kThreads) ? uint32_t(kThreads) : w;
}

}  // namespace

bool tiny_applicable(const CodeParams &p, size_t plen, size_t ostride) {
  return p.n <= uint32_t(kTinyMaxN) && p.k <= uint32_t(kMaxK) && plen >= 1 && plen <= kTinyBytes &&
         ostride % 2 == 0;
}

namespace {
// the code's tables, built once per n on the host (mslot[i] = mtab[skews[i]])
template <int NT>
const TinyTabs<NT> &tiny_tabs(uint32_t n) {
  static const std::array<TinyTabs<NT>, 5> all = [] {
    std::array<TinyTabs<NT>, 5> a{};
    const Field &f = field();
    for (int lg = 0; lg < 5 && (1 << lg) <= NT; ++lg)
      for (uint32_t i = 0; i + 1 < (1u << lg); ++i) a[lg].t[i] = f.mtab[f.skews[i]];
    return a;
  }();
  return all[__builtin_ctz(n)];
}
}  // namespace

hipError_t launch_encode_tiny(const CodeParams &p, const DevTables &t, const uint8_t *h_payload, size_t plen,
                              uint8_t *out, size_t ostride, hipStream_t s, HostSig *sig) {
  if (!tiny_applicable(p, plen, ostride) || !out || !h_payload) return hipErrorInvalidValue;
  const uint32_t logk = uint32_t(__builtin_ctz(p.k));
  const uint32_t npieces = uint32_t(shard_len(p.k, plen) / 2);
  const auto go = [&](auto tag, auto ntag) {
    constexpr int PB = decltype(tag)::value, NT = decltype(ntag)::value;
    TinyArgs<PB> pay;
    // zero past the payload: the last piece's padding and the words a load
    // may read beyond it (clamped to the block)
    const size_t pad_end = std::min(size_t(PB), size_t(2) * p.k * npieces + 8);
    std::memcpy(pay.w, h_payload, plen);
    if (pad_end > plen) std::memset(reinterpret_cast<uint8_t *>(pay.w) + plen, 0, pad_end - plen);
    hipLaunchKernelGGL((encode_tiny<PB, NT>), dim3(1), dim3(block_for(npieces)), 0, s, pay, tiny_tabs<NT>(p.n),
                       p.nv, p.n, logk, npieces, out, uint64_t(ostride), sig ? sig->flag : nullptr,
                       sig ? sig->v : 0u);
  };
  const auto by_n = [&](auto tag) {
    if (p.n <= 8) go(tag, std::integral_constant<int, 8>());
    else go(tag, std::integral_constant<int, kTinyMaxN>());
  };
  if (plen <= 64) by_n(std::integral_constant<int, 64>());
  else if (plen <= 512) by_n(std::integral_constant<int, 512>());
  else by_n(std::integral_constant<int, int(kTinyBytes)>());
  const hipError_t e = hipGetLastError();
  if (e == hipSuccess && sig && sig->flag) sig->fused = true;
  return e;
}

bool systematic_tiny_applicable(const CodeParams &p, size_t slen) {
  return slen >= 2 && slen % 2 == 0 && size_t(p.k) * slen <= kTinyBytes;
}

hipError_t launch_systematic_tiny(const CodeParams &p, const uint8_t *h_shards, size_t slen, size_t sstride,
                                  uint8_t *out, hipStream_t s, HostSig *sig) {
  if (!systematic_tiny_applicable(p, slen) || !out || !h_shards) return hipErrorInvalidValue;
  const size_t bytes = size_t(p.k) * slen;
  const uint32_t logk = uint32_t(__builtin_ctz(p.k));
  const auto go = [&](auto tag) {
    constexpr int PB = decltype(tag)::value;
    TinyArgs<PB> a;
    for (uint32_t y = 0; y < p.k; ++y) std::memcpy(reinterpret_cast<uint8_t *>(a.w) + y * slen, h_shards + y * sstride, slen);
    hipLaunchKernelGGL(systematic_tiny<PB>, dim3(1), dim3(block_for(uint32_t(slen / 2) * p.k)), 0, s, a,
                       uint32_t(slen), logk, out,
                       sig ? sig->flag : nullptr, sig ? sig->v : 0u);
  };
  if (bytes <= 64) go(std::integral_constant<int, 64>());
  else if (bytes <= 512) go(std::integral_constant<int, 512>());
  else go(std::integral_constant<int, int(kTinyBytes)>());
  const hipError_t e = hipGetLastError();
  if (e == hipSuccess && sig && sig->flag) sig->fused = true;
  return e;
}

// one empty launch of each variant (no pieces, no tables, no flag): the first
// launch of a kernel in a process costs ~0.5 ms (mp_calls.cpp: the first
// ECCR_Test_MeasurePerformance encode 546 us, the next ones 8-9 us), so the
// device set-up pays it instead of the first call
hipError_t warm_encode_tiny(hipStream_t s) {
  const auto go = [&](auto tag, auto ntag) {
    constexpr int PB = decltype(tag)::value, NT = decltype(ntag)::value;
    TinyArgs<PB> pay;
    pay.w[0] = 0;
    hipLaunchKernelGGL((encode_tiny<PB, NT>), dim3(1), dim3(kThreads), 0, s, pay, tiny_tabs<NT>(2), 2u, 2u, 0u, 0u,
                       nullptr, uint64_t(0), nullptr, 0u);
  };
  const auto both = [&](auto tag) {
    go(tag, std::integral_constant<int, 8>());
    go(tag, std::integral_constant<int, kTinyMaxN>());
  };
  both(std::integral_constant<int, 64>());
  both(std::integral_constant<int, 512>());
  both(std::integral_constant<int, int(kTinyBytes)>());
  const auto gs = [&](auto tag) {
    constexpr int PB = decltype(tag)::value;
    TinyArgs<PB> a;
    a.w[0] = 0;
    hipLaunchKernelGGL(systematic_tiny<PB>, dim3(1), dim3(kThreads), 0, s, a, 0u, 0u, nullptr, nullptr, 0u);
  };
  gs(std::integral_constant<int, 64>());
  gs(std::integral_constant<int, 512>());
  gs(std::integral_constant<int, int(kTinyBytes)>());
  return hipGetLastError();
}

}  // namespace ecamd
