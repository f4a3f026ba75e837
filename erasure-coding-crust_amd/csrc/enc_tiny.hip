// enc_tiny.hip — the per-call C ABI's encode for tiny codes and payloads
// (n <= 32, i.e. n_validators <= 32; payload <= kTinyBytes): the shape of the
// reference's own benchmark (`benchmark/benchmark.cpp:15`, n_validators = 6,
// 15 B .. 5 KB payloads through ECCR_Test_MeasurePerformance).
//
// A call of that size is launch latency, not work (scripts/micro/small_io.hip:
// launch + host spin on a pinned flag 7.1-7.6 us; reading the payload from
// pinned host memory +0.7-1.1 us).  So:
//  * the payload travels in the kernel arguments (no host-memory reads, no
//    host-side copy into the staging buffer);
//  * the code's skew tables (n - 1 of them, mslot[0 .. n-2]) are fetched in
//    one parallel step into LDS;
//  * one thread per piece keeps its k <= 8 symbols in registers through the
//    IFFT_k and each coset's FFT_k (additive_fft.hpp:99-141; encodeLow,
//    poly_encoder.hpp:217-240), and writes its 2-byte BE symbol of every shard
//    row straight to the pinned output (a wave's 64 pieces are 128 contiguous
//    bytes of a row);
//  * the same workgroup stores the completion flag (HostSig).
// The multiply is mul_acc on byte-planar words with the symbol in byte 0.
#include <hip/hip_runtime.h>

#include <cstring>
#include <type_traits>

#include "ec_device.hpp"
#include "ec_kernels.hpp"

namespace ecamd {
namespace {

constexpr int kThreads = 256;
constexpr int kLogMaxK = 3;
constexpr int kMaxK = 1 << kLogMaxK;

// PB: payload bytes carried (the argument block is copied at every launch:
// 64 / 512 / 2048 by the call's size)
template <int PB>
struct TinyArgs {
  uint32_t w[PB / 4];
};

template <int PB>
__global__ void __launch_bounds__(kThreads) encode_tiny(TinyArgs<PB> pay, uint32_t plen, uint32_t nv,
                                                         uint32_t n, uint32_t logk, uint32_t npieces,
                                                         uint8_t *__restrict__ out, uint64_t ostride,
                                                         const MulTab *__restrict__ mslot,
                                                         uint32_t *sig_flag, uint32_t sig_v) {
  __shared__ MulTab tabs[kTinyMaxN];
  __shared__ uint32_t pw[PB / 4];
  const uint32_t tid = threadIdx.x, k = 1u << logk;
  // one parallel round of loads: the tables (skew slots 0 .. n-2, every
  // table of the code) and the payload's words out of the kernel arguments
  // into LDS (byte loads from the arguments, one per symbol byte, were a
  // chain of dependent round trips)
  if (tid < n - 1) tabs[tid] = mslot[tid];
  for (uint32_t i = tid; i < (plen + 3) / 4; i += kThreads) pw[i] = pay.w[i];
  __syncthreads();
  const uint8_t *P = reinterpret_cast<const uint8_t *>(pw);
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
  for (uint32_t p = tid; p < npieces; p += kThreads) {
    // piece p = symbols p*k .. p*k + k - 1, BE, zero past the payload
    // (poly_encoder.hpp:53-76); symbol in byte 0 of (l, h)
    uint32_t cl[kMaxK], ch[kMaxK];
#pragma unroll
    for (int i = 0; i < kMaxK; ++i) {
      cl[i] = ch[i] = 0;
      if (uint32_t(i) < k) {
        const uint32_t off = 2 * (p * k + i);
        ch[i] = off < plen ? P[off] : 0u;
        cl[i] = off + 1 < plen ? P[off + 1] : 0u;
        if (uint32_t(i) < nv) put(i, p, cl[i], ch[i]);  // systematic rows
      }
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

}  // namespace

bool tiny_applicable(const CodeParams &p, size_t plen, size_t ostride) {
  return p.n <= uint32_t(kTinyMaxN) && p.k <= uint32_t(kMaxK) && plen >= 1 && plen <= kTinyBytes &&
         ostride % 2 == 0;
}

hipError_t launch_encode_tiny(const CodeParams &p, const DevTables &t, const uint8_t *h_payload, size_t plen,
                              uint8_t *out, size_t ostride, hipStream_t s, HostSig *sig) {
  if (!tiny_applicable(p, plen, ostride) || !out || !h_payload) return hipErrorInvalidValue;
  const uint32_t logk = uint32_t(__builtin_ctz(p.k));
  const uint32_t npieces = uint32_t(shard_len(p.k, plen) / 2);
  const auto go = [&](auto tag) {
    constexpr int PB = decltype(tag)::value;
    TinyArgs<PB> pay;
    pay.w[(plen - 1) / 4] = 0;  // (the bytes past plen in the last word: read, unused)
    std::memcpy(pay.w, h_payload, plen);
    hipLaunchKernelGGL(encode_tiny<PB>, dim3(1), dim3(kThreads), 0, s, pay, uint32_t(plen), p.nv, p.n, logk,
                       npieces, out, uint64_t(ostride), t.mslot, sig ? sig->flag : nullptr, sig ? sig->v : 0u);
  };
  if (plen <= 64) go(std::integral_constant<int, 64>());
  else if (plen <= 512) go(std::integral_constant<int, 512>());
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
  const auto go = [&](auto tag) {
    constexpr int PB = decltype(tag)::value;
    TinyArgs<PB> pay;
    pay.w[0] = 0;
    hipLaunchKernelGGL(encode_tiny<PB>, dim3(1), dim3(kThreads), 0, s, pay, 1u, 2u, 1u, 0u, 0u, nullptr,
                       uint64_t(0), nullptr, nullptr, 0u);
  };
  go(std::integral_constant<int, 64>());
  go(std::integral_constant<int, 512>());
  go(std::integral_constant<int, int(kTinyBytes)>());
  return hipGetLastError();
}

}  // namespace ecamd
