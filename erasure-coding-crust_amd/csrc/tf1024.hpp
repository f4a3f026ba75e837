// tf1024.hpp — register-blocked 1024-point additive (I)FFT on one byte-planar
// group per wave (4 codewords / pieces), shared by the k = 1024 encode and the
// n = 4096 reconstruct (enc_k1024.hip, dec_n4096.hip).
//
// A wave holds the 1024 positions of its group as 64 lanes x 16 registers
// (uint2 {low bytes, high bytes} of 4 symbols each) in one of three layouts:
//   A: pos = 16 lane + r                              (register bits = p0..p3)
//   B: pos = (lane & 15) | r << 4 | (lane >> 4) << 8   (register bits = p4..p7)
//   C: pos = lane | ((r >> 2) & 3) << 6 | (r & 3) << 8 (register bits = p8, p9, p6, p7)
// and moves between them through a wave-private 8 KB LDS region (raddr swizzle:
// every access pattern below is bank-conflict free).  The butterflies are
// additive_fft.hpp:99-141 with skew index (pos & ~(2d-1)) + d - 1 relative to
// the transform's offset; the multiply tables for that offset's 1023 skews sit
// in LDS (LdsTabs<1024>) and are addressed linearly (tlin).
#pragma once

#include "ec_device.hpp"

namespace ecamd {
namespace tf {

using Tabs = LdsTabs<1024>;
constexpr int REG_BYTES = 1024 * 8;  // one group: 1024 x uint2

struct S16 {
  uint32_t l[16], h[16];
};

__device__ __forceinline__ uint32_t raddr(uint32_t v) {
  const uint32_t f = (v & 31) ^ ((v >> 4) & 31);
  return ((v >> 5) << 8) | (f << 3);
}

// GF(2)-linear part of LdsTabs::addr: tlin(a | b) = tlin(a) ^ tlin(b) (disjoint a, b)
__host__ __device__ constexpr uint32_t tlin(uint32_t idx) {
  return ((idx >> 4) << 8) | (((idx ^ (idx >> 4) ^ (idx >> 8)) & 15) << 4);
}

__device__ __forceinline__ void tab_at(const uint8_t *lds, uint32_t lin, Tab &T) {
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    const uint4 v = *reinterpret_cast<const uint4 *>(lds + q * Tabs::kPlane + lin);
    T.t[4 * q] = v.x;
    T.t[4 * q + 1] = v.y;
    T.t[4 * q + 2] = v.z;
    T.t[4 * q + 3] = v.w;
  }
}

__device__ __forceinline__ uint32_t skew_idx(uint32_t pos_a, int m) {
  const uint32_t d = 1u << m;
  return (pos_a & ~(2 * d - 1)) + d - 1;
}

__device__ __forceinline__ void ib(S16 &s, int a, int b, const Tab &T) {  // inverse butterfly
  s.l[b] ^= s.l[a];
  s.h[b] ^= s.h[a];
  mul_acc(s.l[b], s.h[b], T, s.l[a], s.h[a]);
}

__device__ __forceinline__ void fb(S16 &s, int a, int b, const Tab &T) {  // forward butterfly
  mul_acc(s.l[b], s.h[b], T, s.l[a], s.h[a]);
  s.l[b] ^= s.l[a];
  s.h[b] ^= s.h[a];
}

// radix-16 passes over position bits B0..B0+3 held in registers; lb = tlin of
// the lane part of the position.  The next block's table is requested one
// step ahead of its use.
template <int B0>
__device__ __forceinline__ void ipass4(S16 &s, const uint8_t *tabs, uint32_t lb) {
  Tab T[2];
  tab_at(tabs, lb ^ tlin(skew_idx(0, B0)), T[0]);
  int k = 0;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int d = 1 << t;
#pragma unroll
    for (int blk = 0; blk < 16; blk += 2 * d, ++k) {
      const int nt = blk + 2 * d < 16 ? t : t + 1, nblk = blk + 2 * d < 16 ? blk + 2 * d : 0;
      if (nt < 4) tab_at(tabs, lb ^ tlin(skew_idx(uint32_t(nblk) << B0, B0 + nt)), T[(k + 1) & 1]);
#pragma unroll
      for (int i = 0; i < d; ++i) ib(s, blk + i, blk + i + d, T[k & 1]);
    }
  }
}

template <int B0>
__device__ __forceinline__ void fpass4(S16 &s, const uint8_t *tabs, uint32_t lb) {
  Tab T[2];
  tab_at(tabs, lb ^ tlin(skew_idx(0, B0 + 3)), T[0]);
  int k = 0;
#pragma unroll
  for (int t = 3; t >= 0; --t) {
    const int d = 1 << t;
#pragma unroll
    for (int blk = 0; blk < 16; blk += 2 * d, ++k) {
      const int nt = blk + 2 * d < 16 ? t : t - 1, nblk = blk + 2 * d < 16 ? blk + 2 * d : 0;
      if (nt >= 0) tab_at(tabs, lb ^ tlin(skew_idx(uint32_t(nblk) << B0, B0 + nt)), T[(k + 1) & 1]);
#pragma unroll
      for (int i = 0; i < d; ++i) fb(s, blk + i, blk + i + d, T[k & 1]);
    }
  }
}

// layout C: stage 8 (skew depends on p9 = r bit 1), stage 9 (one skew)
__device__ __forceinline__ void ipassC(S16 &s, const uint8_t *tabs) {
  Tab Ta, Tb;
  tab_at(tabs, tlin(skew_idx(0, 8)), Ta);
  tab_at(tabs, tlin(skew_idx(1u << 9, 8)), Tb);
#pragma unroll
  for (int hi = 0; hi < 4; ++hi) ib(s, 4 * hi, 4 * hi + 1, Ta);
  tab_at(tabs, tlin(skew_idx(0, 9)), Ta);
#pragma unroll
  for (int hi = 0; hi < 4; ++hi) ib(s, 4 * hi + 2, 4 * hi + 3, Tb);
#pragma unroll
  for (int hi = 0; hi < 4; ++hi) {
    ib(s, 4 * hi, 4 * hi + 2, Ta);
    ib(s, 4 * hi + 1, 4 * hi + 3, Ta);
  }
}

__device__ __forceinline__ void fpassC(S16 &s, const uint8_t *tabs) {
  Tab Ta, Tb;
  tab_at(tabs, tlin(skew_idx(0, 9)), Ta);
  tab_at(tabs, tlin(skew_idx(0, 8)), Tb);
#pragma unroll
  for (int hi = 0; hi < 4; ++hi) {
    fb(s, 4 * hi, 4 * hi + 2, Ta);
    fb(s, 4 * hi + 1, 4 * hi + 3, Ta);
  }
  tab_at(tabs, tlin(skew_idx(1u << 9, 8)), Ta);
#pragma unroll
  for (int hi = 0; hi < 4; ++hi) fb(s, 4 * hi, 4 * hi + 1, Tb);
#pragma unroll
  for (int hi = 0; hi < 4; ++hi) fb(s, 4 * hi + 2, 4 * hi + 3, Ta);
}

__device__ __forceinline__ uint32_t posA(uint32_t lane, int r) { return 16 * lane + uint32_t(r); }
__device__ __forceinline__ uint32_t posB(uint32_t lane, int r) {
  return (lane & 15) | (uint32_t(r) << 4) | ((lane >> 4) << 8);
}
__device__ __forceinline__ uint32_t posC(uint32_t lane, int r) {
  return lane | (uint32_t((r >> 2) & 3) << 6) | (uint32_t(r & 3) << 8);
}

enum Layout { LA, LB, LC };

template <Layout L>
__device__ __forceinline__ uint32_t pos_of(uint32_t lane, int r) {
  if constexpr (L == LA) return posA(lane, r);
  else if constexpr (L == LB) return posB(lane, r);
  else return posC(lane, r);
}

// wave-private exchange of the 16 registers from layout FROM to layout TO
template <Layout FROM, Layout TO>
__device__ __forceinline__ void exchange(S16 &s, uint8_t *my, uint32_t lane) {
  asm volatile("" : "+v"(lane));  // addresses computed here, not hoisted and kept live
#pragma unroll
  for (int r = 0; r < 16; ++r)
    *reinterpret_cast<uint2 *>(my + raddr(pos_of<FROM>(lane, r))) = make_uint2(s.l[r], s.h[r]);
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const uint2 x = *reinterpret_cast<const uint2 *>(my + raddr(pos_of<TO>(lane, r)));
    s.l[r] = x.x;
    s.h[r] = x.y;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// IFFT_1024 (inverse_afft, index = the tables' offset): layout A in, C out
__device__ __forceinline__ void ifft1024(S16 &s, const uint8_t *tabs, uint8_t *my, uint32_t lane) {
  asm volatile("" : "+v"(lane));
  ipass4<0>(s, tabs, tlin(16 * lane));
  exchange<LA, LB>(s, my, lane);
  ipass4<4>(s, tabs, tlin((lane >> 4) << 8));
  exchange<LB, LC>(s, my, lane);
  ipassC(s, tabs);
}

// FFT_1024 (afft): layout C in, A out
__device__ __forceinline__ void fft1024(S16 &s, const uint8_t *tabs, uint8_t *my, uint32_t lane) {
  asm volatile("" : "+v"(lane));
  fpassC(s, tabs);
  exchange<LC, LB>(s, my, lane);
  fpass4<4>(s, tabs, tlin((lane >> 4) << 8));
  exchange<LB, LA>(s, my, lane);
  fpass4<0>(s, tabs, tlin(16 * lane));
}

// byte-planar group (4 pieces / columns) -> big-endian u16 x4
__device__ __forceinline__ uint2 to_be(uint32_t l, uint32_t h) {
  return make_uint2(vperm(l, h, 0x05010400u), vperm(l, h, 0x07030602u));
}

}  // namespace tf
}  // namespace ecamd
