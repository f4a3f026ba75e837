// enc_k256_common.hpp — pieces shared by the k = 256 encode kernels
// (enc_k256.hip: the n = 1024 packed and n = 2048 forms; enc_k256w.hip: the
// n = 1024 two-workgroups-per-CU form).  One byte-planar group of 4 pieces
// per instance (lanes 0-31 / 32-63), 8 positions of the 256-point transforms
// per lane in registers, wave-private LDS exchanges between the radix-8 passes.
#pragma once

#include <hip/hip_runtime.h>

#include "ec_device.hpp"

namespace ecamd {
namespace {

constexpr int GP = 1;  // byte-planar groups per lane

struct State {
  uint32_t l[GP][8], h[GP][8];  // [group][register]: low / high byte planes
};

__device__ __forceinline__ void mul_any(uint32_t xl, uint32_t xh, const Tab &T, uint32_t &yl, uint32_t &yh) {
  mul_acc(xl, xh, T, yl, yh);
}
__device__ __forceinline__ void mul_any(uint32_t xl, uint32_t xh, const SubTab &T, uint32_t &yl,
                                        uint32_t &yh) {
  mul_acc_sub(xl, xh, T, yl, yh);
}
__device__ __forceinline__ void mul_any(uint32_t xl, uint32_t xh, const F9Tab &T, uint32_t &yl,
                                        uint32_t &yh) {
  mul_acc_f9(xl, xh, T, yl, yh);
}

template <typename T>
__device__ __forceinline__ void ibfly(State &s, int ra, int rb, const T &Tb) {
#pragma unroll
  for (int g = 0; g < GP; ++g) {
    s.l[g][rb] ^= s.l[g][ra];
    s.h[g][rb] ^= s.h[g][ra];
    mul_any(s.l[g][rb], s.h[g][rb], Tb, s.l[g][ra], s.h[g][ra]);
  }
}

template <typename T>
__device__ __forceinline__ void fbfly(State &s, int ra, int rb, const T &Tb) {
#pragma unroll
  for (int g = 0; g < GP; ++g) {
    mul_any(s.l[g][rb], s.h[g][rb], Tb, s.l[g][ra], s.h[g][ra]);
    s.l[g][rb] ^= s.l[g][ra];
    s.h[g][rb] ^= s.h[g][ra];
  }
}

__device__ __forceinline__ void bxor(State &s, int ra, int rb) {  // b ^= a (no multiply)
#pragma unroll
  for (int g = 0; g < GP; ++g) {
    s.l[g][rb] ^= s.l[g][ra];
    s.h[g][rb] ^= s.h[g][ra];
  }
}

// stage-7 butterfly reading the IFFT coefficients c and writing s (stage 7
// touches every register, so the coset needs no copy of c)
template <typename T>
__device__ __forceinline__ void fbfly_from(State &s, const State &c, int ra, int rb, const T &Tb) {
  s.l[0][ra] = c.l[0][ra];
  s.h[0][ra] = c.h[0][ra];
  mul_any(c.l[0][rb], c.h[0][rb], Tb, s.l[0][ra], s.h[0][ra]);
  s.l[0][rb] = c.l[0][rb] ^ s.l[0][ra];
  s.h[0][rb] = c.h[0][rb] ^ s.h[0][ra];
}

// position held in register r by lane q (0..31) in each layout
__device__ __forceinline__ uint32_t posA(uint32_t q, int r) { return (q << 3) | uint32_t(r); }
__device__ __forceinline__ uint32_t posB(uint32_t q, int r) {
  return ((q >> 3) << 6) | (uint32_t(r) << 3) | (q & 7);
}
// ---- wave-private exchange -------------------------------------------------
// 8-byte cell u = pos*2 + inst mapped by a GF(2)-linear bijection M
// (found by search, scripts/search_swizzle.py) under which every layout's
// reads (32-lane groups) and writes (16-lane groups) are bank-conflict free.
// u = lane part XOR register part, so addr = M(lane part) ^ M(r part).
constexpr uint32_t kM[9] = {0b110011100, 0b1001101, 0b111110100, 0b110001111, 0b11110011,
                            0b101101010, 0b110000111, 0b111011000, 0b111100000};
__host__ __device__ constexpr uint32_t mswz(uint32_t u) {
  uint32_t a = 0;
  for (int i = 0; i < 9; ++i) a |= uint32_t(__builtin_popcount(kM[i] & u) & 1) << i;
  return a << 3;
}
// lane part / register part of u for each layout
__device__ __forceinline__ uint32_t ulaneA(uint32_t q, uint32_t inst) { return (q << 4) | inst; }
__device__ __forceinline__ uint32_t ulaneB(uint32_t q, uint32_t inst) {
  return ((q >> 3) << 7) | ((q & 7) << 1) | inst;
}
__device__ __forceinline__ uint32_t ulaneC(uint32_t q, uint32_t inst) { return (q << 1) | inst; }
__host__ __device__ constexpr uint32_t uregA(int r) { return uint32_t(r) << 1; }
__host__ __device__ constexpr uint32_t uregB(int r) { return uint32_t(r) << 4; }
__host__ __device__ constexpr uint32_t uregC(int r) {
  return (uint32_t(r & 3) << 7) | (uint32_t(r >> 2) << 6);
}

enum Layout { LA, LB, LC };

struct XBase {  // per-lane exchange base addresses
  uint32_t a, b, c;
};

template <Layout L>
__device__ __forceinline__ uint32_t xcell(const XBase &xb, int r) {
  if constexpr (L == LA) return xb.a ^ mswz(uregA(r));
  else if constexpr (L == LB) return xb.b ^ mswz(uregB(r));
  else return xb.c ^ mswz(uregC(r));
}

template <Layout FROM, Layout TO>
__device__ __forceinline__ void exchange(State &s, uint8_t *xch, const XBase &xb) {
#pragma unroll
  for (int r = 0; r < 8; ++r)
    *reinterpret_cast<uint2 *>(xch + xcell<FROM>(xb, r)) = make_uint2(s.l[0][r], s.h[0][r]);
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const uint2 v = *reinterpret_cast<const uint2 *>(xch + xcell<TO>(xb, r));
    s.l[0][r] = v.x;
    s.h[0][r] = v.y;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// byte-planar group (4 pieces) -> big-endian u16 x4 (pieces 0..3 in order)
__device__ __forceinline__ uint2 to_be(uint32_t l, uint32_t h) {
  return make_uint2(vperm(l, h, 0x05010400u), vperm(l, h, 0x07030602u));
}

// 16 payload bytes at any address, zero past `avail` (bytes valid from p):
// aligned dwords that each hold at least one wanted byte (so nothing outside
// the payload's allocation is touched), funnel-shifted by v_alignbyte
__device__ __forceinline__ uint4 load16_any(const uint8_t *p, uint64_t avail) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  if (avail >= 16 && (a & 15) == 0) return *reinterpret_cast<const uint4 *>(p);
  if (avail == 0) return make_uint4(0, 0, 0, 0);
  const uint32_t sh = uint32_t(a & 3), nb = avail < 16 ? uint32_t(avail) : 16u;
  const uint32_t *q = reinterpret_cast<const uint32_t *>(a & ~uintptr_t(3));
  uint32_t d[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) d[i] = uint32_t(4 * i) < sh + nb ? q[i] : 0u;
  uint32_t w[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    w[j] = __builtin_amdgcn_alignbyte(d[j + 1], d[j], sh);
    const uint32_t have = nb > uint32_t(4 * j) ? nb - uint32_t(4 * j) : 0u;  // valid bytes of word j
    if (have < 4) w[j] &= (1u << (8 * have)) - 1u;
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

}  // namespace
}  // namespace ecamd
