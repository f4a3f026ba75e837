// dec_n1024_common.hpp — the n = 1024, k = 256 reconstruct's shared pieces
// (dec_n1024.hip: the 8-wave kernel and its packed form; dec_n1024x.hip: the
// 12-wave kernel): positions, the region swizzle, table addressing by skew
// slot, the radix-16 inverse pass, cross-lane helpers.
#pragma once

#include <hip/hip_runtime.h>

#include "ec_device.hpp"
#include "ec_kernels.hpp"

namespace ecamd {
namespace n1024 {

constexpr int N = 1024;
constexpr int K = 256;
using Tabs = LdsTabs<1024>;
constexpr int REG_BYTES = N * 8;  // one wave's group: 1024 x uint2


// region address of position v: 8-byte slots XOR-swizzled so that every
// access pattern used below (positions varying in bits 4-8, 0-3+8, 0-4) is
// bank-conflict free
__host__ __device__ constexpr uint32_t raddr(uint32_t v) {
  const uint32_t f = (v & 31) ^ ((v >> 4) & 31);
  return ((v >> 5) << 8) | (f << 3);
}

// raddr is GF(2)-linear in v, so a wave's region access for position
// (lane part) | (register part) is one v_xor of a per-lane LDS address with a
// compile-time constant (lds_addr / lds_ld2 / lds_st2, ec_device.hpp).  The
// region base (a multiple of 8 KB) has no bits in common with raddr (< 8 KB),
// so it folds into the per-lane address too.

__device__ __forceinline__ uint32_t skew_idx(uint32_t pos_a, int m) {
  const uint32_t d = 1u << m;
  return (pos_a & ~(2 * d - 1)) + d - 1;  // FFT index 0 (poly_encoder.hpp:180,183)
}

// skew index at stage 2 whose element equals the skew element of position
// pos_a at stage m (2 (pos_a >> (m + 1)), additive_fft.hpp:47-97 with the Cantor
// relabelling: skews[i] = log(((i + 1) >> ctz(i + 1)) - 1)): that element is
// < 256 iff the result is < 1024, and its image slot holds a subfield table
__device__ __forceinline__ uint32_t sub_alias(uint32_t pos_a, int m) {
  return ((pos_a >> (m + 1)) << 3) | 3u;
}

struct S16 {
  uint32_t l[16], h[16];
};

__device__ __forceinline__ void ib(S16 &s, int a, int b, const Tab &T) {
  s.l[b] ^= s.l[a];
  s.h[b] ^= s.h[a];
  mul_acc(s.l[b], s.h[b], T, s.l[a], s.h[a]);
}
__device__ __forceinline__ void ib(S16 &s, int a, int b, const SubTab &T) {
  s.l[b] ^= s.l[a];
  s.h[b] ^= s.h[a];
  mul_acc_sub(s.l[b], s.h[b], T, s.l[a], s.h[a]);
}

// GF(2)-linear part of the swizzled table address (LdsTabs::addr minus the
// plane term): tlin(a | b) = tlin(a) ^ tlin(b) for disjoint a, b, so a table
// address is a per-lane base XOR a wave-uniform value.
__host__ __device__ constexpr uint32_t tlin(uint32_t idx) {
  return ((idx >> 4) << 8) | (((idx ^ (idx >> 4) ^ (idx >> 8)) & 15) << 4);
}

// the tables are the first thing in the kernel's LDS (address 0: lds_tab_abs)
__device__ __forceinline__ void tab_at(const uint8_t *, uint32_t lin, Tab &T) {
  lds_tab_abs<Tabs::kPlane>(lin, T);
}
// the data runs in tower coordinates and the tables are tower
// image 0: stages >= tower_sub_min(0) = 2 hold subfield tables
__device__ __forceinline__ void tab_at(const uint8_t *, uint32_t lin, SubTab &T) {
  lds_subtab_abs<Tabs::kPlane>(lin, T);
}
constexpr int SUB = tower_sub_min(0);
// IFFT stage 1 with F9 tables (F9 image kind 0)
constexpr bool kF9 = true;
__device__ __forceinline__ void tab_at(const uint8_t *, uint32_t lin, F9Tab &T) {
  lds_f9tab_abs<Tabs::kPlane>(lin, T);
}
__device__ __forceinline__ void ib(S16 &s, int a, int b, const F9Tab &T) {
  s.l[b] ^= s.l[a];
  s.h[b] ^= s.h[a];
  mul_acc_f9(s.l[b], s.h[b], T, s.l[a], s.h[a]);
}

// inverse radix-16 pass over position bits b0..b0+3: pos(r) = lane part | (r << b0),
// lb = tlin(lane part).  15 tables (8 + 4 + 2 + 1), each requested one step
// ahead of its use so a table load is always in flight behind the multiplies.
template <int B0>
__device__ __forceinline__ void ipass4(S16 &s, const uint8_t *tabs, uint32_t lb) {
  Tab T[2];      // stages < SUB: general tables
  F9Tab F[2];    // stage 1 (kF9): F9 tables
  SubTab U[2];   // stages >= SUB: subfield tables
  const auto fetch = [&](int t, int blk, int slot) __attribute__((always_inline)) {
    const uint32_t a = lb ^ tlin(skew_idx(uint32_t(blk) << B0, B0 + t));
    if (B0 + t >= SUB) tab_at(tabs, a, U[slot]);
    else if (kF9 && B0 + t == 1) tab_at(tabs, a, F[slot]);
    else tab_at(tabs, a, T[slot]);
  };
  fetch(0, 0, 0);
  int k = 0;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int d = 1 << t;
#pragma unroll
    for (int blk = 0; blk < 16; blk += 2 * d, ++k) {  // one skew per block of 2d registers
      const int nt = blk + 2 * d < 16 ? t : t + 1, nblk = blk + 2 * d < 16 ? blk + 2 * d : 0;
      if (nt < 4) fetch(nt, nblk, (k + 1) & 1);
#pragma unroll
      for (int i = 0; i < d; ++i) {
        if (B0 + t >= SUB) ib(s, blk + i, blk + i + d, U[k & 1]);
        else if (kF9 && B0 + t == 1) ib(s, blk + i, blk + i + d, F[k & 1]);
        else ib(s, blk + i, blk + i + d, T[k & 1]);
      }
    }
  }
}

__device__ __forceinline__ uint32_t dpp_xor(uint32_t x, int ctrl_sel) {
  switch (ctrl_sel) {  // partner lane = lane + 2^b (lanes whose bit b is 0)
    case 0: return uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x101, 0xf, 0xf, true));
    case 1: return uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x102, 0xf, 0xf, true));
    case 2: return uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x104, 0xf, 0xf, true));
    default: return uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x108, 0xf, 0xf, true));
  }
}

// value of lane (lane + 2^b) for lanes whose bit b is 0 (others: don't care)
__device__ __forceinline__ uint32_t from_upper(uint32_t x, int b) {
  if (b < 4) return dpp_xor(x, b);
  if (b == 4) {
    auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    return r[1];
  }
  auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  return r[1];
}

// swap register bit (pair x: bit=0, y: bit=1) with lane bit b
__device__ __forceinline__ void swap_bit(uint32_t &x, uint32_t &y, int b, bool hi) {
  if (b == 4) {
    auto r = __builtin_amdgcn_permlane16_swap(x, y, false, false);
    x = r[0];
    y = r[1];
    return;
  }
  if (b == 5) {
    auto r = __builtin_amdgcn_permlane32_swap(x, y, false, false);
    x = r[0];
    y = r[1];
    return;
  }
  const uint32_t send = hi ? x : y;  // lane bit 1 sends x, lane bit 0 sends y
  uint32_t recv;
  switch (b) {
    case 0: recv = uint32_t(__builtin_amdgcn_update_dpp(0, int(send), 0xB1, 0xf, 0xf, true)); break;  // quad [1,0,3,2]
    case 1: recv = uint32_t(__builtin_amdgcn_update_dpp(0, int(send), 0x4E, 0xf, 0xf, true)); break;  // quad [2,3,0,1]
    case 2: {
      const uint32_t up = uint32_t(__builtin_amdgcn_update_dpp(0, int(send), 0x104, 0xf, 0xf, true));
      const uint32_t dn = uint32_t(__builtin_amdgcn_update_dpp(0, int(send), 0x114, 0xf, 0xf, true));
      recv = hi ? dn : up;
      break;
    }
    default: recv = uint32_t(__builtin_amdgcn_update_dpp(0, int(send), 0x128, 0xf, 0xf, true)); break;  // row_ror:8
  }
  if (hi) x = recv;
  else y = recv;
}

__device__ __forceinline__ uint32_t mul_index(uint32_t c) { return c == 65535u ? 0u : c; }

// 8 shard bytes at any even address, zero past `avail` (1..8 bytes valid
// from p): three dword loads, each clamped to the dword that holds the last
// wanted byte (so nothing past the row is touched), funnel-shifted by
// v_alignbyte; no branches
__device__ __forceinline__ uint2 load8_any(const uint8_t *p, uint32_t avail) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p), a0 = a & ~uintptr_t(3);
  const uintptr_t last = (a + avail - 1) & ~uintptr_t(3);
  const uint32_t sh = uint32_t(a & 3);
  const uint32_t d0 = *reinterpret_cast<const uint32_t *>(a0);
  const uint32_t d1 = *reinterpret_cast<const uint32_t *>(a0 + 4 < last ? a0 + 4 : last);
  const uint32_t d2 = *reinterpret_cast<const uint32_t *>(a0 + 8 < last ? a0 + 8 : last);
  const uint64_t keep = avail >= 8 ? ~0ull : (1ull << (8 * avail)) - 1;
  return make_uint2(__builtin_amdgcn_alignbyte(d1, d0, sh) & uint32_t(keep),
                    __builtin_amdgcn_alignbyte(d2, d1, sh) & uint32_t(keep >> 32));
}

// The two waves of a SIMD (w, w + 4) take turns at the higher issue priority
// (pass A: w + 4, pass B: w, pass C to the FFT: w + 4, output and gather:
// equal), so
// neither runs far ahead and then idles at the tile barrier while the other
// finishes alone (the arbiter otherwise favours the older wave throughout).
// A/B at B = 2048: 7.06 -> 7.01 ms; one fixed priority for the whole
// transform 7.08, four turns 7.09.
__device__ __forceinline__ void prio_lead(bool lead) {
  if (lead) __builtin_amdgcn_s_setprio(2);
  else __builtin_amdgcn_s_setprio(0);
}


}  // namespace n1024
}  // namespace ecamd
