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

__host__ __device__ constexpr uint32_t raddr(uint32_t v) {
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

// tower images: stages >= SM hold subfield tables; SM =
// kNoTower: a symbol-coordinate image (every stage general)
constexpr int kNoTower = 64;
__device__ __forceinline__ void tab_at(const uint8_t *lds, uint32_t lin, SubTab &T) {
  T.t[4] = *reinterpret_cast<const uint32_t *>(lds + Tabs::kPlane + lin);
  const uint4 v = *reinterpret_cast<const uint4 *>(lds + lin);
  T.t[0] = v.x;
  T.t[1] = v.y;
  T.t[2] = v.z;
  T.t[3] = v.w;
}
template <bool SUBF>
struct TabSel {
  using type = Tab;
};
template <>
struct TabSel<true> {
  using type = SubTab;
};
template <int M, int SM>
using TabAt = typename TabSel<(M >= SM)>::type;

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
__device__ __forceinline__ void ib(S16 &s, int a, int b, const SubTab &T) {
  s.l[b] ^= s.l[a];
  s.h[b] ^= s.h[a];
  mul_acc_sub(s.l[b], s.h[b], T, s.l[a], s.h[a]);
}
__device__ __forceinline__ void fb(S16 &s, int a, int b, const SubTab &T) {
  mul_acc_sub(s.l[b], s.h[b], T, s.l[a], s.h[a]);
  s.l[b] ^= s.l[a];
  s.h[b] ^= s.h[a];
}

// radix-16 passes over position bits B0..B0+3 held in registers; lb = tlin of
// the lane part of the position.  The next block's table is requested one
// step ahead of its use.
template <int B0, int SM = kNoTower>
__device__ __forceinline__ void ipass4(S16 &s, const uint8_t *tabs, uint32_t lb) {
  Tab T[2];
  SubTab U[2];
  const auto fetch = [&](int t, int blk, int slot) __attribute__((always_inline)) {
    const uint32_t a = lb ^ tlin(skew_idx(uint32_t(blk) << B0, B0 + t));
    if (B0 + t >= SM) tab_at(tabs, a, U[slot]);
    else tab_at(tabs, a, T[slot]);
  };
  fetch(0, 0, 0);
  int k = 0;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int d = 1 << t;
#pragma unroll
    for (int blk = 0; blk < 16; blk += 2 * d, ++k) {
      const int nt = blk + 2 * d < 16 ? t : t + 1, nblk = blk + 2 * d < 16 ? blk + 2 * d : 0;
      if (nt < 4) fetch(nt, nblk, (k + 1) & 1);
#pragma unroll
      for (int i = 0; i < d; ++i) {
        if (B0 + t >= SM) ib(s, blk + i, blk + i + d, U[k & 1]);
        else ib(s, blk + i, blk + i + d, T[k & 1]);
      }
    }
  }
}

template <int B0, int SM = kNoTower>
__device__ __forceinline__ void fpass4(S16 &s, const uint8_t *tabs, uint32_t lb) {
  Tab T[2];
  SubTab U[2];
  const auto fetch = [&](int t, int blk, int slot) __attribute__((always_inline)) {
    const uint32_t a = lb ^ tlin(skew_idx(uint32_t(blk) << B0, B0 + t));
    if (B0 + t >= SM) tab_at(tabs, a, U[slot]);
    else tab_at(tabs, a, T[slot]);
  };
  fetch(3, 0, 0);
  int k = 0;
#pragma unroll
  for (int t = 3; t >= 0; --t) {
    const int d = 1 << t;
#pragma unroll
    for (int blk = 0; blk < 16; blk += 2 * d, ++k) {
      const int nt = blk + 2 * d < 16 ? t : t - 1, nblk = blk + 2 * d < 16 ? blk + 2 * d : 0;
      if (nt >= 0) fetch(nt, nblk, (k + 1) & 1);
#pragma unroll
      for (int i = 0; i < d; ++i) {
        if (B0 + t >= SM) fb(s, blk + i, blk + i + d, U[k & 1]);
        else fb(s, blk + i, blk + i + d, T[k & 1]);
      }
    }
  }
}

// layout C: stage 8 (skew depends on p9 = r bit 1), stage 9 (one skew)
template <int SM = kNoTower>
__device__ __forceinline__ void ipassC(S16 &s, const uint8_t *tabs) {
  TabAt<8, SM> Ta, Tb;
  TabAt<9, SM> Tc;
  tab_at(tabs, tlin(skew_idx(0, 8)), Ta);
  tab_at(tabs, tlin(skew_idx(1u << 9, 8)), Tb);
#pragma unroll
  for (int hi = 0; hi < 4; ++hi) ib(s, 4 * hi, 4 * hi + 1, Ta);
  tab_at(tabs, tlin(skew_idx(0, 9)), Tc);
#pragma unroll
  for (int hi = 0; hi < 4; ++hi) ib(s, 4 * hi + 2, 4 * hi + 3, Tb);
#pragma unroll
  for (int hi = 0; hi < 4; ++hi) {
    ib(s, 4 * hi, 4 * hi + 2, Tc);
    ib(s, 4 * hi + 1, 4 * hi + 3, Tc);
  }
}

template <int SM = kNoTower>
__device__ __forceinline__ void fpassC(S16 &s, const uint8_t *tabs) {
  TabAt<9, SM> Ta;
  TabAt<8, SM> Tb, Tc;
  tab_at(tabs, tlin(skew_idx(0, 9)), Ta);
  tab_at(tabs, tlin(skew_idx(0, 8)), Tb);
#pragma unroll
  for (int hi = 0; hi < 4; ++hi) {
    fb(s, 4 * hi, 4 * hi + 2, Ta);
    fb(s, 4 * hi + 1, 4 * hi + 3, Ta);
  }
  tab_at(tabs, tlin(skew_idx(1u << 9, 8)), Tc);
#pragma unroll
  for (int hi = 0; hi < 4; ++hi) fb(s, 4 * hi, 4 * hi + 1, Tb);
#pragma unroll
  for (int hi = 0; hi < 4; ++hi) fb(s, 4 * hi + 2, 4 * hi + 3, Tc);
}

// The same two passes for the transform at index 0, where a stage's block at
// j = d has skew skews[d - 1] = 0xFFFF (no multiply, additive_fft.hpp:99-141):
// stage 9 and stage 8's p9 = 0 block are b ^= a (IFFT) / b ^= a after an
// a ^= 0 (FFT).
__device__ __forceinline__ void bx(S16 &s, int a, int b) {  // b ^= a
  s.l[b] ^= s.l[a];
  s.h[b] ^= s.h[a];
}

template <int SM = kNoTower>
__device__ __forceinline__ void ipassC0(S16 &s, const uint8_t *tabs) {
  TabAt<8, SM> Tb;
  tab_at(tabs, tlin(skew_idx(1u << 9, 8)), Tb);
#pragma unroll
  for (int hi = 0; hi < 4; ++hi) bx(s, 4 * hi, 4 * hi + 1);
#pragma unroll
  for (int hi = 0; hi < 4; ++hi) ib(s, 4 * hi + 2, 4 * hi + 3, Tb);
#pragma unroll
  for (int hi = 0; hi < 4; ++hi) {
    bx(s, 4 * hi, 4 * hi + 2);
    bx(s, 4 * hi + 1, 4 * hi + 3);
  }
}

template <int SM = kNoTower>
__device__ __forceinline__ void fpassC0(S16 &s, const uint8_t *tabs) {
  TabAt<8, SM> Ta;
  tab_at(tabs, tlin(skew_idx(1u << 9, 8)), Ta);
#pragma unroll
  for (int hi = 0; hi < 4; ++hi) {
    bx(s, 4 * hi, 4 * hi + 2);
    bx(s, 4 * hi + 1, 4 * hi + 3);
  }
#pragma unroll
  for (int hi = 0; hi < 4; ++hi) bx(s, 4 * hi, 4 * hi + 1);
#pragma unroll
  for (int hi = 0; hi < 4; ++hi) fb(s, 4 * hi + 2, 4 * hi + 3, Ta);
}

__host__ __device__ constexpr uint32_t posA(uint32_t lane, int r) { return 16 * lane + uint32_t(r); }
__host__ __device__ constexpr uint32_t posB(uint32_t lane, int r) {
  return (lane & 15) | (uint32_t(r) << 4) | ((lane >> 4) << 8);
}
__host__ __device__ constexpr uint32_t posC(uint32_t lane, int r) {
  return lane | (uint32_t((r >> 2) & 3) << 6) | (uint32_t(r & 3) << 8);
}

enum Layout { LA, LB, LC };

template <Layout L>
__host__ __device__ constexpr uint32_t pos_of(uint32_t lane, int r) {
  if constexpr (L == LA) return posA(lane, r);
  else if constexpr (L == LB) return posB(lane, r);
  else return posC(lane, r);
}

// LDS address of position pos_of<X>(lane, r) in the wave's region `my`
// (8 KB aligned): raddr is GF(2)-linear and the lane and register parts of a
// position are disjoint, so it is (per-lane address) ^ (constant of r)
template <Layout X>
__device__ __forceinline__ uint32_t region_lane(const uint8_t *my, uint32_t lane) {
  return lds_addr(my) | raddr(pos_of<X>(lane, 0));
}
template <Layout X>
__device__ __forceinline__ uint32_t region_at(uint32_t lane_addr, int r) {
  return lane_addr ^ raddr(pos_of<X>(0, r));
}

// wave-private exchange of the 16 registers from layout FROM to layout TO
template <Layout FROM, Layout TO>
__device__ __forceinline__ void exchange(S16 &s, uint8_t *my, uint32_t lane) {
  asm volatile("" : "+v"(lane));  // addresses computed here, not hoisted and kept live
  const uint32_t af = region_lane<FROM>(my, lane);
#pragma unroll
  for (int r = 0; r < 16; ++r) lds_st2(region_at<FROM>(af, r), make_uint2(s.l[r], s.h[r]));
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
  const uint32_t at = region_lane<TO>(my, lane);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const uint2 x = lds_ld2(region_at<TO>(at, r));
    s.l[r] = x.x;
    s.h[r] = x.y;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// IFFT_1024 (inverse_afft, index = the tables' offset; INDEX0: the offset is
// 0): layout A in, C out
// SM: the table image's first subfield stage (tower images; kNoTower: none)
template <bool INDEX0 = false, int SM = kNoTower>
__device__ __forceinline__ void ifft1024(S16 &s, const uint8_t *tabs, uint8_t *my, uint32_t lane) {
  asm volatile("" : "+v"(lane));
  ipass4<0, SM>(s, tabs, tlin(16 * lane));
  exchange<LA, LB>(s, my, lane);
  ipass4<4, SM>(s, tabs, tlin((lane >> 4) << 8));
  exchange<LB, LC>(s, my, lane);
  if constexpr (INDEX0) ipassC0<SM>(s, tabs);
  else ipassC<SM>(s, tabs);
}

// FFT_1024 (afft): layout C in, A out
template <bool INDEX0 = false, int SM = kNoTower>
__device__ __forceinline__ void fft1024(S16 &s, const uint8_t *tabs, uint8_t *my, uint32_t lane) {
  asm volatile("" : "+v"(lane));
  if constexpr (INDEX0) fpassC0<SM>(s, tabs);
  else fpassC<SM>(s, tabs);
  exchange<LC, LB>(s, my, lane);
  fpass4<4, SM>(s, tabs, tlin((lane >> 4) << 8));
  exchange<LB, LA>(s, my, lane);
  fpass4<0, SM>(s, tabs, tlin(16 * lane));
}

// ---- cross-lane helpers, layout bit maps, closed-form derivative and the
// restricted FFT (reconstruct_gen, reconstruct_n4096)
__device__ __forceinline__ uint32_t dpp_up(uint32_t x, int b) {  // value of lane + 2^b (b < 4)
  switch (b) {
    case 0: return uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x101, 0xf, 0xf, true));
    case 1: return uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x102, 0xf, 0xf, true));
    case 2: return uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x104, 0xf, 0xf, true));
    default: return uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x108, 0xf, 0xf, true));
  }
}

// value of lane (lane + 2^b) for lanes whose bit b is 0 (others: don't care)
__device__ __forceinline__ uint32_t from_upper(uint32_t x, int b) {
  if (b < 4) return dpp_up(x, b);
  if (b == 4) {
    auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    return r[1];
  }
  auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  return r[1];
}

// position bit held by register bit t / lane bit u in each layout (tf1024.hpp)
template <Layout X>
__host__ __device__ constexpr int reg_pbit(int t) {
  if constexpr (X == LA) return t;
  else if constexpr (X == LB) return t + 4;
  else return t == 0 ? 8 : t == 1 ? 9 : t == 2 ? 6 : 7;
}
template <Layout X>
__host__ __device__ constexpr int lane_pbit(int u) {
  if constexpr (X == LB) return u < 4 ? u : u + 4;
  else if constexpr (X == LA) return u + 4;
  else return u;
}


// formal derivative (poly_encoder.hpp:195-215), closed form, in layout X, in
// place: registers in increasing order (register partners r | 2^t > r are
// still original), lane partners read the other lanes' original register r.
// Only registers with LIVE(r) are computed (the others keep their values, so
// they still read as original partners): before fft_restricted<X, L, KB> the
// registers that reach y < k, since its stages t >= KB pass y < k through.
template <Layout X, int L, int KB = L>
__device__ __forceinline__ void derivative(S16 &s, uint32_t lane);

// register r is still needed after the a-only stages above t (t = KB - 1: all)
template <Layout X, int L, int KB>
__host__ __device__ constexpr bool live_above(int r, int t);

template <Layout X, int L, int KB>
__device__ __forceinline__ void derivative(S16 &s, uint32_t lane) {
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    if (!live_above<X, L, KB>(r, KB - 1)) continue;
    uint32_t al = 0, ah = 0;
#pragma unroll
    for (int u = 0; u < 6; ++u) {
      if (lane_pbit<X>(u) >= L) continue;  // an instance bit
      const uint32_t m = ((lane >> u) & 1) ? 0u : 0xffffffffu;
      al ^= from_upper(s.l[r], u) & m;
      ah ^= from_upper(s.h[r], u) & m;
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
      if (reg_pbit<X>(t) < L && !(r & (1 << t))) {
        al ^= s.l[r | (1 << t)];
        ah ^= s.h[r | (1 << t)];
      }
    s.l[r] ^= al;
    s.h[r] ^= ah;
  }
}


// ---- FFT_n restricted to the outputs y < k = 2^KB (afft, additive_fft.hpp:121-141,
// index 0), from the layout the derivative ran in (X = C for n >= 512, B below):
//  * register-held stages t >= KB: only the side that reaches y < k is kept
//    (a ^= b * s), and that is the block at j = 2^t whose skew skews[2^t - 1]
//    is 0xFFFF (no multiply): these stages pass y < k through, nothing runs;
//  * register-held stages below KB are full butterflies on the live registers;
//  * the lane-held stages (p5..p0 in C, p3..p0 in B) run in registers after
//    swapping each lane bit with register bit SB (the one of p6 / p4, whose
//    stage is done) by DPP / v_permlane*_swap: no LDS exchange.
// Afterwards: SB = p0, lane bits 0.. = p1.., the other register bits unchanged.
template <Layout X>
__host__ __device__ constexpr int rbit_of(int p) {
  return reg_pbit<X>(0) == p ? 0 : reg_pbit<X>(1) == p ? 1 : reg_pbit<X>(2) == p ? 2
                                 : reg_pbit<X>(3) == p ? 3 : -1;
}
template <Layout X, int L, int KB>
__host__ __device__ constexpr bool live_above(int r, int t) {
  for (int p = (t + 1 > KB ? t + 1 : KB); p < L; ++p) {
    const int b = rbit_of<X>(p);
    if (b >= 0 && ((r >> b) & 1)) return false;
  }
  return true;
}
// local position bits held in register r (register bit skip excluded)
template <Layout X, int L>
__host__ __device__ constexpr uint32_t reg_pos(int r, int skip) {
  uint32_t v = 0;
  for (int b = 0; b < 4; ++b)
    if (b != skip && ((r >> b) & 1) && reg_pbit<X>(b) < L) v |= 1u << reg_pbit<X>(b);
  return v;
}
template <Layout X>
__host__ __device__ constexpr int swap_rbit() { return X == LC ? 2 : 0; }  // p6 / p4
template <Layout X>
__host__ __device__ constexpr int lane_stages() { return X == LC ? 6 : 4; }  // p0..p5 / p0..p3

// swap register bit (x: bit 0, y: bit 1) with lane bit b; hi = this lane's bit b
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

template <Layout X, int L, int KB, int SM = kNoTower>
__device__ __forceinline__ void fft_restricted(S16 &s, const uint8_t *tabs, uint32_t lane) {
  constexpr int F = X == LC ? 6 : 4;  // lowest register-held position bit
  constexpr int SB = swap_rbit<X>(), NL = lane_stages<X>();
  // register-held stages L-1 .. F (tables: wave-uniform, from the register bits above t)
#pragma unroll
  for (int t = (KB - 1 < L - 1 ? KB - 1 : L - 1); t >= F; --t) {
    const int b = rbit_of<X>(t);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (((r >> b) & 1) || !live_above<X, L, KB>(r, t)) continue;
      const uint32_t a = tlin(skew_idx(reg_pos<X, L>(r, -1), t));
      if (t >= SM) {
        SubTab T;
        tab_at(tabs, a, T);
        fb(s, r, r | (1 << b), T);
      } else {
        Tab T;
        tab_at(tabs, a, T);
        fb(s, r, r | (1 << b), T);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  // lane-held stages NL-1 .. 0: swap lane bit u into register bit SB, butterfly
#pragma unroll
  for (int u = NL - 1; u >= 0; --u) {
    uint32_t l = lane;
    asm volatile("" : "+v"(l));
    const bool hi = (l >> u) & 1;
    // bits above u now: p(u+1)..p(NL) in lane bits u..NL-1, the rest in registers
    const uint32_t lane_hi = ((l & ((1u << NL) - 1)) >> u) << (u + 1);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (((r >> SB) & 1) || !live_above<X, L, KB>(r & ~(1 << SB), KB - 1)) continue;
      const int r1 = r | (1 << SB);
      swap_bit(s.l[r], s.l[r1], u, hi);
      swap_bit(s.h[r], s.h[r1], u, hi);
      const uint32_t a = tlin(skew_idx((lane_hi | reg_pos<X, L>(r, SB)) & ((1u << L) - 1), u));
      if (u >= SM) {
        SubTab T;
        tab_at(tabs, a, T);
        fb(s, r, r1, T);
      } else {
        Tab T;
        tab_at(tabs, a, T);
        fb(s, r, r1, T);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}


// byte-planar group (4 pieces / columns) -> big-endian u16 x4
__device__ __forceinline__ uint2 to_be(uint32_t l, uint32_t h) {
  return make_uint2(vperm(l, h, 0x05010400u), vperm(l, h, 0x07030602u));
}

}  // namespace tf
}  // namespace ecamd
