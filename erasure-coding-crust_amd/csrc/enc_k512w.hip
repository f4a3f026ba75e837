// enc_k512w.hip — encode for k = 512, n = 2048 / 4096 (n_validators 1534..3069:
// the shapes just above a power of two), two 8-wave workgroups per CU.
//
// encode_k256w's model (enc_k256w.hip) at k = 512: per piece
// (1024 payload bytes = 512 symbols) IFFT_512 at index 0, then FFT_512 at each
// coset 512 j below n_validators (encodeLow, poly_encoder.hpp:217-240), radix-8
// register passes in tower coordinates, wave-private LDS exchanges.  What
// differs:
//  * one byte-planar group of 4 pieces per wave, its 512 positions over the
//    64 lanes x 8 registers; the position bit 8 is lane bit 5 (encode_k256w's
//    instance bit), so layouts A / B / C and their exchanges are encode_k256w's.
//    Stages 6-8 run in layout C' = C with register bit 2 (p5) and lane bit 5
//    (p8) swapped by v_permlane32_swap, where all three are register bits and
//    every element is wave-uniform;
//  * multiply tables: the compact image's subfield and F9 entries (elements
//    x < 256, 12 KB, resident) and, per coset, an extension image of the
//    general tables its stages 0..2 need (x >= 256: 20-35 KB, ec_kernels.hpp
//    kEImg512*), brought in by LDS-DMA while the previous coset's rows are
//    stored (its stage-0 tables alone are 256 distinct elements per coset:
//    all cosets' would not fit beside the regions, twice per CU);
//  * the tile is 32 pieces (8 waves x 4), each shard row a 64-B segment,
//    stored as 16 B per lane from two adjacent waves' regions.
//
// LDS per workgroup (80 KB, two per CU): extension stage 0 [0, 20480), the
// compact image's F9 and subfield areas at their own offsets [20480, 32768)
// (cimg.hpp ctab reads them unchanged), extension stages 1, 2 [32768, 48128),
// the tile slot, 8 wave regions of 4 KB [49152, 81920).
#include <hip/hip_runtime.h>

#include <type_traits>

#include "ec_device.hpp"
#include "ec_kernels.hpp"
#include "cimg.hpp"
#include "enc_k256_common.hpp"

namespace ecamd {
namespace {

constexpr int K = 512;
constexpr int WAVES = 8;
constexpr int THREADS = 64 * WAVES;
constexpr int TILE = 4 * WAVES;                          // pieces per tile
constexpr uint32_t BASE_LO = kCImgF9;                    // compact image bytes [20480, 32768)
constexpr uint32_t EXT[3] = {0, kCImgBytes, kCImgBytes + 5 * 2048};  // extension stages 0, 1, 2
constexpr uint32_t SLOT = EXT[2] + 5 * 1024;             // the next tile's index
constexpr uint32_t XCH0 = 49152;                         // the wave regions (4 KB aligned: XOR addressing)
constexpr uint32_t XCH_BYTES = 4096;
constexpr int LDS_BYTES = int(XCH0 + WAVES * XCH_BYTES);
static_assert(SLOT + 16 <= XCH0 && XCH0 % (2 * XCH_BYTES) == 0, "LDS map: region pairs XOR-addressed");
static_assert(EXT[0] + 5 * 4096 == BASE_LO && kEImg512Stage[1] == 20480 && kEImg512Stage[2] == 30720,
              "extension stage 0 ends where the compact image's F9 area starts");
static_assert(2 * LDS_BYTES <= 160 * 1024, "two workgroups per CU");

// extension image chunks (1 KB, one LDS-DMA wave-instruction each) coset j needs
__host__ __device__ constexpr uint32_t ext_chunks(uint32_t j) { return j == 1 ? 20 : j <= 3 ? 30 : 35; }

// Table kinds of a stage: the compact image's subfield / F9 entries (SubTab,
// F9Tab) or a general table of extension stage M (EG<M>).
template <int M>
struct EG {};
template <typename K_>
struct TabOf {
  using type = K_;
};
template <int M>
struct TabOf<EG<M>> {
  using type = Tab;
};

// table of element x = lane part ^ block part r ^ uniform part u (each the
// cimg_lin of its bits): compact-image kinds at their element address,
// extension tables at the coset-local one (u dropped: the coset's offset bits)
template <typename K_>
__device__ __forceinline__ void ftab(uint32_t lt, uint32_t r, uint32_t u, typename TabOf<K_>::type &T) {
  if constexpr (std::is_same_v<K_, SubTab> || std::is_same_v<K_, F9Tab>) {
    ctab(lt, r ^ u, T);
  } else {
    constexpr int M = [] {
      if constexpr (std::is_same_v<K_, EG<0>>) return 0;
      else if constexpr (std::is_same_v<K_, EG<1>>) return 1;
      else return 2;
    }();
    const uint32_t a = lt ^ r;
#pragma unroll
    for (int q = 4; q >= 0; --q) {
      const v4u v = lds_r128(a + EXT[M] + uint32_t(q) * (4096u >> M));
      T.t[4 * q] = v.x;
      T.t[4 * q + 1] = v.y;
      T.t[4 * q + 2] = v.z;
      T.t[4 * q + 3] = v.w;
    }
  }
}

// IFFT stage-0 table of element x = 4 lane + rr < 256 (lane part lt =
// cimg_lin(4 lane)): subfield for lanes 0-31 (p8 = 0), F9 for lanes 32-63,
// both read as an F9 table (gf_field.cpp f9_tab: a subfield c0 is (c0, 0, c0,
// mask 0)); the subfield area's plane-1 slots hold (w4, 0, 0, 0)
__device__ __forceinline__ void mixtab(uint32_t lt, uint32_t r, bool hi, F9Tab &T) {
  const uint32_t a = lt ^ r ^ (hi ? cimg_lin(128) : 0u);  // entry 4 (lane & 31) + rr of either area
  const uint32_t p0 = a + (hi ? kCImgF9 : kCImgSub0), p1 = a + (hi ? kCImgF9 + kCImgF9Plane : kCImgSub1);
  const v4u v3 = lds_r128(a + kCImgF9 + 3 * kCImgF9Plane), v2 = lds_r128(a + kCImgF9 + 2 * kCImgF9Plane);
  const v4u v1 = lds_r128(p1), v0 = lds_r128(p0);
  T.t[0] = v0.x;
  T.t[1] = v0.y;
  T.t[2] = v0.z;
  T.t[3] = v0.w;
  T.t[4] = v1.x;
  T.t[5] = v1.y;
  T.t[6] = v1.z;
  T.t[7] = v1.w;
  T.t[8] = hi ? v2.x : 0u;
  T.t[9] = hi ? v2.y : 0u;
  T.t[10] = hi ? v2.z : v0.x;
  T.t[11] = hi ? v2.w : v0.y;
  T.t[12] = hi ? v3.x : v0.z;
  T.t[13] = hi ? v3.y : v0.w;
  T.t[14] = hi ? v3.z : v1.x;
  T.t[15] = hi ? v3.w : 0u;
}

struct XLanes {
  uint32_t l0, l1, l2;
};
// lane parts of a radix-8 pass over position bits B0..B0+2 (enc_k256w.hip)
template <int B0>
__device__ __forceinline__ XLanes xlanes(uint32_t base) {
  return {cimg_lin(base >> (B0 + 1)), cimg_lin(base >> (B0 + 2)), cimg_lin(base >> (B0 + 3))};
}

// IFFT pass A (stages 0-2, index 0), base = 8 lane
__device__ __forceinline__ void ipassA(State &s, uint32_t base, bool hi) {
  const XLanes x = xlanes<0>(base);
  F9Tab Ta0, Tb0;
  SubTab Ta1, Tb1, Ta2;
  mixtab(x.l0, cimg_lin(0), hi, Ta0);
  mixtab(x.l0, cimg_lin(1), hi, Tb0);
  ibfly(s, 0, 1, Ta0);
  mixtab(x.l0, cimg_lin(2), hi, Ta0);
  ibfly(s, 2, 3, Tb0);
  mixtab(x.l0, cimg_lin(3), hi, Tb0);
  ibfly(s, 4, 5, Ta0);
  ctab(x.l1, cimg_lin(0), Ta1);
  ibfly(s, 6, 7, Tb0);
  ctab(x.l1, cimg_lin(1), Tb1);
  ibfly(s, 0, 2, Ta1);
  ibfly(s, 1, 3, Ta1);
  ctab(x.l2, cimg_lin(0), Ta2);
  ibfly(s, 4, 6, Tb1);
  ibfly(s, 5, 7, Tb1);
#pragma unroll
  for (int r = 0; r < 4; ++r) ibfly(s, r, r + 4, Ta2);
}

// IFFT pass B (stages 3-5, index 0): every element < 128 (subfield)
__device__ __forceinline__ void ipassB(State &s, uint32_t base) {
  const XLanes x = xlanes<3>(base);
  SubTab Ta0, Tb0, Ta1, Tb1, Ta2;
  ctab(x.l0, cimg_lin(0), Ta0);
  ctab(x.l0, cimg_lin(1), Tb0);
  ibfly(s, 0, 1, Ta0);
  ctab(x.l0, cimg_lin(2), Ta0);
  ibfly(s, 2, 3, Tb0);
  ctab(x.l0, cimg_lin(3), Tb0);
  ibfly(s, 4, 5, Ta0);
  ctab(x.l1, cimg_lin(0), Ta1);
  ibfly(s, 6, 7, Tb0);
  ctab(x.l1, cimg_lin(1), Tb1);
  ibfly(s, 0, 2, Ta1);
  ibfly(s, 1, 3, Ta1);
  ctab(x.l2, cimg_lin(0), Ta2);
  ibfly(s, 4, 6, Tb1);
  ibfly(s, 5, 7, Tb1);
#pragma unroll
  for (int r = 0; r < 4; ++r) ibfly(s, r, r + 4, Ta2);
}

// layout C' (register bit 0 = p6, bit 1 = p7, bit 2 = p8): IFFT stages 6-8 at
// index 0, elements x = pos >> (m + 1) uniform: stage 6 block rr (p7 + 2 p8)
// x = rr, stage 7 block p8 x = p8, stage 8 x = 0; x = 0 is b ^= a only (the
// skew 0xFFFF of additive_fft.hpp:110-112)
__device__ __forceinline__ void ipassC9(State &s) {
  SubTab T1, T2;
  ctab(0u, cimg_lin(1), T1);
  ctab(0u, cimg_lin(2), T2);
  bxor(s, 0, 1);
  ibfly(s, 2, 3, T1);
  ibfly(s, 4, 5, T2);
  ctab(0u, cimg_lin(3), T2);
  ibfly(s, 6, 7, T2);
  bxor(s, 0, 2);
  bxor(s, 1, 3);
  ibfly(s, 4, 6, T1);
  ibfly(s, 5, 7, T1);
#pragma unroll
  for (int r = 0; r < 4; ++r) bxor(s, r, r + 4);
}

// FFT stages 8, 7, 6 at index off (layout C'), reading the IFFT coefficients
// c and writing s: stage 8 x = off >> 9, stage 7 x = off >> 8 | p8, stage 6
// x = off >> 7 | (p7 + 2 p8); all subfield (x < 32)
__device__ __forceinline__ void fpassC9(State &s, const State &c, uint32_t off) {
  const uint32_t u0 = cimg_lin(off >> 7), u1 = cimg_lin(off >> 8), u2 = cimg_lin(off >> 9);
  SubTab Ta2, Ta1, Tb1, Ta0, Tb0;
  ctab(0u, u2, Ta2);
  ctab(0u, u1, Tb1);
#pragma unroll
  for (int r = 0; r < 4; ++r) fbfly_from(s, c, r, r + 4, Ta2);
  ctab(0u, u1 ^ cimg_lin(1), Ta1);
  fbfly(s, 0, 2, Tb1);
  fbfly(s, 1, 3, Tb1);
  ctab(0u, u0, Tb0);
  fbfly(s, 4, 6, Ta1);
  fbfly(s, 5, 7, Ta1);
  ctab(0u, u0 ^ cimg_lin(1), Ta0);
  fbfly(s, 0, 1, Tb0);
  ctab(0u, u0 ^ cimg_lin(2), Tb0);
  fbfly(s, 2, 3, Ta0);
  ctab(0u, u0 ^ cimg_lin(3), Ta0);
  fbfly(s, 4, 5, Tb0);
  fbfly(s, 6, 7, Ta0);
}

// C <-> C': register bit 2 and lane bit 5 swapped (registers r, r + 4)
__device__ __forceinline__ void swap_c(State &s) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    auto l = __builtin_amdgcn_permlane32_swap(s.l[0][r], s.l[0][r + 4], false, false);
    auto h = __builtin_amdgcn_permlane32_swap(s.h[0][r], s.h[0][r + 4], false, false);
    s.l[0][r] = l[0];
    s.l[0][r + 4] = l[1];
    s.h[0][r] = h[0];
    s.h[0][r + 4] = h[1];
  }
}

// forward radix-8 pass at index off over position bits B0..B0+2: stages B0+2,
// B0+1, B0 with table kinds K2, K1, K0 (the elements' kinds, known per coset)
template <int B0, typename K2, typename K1, typename K0>
__device__ __forceinline__ void fpass(State &s, uint32_t base, uint32_t off) {
  const XLanes x = xlanes<B0>(base);
  const uint32_t u0 = cimg_lin(off >> (B0 + 1)), u1 = cimg_lin(off >> (B0 + 2)), u2 = cimg_lin(off >> (B0 + 3));
  typename TabOf<K2>::type Ta2;
  typename TabOf<K1>::type Ta1, Tb1;
  typename TabOf<K0>::type Ta0, Tb0;
  ftab<K2>(x.l2, 0u, u2, Ta2);
  ftab<K1>(x.l1, 0u, u1, Tb1);
#pragma unroll
  for (int r = 0; r < 4; ++r) fbfly(s, r, r + 4, Ta2);
  ftab<K1>(x.l1, cimg_lin(1), u1, Ta1);
  fbfly(s, 0, 2, Tb1);
  fbfly(s, 1, 3, Tb1);
  ftab<K0>(x.l0, 0u, u0, Tb0);
  fbfly(s, 4, 6, Ta1);
  fbfly(s, 5, 7, Ta1);
  ftab<K0>(x.l0, cimg_lin(1), u0, Ta0);
  fbfly(s, 0, 1, Tb0);
  ftab<K0>(x.l0, cimg_lin(2), u0, Tb0);
  fbfly(s, 2, 3, Ta0);
  ftab<K0>(x.l0, cimg_lin(3), u0, Ta0);
  fbfly(s, 4, 5, Tb0);
  fbfly(s, 6, 7, Ta0);
}

// wave-private exchange (enc_k256_common.hpp exchange) at the wave's region
// folded into the lane bases xb (bits >= 12): the bases are laundered here, so
// the 16 cell addresses are formed at the exchange (one XOR each) instead of
// being hoisted out of the tile loop and kept live (spilled) across it
template <Layout FROM, Layout TO>
__device__ __forceinline__ void xchg(State &s, XBase xb) {
  asm volatile("" : "+v"(xb.a), "+v"(xb.b), "+v"(xb.c));
#pragma unroll
  for (int r = 0; r < 8; ++r) lds_st2(xcell<FROM>(xb, r), make_uint2(s.l[0][r], s.h[0][r]));
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const uint2 v = lds_ld2(xcell<TO>(xb, r));
    s.l[0][r] = v.x;
    s.h[0][r] = v.y;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// ---- own-region staging: wave w stages its 4 pieces x 512 rows in its own
// 4 KB region, 8 B per row: row v at ((v >> 5) << 8) | 8 ((v ^ (v >> 5) ^
// 8 (w >> 1)) & 31).  Layout-A writes (rows 8 lane + r) and the store reads
// (8 rows x the 4 chunk pairs of regions (2c, 2c + 1) per 32 lanes) touch 32
// distinct 8-B slots of one 256-B block.
__host__ __device__ constexpr uint32_t soff(uint32_t v, uint32_t w) {
  return ((v >> 5) << 8) | ((((v ^ (v >> 5)) ^ ((w >> 1) << 3)) & 31) << 3);
}

__device__ __forceinline__ void stage_own(const State &s, uint32_t lane, uint32_t wave) {
  const uint32_t a = XCH0 + wave * XCH_BYTES + soff(8 * lane, wave);
#pragma unroll
  for (int r = 0; r < 8; ++r) lds_st2(a ^ soff(uint32_t(r), 0), to_be(s.l[0][r], s.h[0][r]));
}

// all waves: rows [s0, s0 + 512) from the 8 regions -> shards.  Lane = (row
// in 16, chunk c = pieces 8c..8c+7 = regions 2c, 2c + 1); row v = it * 128 +
// wave * 16 + lane / 4.  Fast path (uniform): 16-B aligned rows, the whole tile
// inside the payload, all 512 rows below n_validators -- 4 streaming 16-B
// stores per lane.
__device__ __forceinline__ bool store_fast(const uint8_t *SH, uint64_t sstride, uint32_t s0, int nv,
                                           uint64_t piece0, uint64_t npieces) {
  return ((sstride | reinterpret_cast<uintptr_t>(SH)) & 15) == 0 && piece0 + TILE <= npieces &&
         int(s0) + K <= nv;
}

template <typename Then>
__device__ __forceinline__ void store_own(uint8_t *SH, uint64_t sstride, uint32_t s0, int nv,
                                          uint64_t piece0, uint64_t npieces, uint32_t wave,
                                          uint32_t lane, Then &&then) {
  asm volatile("" : "+v"(lane));  // recomputed here, not kept live across the FFTs
  const uint32_t c = lane & 3;
  const uint32_t v0 = wave * 16 + (lane >> 2);
  const uint32_t ra = XCH0 + 2 * c * XCH_BYTES + soff(v0, 2 * c);  // soff(v, 2c) == soff(v, 2c + 1)
  if (store_fast(SH, sstride, s0, nv, piece0, npieces)) {
    uint8_t *dst = SH + uint64_t(s0 + v0) * sstride + 2 * (piece0 + 8 * c);
    const uint64_t dstep = uint64_t(16 * WAVES) * sstride;
#pragma unroll
    for (int it = 0; it < K / (16 * WAVES); ++it) {  // soff is GF(2)-linear in v = it * 128 | v0
      const uint32_t o = soff(uint32_t(it) * 16 * WAVES, 0);
      const uint2 x = lds_ld2(ra ^ o), y = lds_ld2((ra + XCH_BYTES) ^ o);
      __builtin_nontemporal_store(v4u{x.x, x.y, y.x, y.y}, reinterpret_cast<v4u *>(dst + it * dstep));
    }
    then();
    asm volatile("; store_own fast path end" ::: "memory");
    return;
  }
  const uint64_t p = piece0 + 8 * c;
  const bool wide = ((sstride | reinterpret_cast<uintptr_t>(SH)) & 15) == 0;
#pragma unroll
  for (int it = 0; it < K / (16 * WAVES); ++it) {
    const uint32_t v = uint32_t(it) * 16 * WAVES + v0;
    const uint32_t o = soff(uint32_t(it) * 16 * WAVES, 0);
    const uint2 x = lds_ld2(ra ^ o), y = lds_ld2((ra + XCH_BYTES) ^ o);
    const uint32_t shard = s0 + v;
    if (int(shard) >= nv) continue;
    uint8_t *dst = SH + uint64_t(shard) * sstride + 2 * p;
    const uint32_t w[4] = {x.x, x.y, y.x, y.y};
    if (p + 8 <= npieces) {
      if (wide) {
        *reinterpret_cast<v4u *>(dst) = v4u{w[0], w[1], w[2], w[3]};
      } else {
        reinterpret_cast<uint2 *>(dst)[0] = make_uint2(w[0], w[1]);
        reinterpret_cast<uint2 *>(dst)[1] = make_uint2(w[2], w[3]);
      }
    } else if (p < npieces) {
      for (uint64_t e = 0; e < npieces - p; ++e)
        *reinterpret_cast<uint16_t *>(dst + 2 * e) = uint16_t(w[e >> 1] >> (16 * (e & 1)));
    }
  }
  then();
  asm volatile("; store_own slow path end" ::: "memory");
}

// 4 x 16 payload bytes (4 pieces, positions 8 lane .. 8 lane + 7) ->
// byte-planar State (enc_k256w.hip to_state)
__device__ __forceinline__ void to_state(const v4u (&d)[4], State &s) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t D0 = d[0][j], D1 = d[1][j], D2 = d[2][j], D3 = d[3][j];
    const uint32_t t0 = vperm(D1, D0, 0x05010400u), t1 = vperm(D1, D0, 0x07030602u);
    const uint32_t u0 = vperm(D3, D2, 0x05010400u), u1 = vperm(D3, D2, 0x07030602u);
    s.h[0][2 * j] = vperm(u0, t0, 0x05040100u);
    s.l[0][2 * j] = vperm(u0, t0, 0x07060302u);
    s.h[0][2 * j + 1] = vperm(u1, t1, 0x05040100u);
    s.l[0][2 * j + 1] = vperm(u1, t1, 0x07060302u);
  }
}

// coset j's extension image -> LDS by LDS-DMA, chunk i (1 KB) by wave i % 8:
// chunks 0..19 = stage 0, 20..34 = stages 1, 2 (ec_kernels.hpp kEImg512Stage)
__device__ __forceinline__ void dma_ext(const uint8_t *eimg, uint32_t j, uint32_t wave, uint32_t lane) {
  const uint8_t *src = eimg + (j - 1) * kEImg512Bytes + 16 * lane;
  const uint32_t n = ext_chunks(j);
  for (uint32_t i = wave; i < n; i += WAVES)
    lds_dma16(i < 20 ? EXT[0] + 1024 * i : EXT[1] + 1024 * (i - 20), src + 1024 * i);
}

}  // namespace

__global__ void __launch_bounds__(THREADS, 4) encode_k512w(const uint8_t *__restrict__ payloads,
                                                           uint64_t plen, uint64_t pstride,
                                                           uint8_t *__restrict__ shards, uint64_t slen,
                                                           uint64_t sstride, int nv, uint32_t batch,
                                                           const uint8_t *__restrict__ cimg,
                                                           const uint8_t *__restrict__ eimg,
                                                           uint32_t *__restrict__ tick) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const uint32_t tid0 = threadIdx.x;
  auto *slot = reinterpret_cast<__attribute__((address_space(3))) volatile uint32_t *>(uintptr_t(SLOT));
  // this workgroup's first tile; without a counter a static grid stride
  if (tid0 == 0) *slot = tick ? atomicAdd(tick, 1u) : blockIdx.x;
  {  // the compact image's F9 + subfield areas (12 KB, 768 chunks of 16 B)
    constexpr uint32_t c0 = BASE_LO / 16, n = (kCImgBytes - BASE_LO) / 16;
    const v4u a = reinterpret_cast<const v4u *>(cimg)[c0 + tid0];
    v4u b = v4u{0, 0, 0, 0};
    if (tid0 + THREADS < n) b = reinterpret_cast<const v4u *>(cimg)[c0 + THREADS + tid0];
    reinterpret_cast<v4u *>(lds)[c0 + tid0] = a;
    if (tid0 + THREADS < n) reinterpret_cast<v4u *>(lds)[c0 + THREADS + tid0] = b;
  }
  __syncthreads();

  const uint64_t npieces = slen / 2;
  const uint32_t tiles_pp = uint32_t((npieces + TILE - 1) / TILE);
  const uint32_t total = tiles_pp * batch;  // < 2^32 (launch_encode_k512w)
  const uint32_t wave_s = __builtin_amdgcn_readfirstlane(tid0 >> 6);
  // cosets 512 j, j = 1..J, below n_validators (nv <= n: launch_encode_k512w)
  const uint32_t J = uint32_t(nv - 1) / K;
  // Dynamic schedule (enc_k256w.hip): thread 0 takes tile t + 1 at the start
  // of tile t and publishes it in the slot after the systematic stores; every
  // wave reads it in the last coset, after further barriers; the slot is
  // rewritten only after the next tile's second barrier.
  uint32_t cur = __builtin_amdgcn_readfirstlane(*slot);

  // This lane's 4 x 16 payload bytes of tile (b, i): pieces i * TILE + 4 wave
  // + u, bytes 16 lane .. 16 lane + 15 of each, zero past plen; issued in the
  // previous tile's last coset, turned into the next State after its stores.
  v4u d[4];
  State nxt;
  const auto fetch = [&](uint64_t fb, uint64_t fi) __attribute__((always_inline)) {
    const uint8_t *FP = payloads + fb * pstride;
    const uint64_t pw = fi * TILE + 4 * wave_s;  // this wave's first piece (uniform)
    uint32_t flane = tid0;
    asm volatile("" : "+v"(flane));
    flane &= 63;
    if ((pw + 4) * 2 * K <= plen) {
      const uint8_t *src = FP + pw * 2 * K + 16 * flane;
#pragma unroll
      for (int u = 0; u < 4; ++u) d[u] = *reinterpret_cast<const v4u *>(src + u * 2 * K);
    } else if (pw < npieces) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint64_t off = (pw + u) * 2 * K + 16 * flane;
        uint32_t w[4] = {0, 0, 0, 0};
        if (off + 16 <= plen) {
          const v4u x = *reinterpret_cast<const v4u *>(FP + off);
          w[0] = x.x;
          w[1] = x.y;
          w[2] = x.z;
          w[3] = x.w;
        } else {
          for (uint64_t e = off; e < plen && e < off + 16; ++e)
            w[(e - off) >> 2] |= uint32_t(FP[e]) << (8 * ((e - off) & 3));
        }
        d[u] = v4u{w[0], w[1], w[2], w[3]};
      }
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) d[u] = v4u{0, 0, 0, 0};
    }
  };
  if (cur < total) {
    fetch(cur / tiles_pp, cur % tiles_pp);
    to_state(d, nxt);
  }

  while (cur < total) {
    uint32_t tid = tid0;
    asm volatile("" : "+v"(tid));
    const uint32_t lane = tid & 63, wave = tid >> 6;
    const uint32_t inst = lane >> 5, q = lane & 31;
    const bool hi = inst != 0;  // p8 in layouts A, B, C
    const uint32_t reg0 = XCH0 + wave * XCH_BYTES;  // this wave's region (bits >= 12)
    XBase xb;
    xb.a = reg0 | mswz(ulaneA(q, inst));
    xb.b = reg0 | mswz(ulaneB(q, inst));
    xb.c = reg0 | mswz(ulaneC(q, inst));
    const uint64_t b = cur / tiles_pp, piece0 = uint64_t(cur % tiles_pp) * TILE;
    uint32_t taken = 0;
    if (tid0 == 0) taken = tick ? atomicAdd(tick, 1u) : cur + gridDim.x;
    uint32_t next = 0;
    uint8_t *SH = shards + b * uint64_t(nv) * sstride;
    // every store phase of this tile takes the fast path (4 stores per lane)
    // or none does (rows 512 j < n_validators for j <= J)
    const bool fast = store_fast(SH, sstride, 0, nv, piece0, npieces);
    const auto fetch_next = [&]() __attribute__((always_inline)) {
      next = __builtin_amdgcn_readfirstlane(*slot);
      fetch(next < total ? next / tiles_pp : 0, next < total ? next % tiles_pp : tiles_pp);
    };
    const auto rsync = [&]() __attribute__((always_inline)) { lds_barrier(); };
    // coset j's extension image landed in every wave, then a barrier.  Coset
    // 1's was issued after the systematic stores (nothing after it), coset
    // j's after the barrier that precedes coset j - 1's store phase (4 stores
    // per lane after it on the fast path)
    const auto ext_ready = [&](uint32_t j) __attribute__((always_inline)) {
      if (j > 1 && fast) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      rsync();
    };
    const auto store = [&](uint32_t s0, bool last) __attribute__((always_inline)) {
      __builtin_amdgcn_s_setprio(1);
      if (last)
        store_own(SH, sstride, s0, nv, piece0, npieces, wave_s, lane,
                  [&]() __attribute__((always_inline)) { to_state(d, nxt); });
      else
        store_own(SH, sstride, s0, nv, piece0, npieces, wave_s, lane, [] {});
      __builtin_amdgcn_s_setprio(0);
    };
    const auto store_sys = [&]() __attribute__((always_inline)) {
      __builtin_amdgcn_s_setprio(1);
      store_own(SH, sstride, 0, nv, piece0, npieces, wave_s, lane, [&]() __attribute__((always_inline)) {
        if (tid0 == 0) *slot = taken;
      });
      __builtin_amdgcn_s_setprio(0);
    };
    // coset 1's extension image, after the systematic stores (their tile-slot
    // write waits for thread 0's ticket: a DMA issued before them would be
    // waited for with it): the last tile's last coset is past its tables
    // (every wave passed that coset's rows-staged barrier)
    const auto store_sys_dma = [&]() __attribute__((always_inline)) {
      store_sys();
      dma_ext(eimg, 1, wave_s, lane);
    };

    // a wave none of whose 4 pieces exist (the payload's last, partial tile)
    // takes part only in the barriers, the DMAs and the row stores (uniform)
    if (piece0 + 4 * wave_s >= npieces) {
      rsync();  // tile start
      rsync();  // systematic rows staged
      store_sys_dma();
      rsync();  // after IFFT pass A
      for (uint32_t j = 1;; ++j) {
        ext_ready(j);
        if (j == J) {
          fetch_next();
          rsync();  // rows staged
          store(K * j, true);
          break;
        }
        rsync();  // rows staged
        dma_ext(eimg, j + 1, wave_s, lane);
        store(K * j, false);
        __builtin_amdgcn_sched_barrier(0);
      }
      cur = next;
      continue;
    }

    State s = nxt;
    // ---- systematic shards 0..511 = the data symbols (poly_encoder.hpp:239)
    rsync();  // the other waves are done reading the regions (last tile)
    stage_own(s, lane, wave);
    rsync();
    store_sys_dma();
    __builtin_amdgcn_sched_barrier(0);
    {  // into tower coordinates
      const TowerK tk = tower_k();
#pragma unroll
      for (int r = 0; r < 8; ++r) s.l[0][r] = tower_lo(s.l[0][r], s.h[0][r], tk);
    }

    // ---- IFFT_512 (index 0): passes A (bits 0-2), B (3-5), C' (6-8)
    const uint32_t baseA = 8 * lane, baseB = (inst << 8) | posB(q, 0);
    ipassA(s, baseA, hi);
    rsync();  // systematic rows read out of the regions
    xchg<LA, LB>(s, xb);
    ipassB(s, baseB);
    xchg<LB, LC>(s, xb);
    swap_c(s);
    ipassC9(s);
    State coef = s;

    // ---- FFT_512 at each coset 512 j (encodeLow, poly_encoder.hpp:229-237).
    // Kinds by coset (x = (pos + off) >> (m + 1), ec_kernels.hpp): stage 3
    // subfield for j <= 3, F9 above; stage 2 subfield (j = 1), F9 (2, 3),
    // extension (4..7); stage 1 F9 (j = 1), extension above; stage 0
    // extension; stages 4-8 subfield.
    const auto coset = [&](auto k3, auto k2, auto k1, const uint32_t j) __attribute__((always_inline)) {
      using K3 = decltype(k3);
      using K2 = decltype(k2);
      using K1 = decltype(k1);
      const uint32_t off = K * j;
      // lane bases laundered per coset: the table addresses derived from them
      // are formed in the passes, not hoisted out of the coset loop (spilled)
      uint32_t bA = baseA, bB = baseB;
      asm volatile("" : "+v"(bA), "+v"(bB));
#pragma unroll
      for (int r = 0; r < 8; ++r) asm volatile("" : "+v"(coef.l[0][r]), "+v"(coef.h[0][r]));
      fpassC9(s, coef, off);
      swap_c(s);
      ext_ready(j);  // + the previous coset's rows read out of the regions
      xchg<LC, LB>(s, xb);
      fpass<3, SubTab, SubTab, K3>(s, bB, off);
      xchg<LB, LA>(s, xb);
      fpass<0, K2, K1, EG<0>>(s, bA, off);
      {  // back to symbol coordinates
        const TowerK tk = tower_k();
#pragma unroll
        for (int r = 0; r < 8; ++r) s.l[0][r] = tower_lo(s.l[0][r], s.h[0][r], tk);
      }
      stage_own(s, lane, wave);
    };
    // the cosets in a loop (three bodies, by table kinds); the last one leaves
    // it, so the next tile's payload (d, nxt) is live in that one only
    for (uint32_t j = 1;; ++j) {
      if (j == 1) coset(SubTab(), SubTab(), F9Tab(), j);
      else if (j <= 3) coset(SubTab(), F9Tab(), EG<1>(), j);
      else coset(F9Tab(), EG<2>(), EG<1>(), j);
      if (j == J) {
        fetch_next();  // coef and s are dead here
        rsync();       // rows staged
        store(K * j, true);
        break;
      }
      rsync();  // rows staged; every wave is past this coset's tables
      dma_ext(eimg, j + 1, wave_s, lane);
      store(K * j, false);
      __builtin_amdgcn_sched_barrier(0);
    }
    cur = next;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA outlives the workgroup
}

bool k512w_applicable(const CodeParams &p) { return p.k == 512 && (p.n == 2048 || p.n == 4096); }

size_t k512w_scratch_bytes(const CodeParams &p) { return k512w_applicable(p) ? 256 : 0; }

hipError_t launch_encode_k512w(const CodeParams &p, const DevTables &t, const uint8_t *d_payloads,
                               size_t plen, size_t pstride, size_t batch, uint8_t *d_shards,
                               size_t sstride, void *scratch, hipStream_t s) {
  int cus = 0;
  if (!t.cimg || !t.eimg512) return hipErrorInvalidValue;
  if (const hipError_t e = prepare_kernel(reinterpret_cast<const void *>(&encode_k512w), LDS_BYTES, &cus);
      e != hipSuccess)
    return e;
  if (!k512w_applicable(p) || p.nv <= uint32_t(K) || p.nv > p.n) return hipErrorInvalidValue;
  const size_t sl = shard_len(p.k, plen);
  const size_t tiles = (sl / 2 + TILE - 1) / TILE * batch;
  if (tiles >= (size_t(1) << 32) - size_t(4) * cus) return hipErrorInvalidValue;
  uint32_t *tick = static_cast<uint32_t *>(scratch);  // none: the static schedule
  if (tick)
    if (const hipError_t e = launch_zero_counters(tick, sizeof(uint32_t), s); e != hipSuccess) return e;
  const size_t slots = 2 * size_t(cus);  // two workgroups per CU
  const unsigned grid = unsigned(tiles < slots ? tiles : slots);
  hipLaunchKernelGGL(encode_k512w, dim3(grid), dim3(THREADS), LDS_BYTES, s, d_payloads, uint64_t(plen),
                     uint64_t(pstride), d_shards, uint64_t(sl), uint64_t(sstride), int(p.nv),
                     uint32_t(batch), t.cimg, t.eimg512, tick);
  return hipGetLastError();
}

}  // namespace ecamd
