// enc_kw.hip — encode for k = 2^M = 16, 32, 64, 128 (n <= 8 k: n_validators
// 46..765, the Polkadot validator counts of today among them) and k = 256 at
// n = 2048 (n_validators 1025..1533), two 8-wave workgroups per CU.
//
// encode_k256w's model (enc_k256w.hip): per piece (2 k
// payload bytes = k symbols) IFFT_k at index 0, then FFT_k at each coset k j
// below n_validators (encodeLow, poly_encoder.hpp:217-240), radix-8 register
// passes in tower coordinates, wave-private LDS exchanges.  A wave holds NG =
// 512 / k byte-planar groups of 4 pieces; a group's k positions lie over k / 8
// lanes x 8 registers, the group index in the lane bits above.  Read as
// position bits M..7 and encode_k256w's instance bit, the group bits make
// every layout and exchange encode_k256w's:
//  * layout A: registers p0..p2 (lane part 8 q, q = lane & (k/8 - 1));
//  * layout B: registers p3..p5 as far as they are positions (M = 4: p3 only,
//    M = 5: p3, p4), lanes p0..p2 and p6; for M <= 6 its elements are
//    wave-uniform;
//  * M = 7: stage 6 in layout C's register bit 0; M = 8: stages 6, 7 in
//    layout C (encode_k256w's pass C);
//  * every element of k <= 128 is x < 2^(M+2) <= 512: the 32 KB compact image
//    holds all tables (LDS 64 KB per workgroup); at k = 256, n = 2048 the
//    stage-0 elements of cosets 4..7 (512..1023) come from a 10 KB per-coset
//    extension image brought in by LDS-DMA, as in enc_k512w.hip (74 KB);
//  * tiles of 8 NG pieces per wave (32 KB of payload), shard-row segments of
//    64 NG bytes stored as 16 B per lane (two groups of one wave).
#include <hip/hip_runtime.h>

#include "ec_device.hpp"
#include "ec_kernels.hpp"
#include "cimg.hpp"
#include "enc_k256_common.hpp"

#include <type_traits>

namespace ecamd {
namespace {

constexpr int WAVES = 8;
constexpr int THREADS = 64 * WAVES;
constexpr uint32_t XCH0 = kCImgBytes;        // the wave regions follow the tables
constexpr uint32_t XCH_BYTES = 4096;
constexpr uint32_t SLOT = XCH0 + WAVES * XCH_BYTES;  // the next tile's index
// k = 256 (n = 2048 only): the extension tables of cosets 4..7 (stage 0,
// elements 512..1023: ec_kernels.hpp kEImg256*) after the slot
constexpr uint32_t EXT8 = SLOT + 1024;
template <int M>
constexpr int lds_bytes() { return int(M == 8 ? EXT8 + kEImg256Bytes : SLOT + 16); }
static_assert(2 * lds_bytes<8>() <= 160 * 1024, "two workgroups per CU");
static_assert(XCH0 % (2 * XCH_BYTES) == 0, "XOR-addressed regions");
static_assert(kCImgBytes % (16 * THREADS) == 0, "whole image chunks per thread");

template <int M>
struct Geo {
  static constexpr uint32_t K = 1u << M;
  static constexpr int NG = 512 >> M;          // byte-planar groups per wave
  static constexpr int WP = 4 * NG;            // pieces per wave
  static constexpr int TILE = WP * WAVES;      // pieces per tile (32 KB of payload)
  static constexpr int RC = 4 * NG;            // 16-B chunks per shard-row segment
  static constexpr int RPI = 512 / RC;         // rows per store iteration (all waves), 0 if < 1
  static constexpr uint32_t QM = (1u << (M - 3)) - 1;  // lane mask of the layout-A position part
  static_assert(M >= 4 && M <= 8, "k = 16 .. 256");
};

struct XLanes {
  uint32_t l0, l1, l2;
};
template <int B0>
__device__ __forceinline__ XLanes xlanes(uint32_t base) {
  return {cimg_lin(base >> (B0 + 1)), cimg_lin(base >> (B0 + 2)), cimg_lin(base >> (B0 + 3))};
}

// inverse radix-8 pass at index 0: every element < 64 (subfield)
template <int B0>
__device__ __forceinline__ void ipass(State &s, uint32_t base) {
  const XLanes x = xlanes<B0>(base);
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

// Table kinds of a stage: the compact image's subfield / F9 / general entries
// (SubTab, F9Tab, Tab), or (k = 256 at n = 2048, stage 0 of cosets 4..7) a
// general table of the coset's extension image in LDS (Ext0)
struct Ext0 {};
template <typename K_>
struct TabOf {
  using type = K_;
};
template <>
struct TabOf<Ext0> {
  using type = Tab;
};
// table of element x = lane part lt ^ block part r ^ uniform part u (each the
// cimg_lin of its bits); an extension table sits at the coset-local entry
// (u, the coset's offset bits, dropped)
template <typename K_>
__device__ __forceinline__ void ftab(uint32_t lt, uint32_t r, uint32_t u, typename TabOf<K_>::type &T) {
  if constexpr (std::is_same_v<K_, Ext0>) {
    const uint32_t a = lt ^ r;
#pragma unroll
    for (int q = 4; q >= 0; --q) {
      const v4u v = lds_r128(a + EXT8 + uint32_t(q) * (kEImg256Bytes / 5));
      T.t[4 * q] = v.x;
      T.t[4 * q + 1] = v.y;
      T.t[4 * q + 2] = v.z;
      T.t[4 * q + 3] = v.w;
    }
  } else {
    ctab(lt, r ^ u, T);
  }
}

// forward radix-8 pass at index off: stages B0+2, B0+1, B0 with table kinds
// K2, K1, K0 (known per coset)
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

// ---- layout C for k = 256 (register bit 0 = p6, bit 1 = p7, bit 2 = p5):
// the elements of stages 6, 7 are lane-uniform (enc_k256w.hip ipassC0w /
// fpassCw).  IFFT at index 0: stage 7 (x = 0) and stage 6's p7 = 0 block (x =
// 0) are b ^= a only; stage 6's p7 = 1 block has x = 1.
__device__ __forceinline__ void ipassC8(State &s) {
  SubTab Tb;
  ctab(0u, cimg_lin(1), Tb);
  bxor(s, 0, 1);
  bxor(s, 4, 5);
  ibfly(s, 2, 3, Tb);
  ibfly(s, 6, 7, Tb);
  bxor(s, 0, 2);
  bxor(s, 1, 3);
  bxor(s, 4, 6);
  bxor(s, 5, 7);
}
// FFT stages 7, 6 at index off from the IFFT coefficients c: stage 7 x = off
// >> 8, stage 6 x = off >> 7 | p7
__device__ __forceinline__ void fpassC8(State &s, const State &c, uint32_t off) {
  SubTab Ta, Tb;
  ctab(0u, cimg_lin(off >> 8), Ta);
  ctab(0u, cimg_lin(off >> 7), Tb);
  fbfly_from(s, c, 0, 2, Ta);
  fbfly_from(s, c, 1, 3, Ta);
  fbfly_from(s, c, 4, 6, Ta);
  fbfly_from(s, c, 5, 7, Ta);
  ctab(0u, cimg_lin((off >> 7) | 1u), Ta);
  fbfly(s, 0, 1, Tb);
  fbfly(s, 4, 5, Tb);
  fbfly(s, 2, 3, Ta);
  fbfly(s, 6, 7, Ta);
}

// ---- layout B for M <= 6: registers p3, p4, p5 as far as they are positions
// (the others group bits), no lane part: every element is x = (register
// position bits above m) | (off >> (m + 1)), wave-uniform.  Stage 3 pairs
// registers (2 rr, 2 rr + 1), rr = (p4, p5); stage 4 (r, r + 2), block p5;
// stage 5 (r, r + 4).
template <int M>
constexpr uint32_t bmask3() { return (M > 4 ? 1u : 0u) | (M > 5 ? 2u : 0u); }
template <int M>
constexpr uint32_t bmask4() { return M > 5 ? 1u : 0u; }

// IFFT stages 3 .. M - 1 at index 0 (x = 0: b ^= a only, additive_fft.hpp:110-112)
template <int M>
__device__ __forceinline__ void ipassB_u(State &s) {
  SubTab T1, T2, T3;
  ctab(0u, cimg_lin(1), T1);
  if constexpr (M > 5) {
    ctab(0u, cimg_lin(2), T2);
    ctab(0u, cimg_lin(3), T3);
  }
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const uint32_t x = uint32_t(rr) & bmask3<M>();
    if (x == 0) bxor(s, 2 * rr, 2 * rr + 1);
    else if (x == 1) ibfly(s, 2 * rr, 2 * rr + 1, T1);
    else if (x == 2) ibfly(s, 2 * rr, 2 * rr + 1, T2);
    else ibfly(s, 2 * rr, 2 * rr + 1, T3);
  }
  if constexpr (M > 4) {
#pragma unroll
    for (int r : {0, 1, 4, 5}) {
      if (((uint32_t(r) >> 2) & bmask4<M>()) == 0) bxor(s, r, r + 2);
      else ibfly(s, r, r + 2, T1);
    }
  }
  if constexpr (M > 5) {
#pragma unroll
    for (int r = 0; r < 4; ++r) bxor(s, r, r + 4);
  }
}

// FFT stages M - 1 .. 3 at index off, the first one reading the IFFT
// coefficients c
template <int M>
__device__ __forceinline__ void fpassB_u(State &s, const State &c, uint32_t off) {
  if constexpr (M > 5) {  // stage 5, x = off >> 6
    SubTab T;
    ctab(0u, cimg_lin(off >> 6), T);
#pragma unroll
    for (int r = 0; r < 4; ++r) fbfly_from(s, c, r, r + 4, T);
  }
  if constexpr (M > 4) {  // stage 4, x = off >> 5 | p5
    SubTab Ta, Tb;
    ctab(0u, cimg_lin(off >> 5), Ta);
    ctab(0u, cimg_lin(off >> 5) ^ cimg_lin(bmask4<M>()), Tb);
#pragma unroll
    for (int r : {0, 1, 4, 5}) {
      const SubTab &T = (uint32_t(r) >> 2) & bmask4<M>() ? Tb : Ta;
      if constexpr (M == 5) fbfly_from(s, c, r, r + 2, T);
      else fbfly(s, r, r + 2, T);
    }
  }
  {  // stage 3, x = off >> 4 | (p4, p5)
    SubTab T[4];
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) ctab(0u, cimg_lin(off >> 4) ^ cimg_lin(uint32_t(rr) & bmask3<M>()), T[rr]);
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      if constexpr (M == 4) fbfly_from(s, c, 2 * rr, 2 * rr + 1, T[rr]);
      else fbfly(s, 2 * rr, 2 * rr + 1, T[rr]);
    }
  }
}

// wave-private exchange at the wave's region folded into the lane bases (bits
// >= 12), the bases laundered so the cell addresses are formed here
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

// ---- own-region staging: wave w stages its NG groups x k rows in its own
// 4 KB region, 8 B per (row v, group g) at slot (v NG + g) ^ (v >> 3) << (8 -
// M) ^ ((w << (9 - M)) & 31).  Layout-A writes (rows 8 q + r; 32 lanes = the
// q and the low group bits) and the store reads (16 lanes x 16 B = group pairs
// (2h, 2h + 1) of one row across waves) hit distinct banks.
// k = 256 (NG = 2): bit 0 stays the group (a store read takes groups 0 and 1
// of a row as one 16-B pair), the row's bits 3-6 go to bits 1-4 (16-lane
// write groups distinct) and the wave to bits 2-4 (the two rows of a 16-lane
// store read, which differ in bit 1, keep their 8 chunks apart).
template <int M>
__host__ __device__ constexpr uint32_t soff(uint32_t v, uint32_t g, uint32_t w) {
  if constexpr (M == 8)
    return (((v << 1) | g) ^ (((v >> 3) & 15u) << 1) ^ ((w << 2) & 31u)) << 3;
  else
    return (((v << (9 - M)) | g) ^ ((v >> 3) << (8 - M)) ^ ((w << (9 - M)) & 31u)) << 3;
}

template <int M>
__device__ __forceinline__ void stage_own(const State &s, uint32_t q, uint32_t g, uint32_t wave) {
  const uint32_t a = XCH0 + wave * XCH_BYTES + soff<M>(8 * q, g, wave);
#pragma unroll
  for (int r = 0; r < 8; ++r) lds_st2(a ^ soff<M>(uint32_t(r), 0, 0), to_be(s.l[0][r], s.h[0][r]));
}

// all waves: rows [s0, s0 + k) from the 8 regions -> shards.  Chunk G = it *
// 512 + thread: row v = G / RC, chunk c = G % RC (16 B = pieces 8c..8c+7 =
// groups 2h, 2h + 1 of wave c / (NG / 2)).  Fast path (uniform): 16-B aligned
// rows, the whole tile inside the payload, all k rows below n_validators -- 4
// streaming 16-B stores per lane.
template <int M>
__device__ __forceinline__ bool store_fast(const uint8_t *SH, uint64_t sstride, uint32_t s0, int nv,
                                           uint64_t piece0, uint64_t npieces) {
  return ((sstride | reinterpret_cast<uintptr_t>(SH)) & 15) == 0 && piece0 + Geo<M>::TILE <= npieces &&
         int(s0) + int(Geo<M>::K) <= nv;
}

template <int M, typename Then>
__device__ __forceinline__ void store_own(uint8_t *SH, uint64_t sstride, uint32_t s0, int nv,
                                          uint64_t piece0, uint64_t npieces, uint32_t wave,
                                          uint32_t lane, Then &&then) {
  using G = Geo<M>;
  asm volatile("" : "+v"(lane));  // recomputed here, not kept live across the FFTs
  const uint32_t t = wave * 64 + lane;
  const uint32_t v0 = t / G::RC, c = t % G::RC;  // it = 0
  const uint32_t cw = c / (G::NG / 2), h = c % (G::NG / 2);
  const uint32_t ra = XCH0 + cw * XCH_BYTES + soff<M>(v0, 2 * h, cw);  // 16-B aligned: groups 2h, 2h + 1
  constexpr uint32_t VSTEP = 512 / G::RC;  // rows per iteration
  if (store_fast<M>(SH, sstride, s0, nv, piece0, npieces)) {
    uint8_t *dst = SH + uint64_t(s0 + v0) * sstride + 2 * (piece0 + 8 * c);
    const uint64_t dstep = uint64_t(VSTEP) * sstride;
#pragma unroll
    for (int it = 0; it < 4; ++it) {  // soff is GF(2)-linear in v = it * VSTEP | v0
      const v4u val = lds_r128(ra ^ soff<M>(uint32_t(it) * VSTEP, 0, 0));
      __builtin_nontemporal_store(val, reinterpret_cast<v4u *>(dst + it * dstep));
    }
    then();
    asm volatile("; store_own fast path end" ::: "memory");
    return;
  }
  const uint64_t p = piece0 + 8 * c;
  const bool wide = ((sstride | reinterpret_cast<uintptr_t>(SH)) & 15) == 0;
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const uint32_t v = uint32_t(it) * VSTEP + v0;
    const v4u val = lds_r128(ra ^ soff<M>(uint32_t(it) * VSTEP, 0, 0));
    const uint32_t shard = s0 + v;
    if (int(shard) >= nv) continue;
    uint8_t *dst = SH + uint64_t(shard) * sstride + 2 * p;
    if (p + 8 <= npieces) {
      if (wide) {
        *reinterpret_cast<v4u *>(dst) = val;
      } else {
        reinterpret_cast<uint2 *>(dst)[0] = make_uint2(val.x, val.y);
        reinterpret_cast<uint2 *>(dst)[1] = make_uint2(val.z, val.w);
      }
    } else if (p < npieces) {
      const uint32_t w[4] = {val.x, val.y, val.z, val.w};
      for (uint64_t e = 0; e < npieces - p; ++e)
        *reinterpret_cast<uint16_t *>(dst + 2 * e) = uint16_t(w[e >> 1] >> (16 * (e & 1)));
    }
  }
  then();
  asm volatile("; store_own slow path end" ::: "memory");
}

// 4 x 16 payload bytes (4 pieces, positions 8 q .. 8 q + 7) -> byte-planar
// State (enc_k256w.hip to_state)
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

}  // namespace

template <int M>
__global__ void __launch_bounds__(THREADS, 4) encode_kw(const uint8_t *__restrict__ payloads,
                                                        uint64_t plen, uint64_t pstride,
                                                        uint8_t *__restrict__ shards, uint64_t slen,
                                                        uint64_t sstride, int nv, uint32_t batch,
                                                        const uint8_t *__restrict__ cimg,
                                                        const uint8_t *__restrict__ eimg,
                                                        uint32_t *__restrict__ tick) {
  using G = Geo<M>;
  constexpr uint32_t K = G::K;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const uint32_t tid0 = threadIdx.x;
  auto *slot = reinterpret_cast<__attribute__((address_space(3))) volatile uint32_t *>(uintptr_t(SLOT));
  if (tid0 == 0) *slot = tick ? atomicAdd(tick, 1u) : blockIdx.x;
  {  // the compact image (32 KB), every load issued before the first store
    constexpr int kPer = int(kCImgBytes / 16 / THREADS);
    v4u v[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) v[k] = reinterpret_cast<const v4u *>(cimg)[tid0 + k * THREADS];
#pragma unroll
    for (int k = 0; k < kPer; ++k) reinterpret_cast<v4u *>(lds)[tid0 + k * THREADS] = v[k];
  }
  __syncthreads();

  const uint64_t npieces = slen / 2;
  const uint32_t tiles_pp = uint32_t((npieces + G::TILE - 1) / G::TILE);
  const uint32_t total = tiles_pp * batch;  // < 2^32 (launch_encode_kw)
  const uint32_t wave_s = __builtin_amdgcn_readfirstlane(tid0 >> 6);
  const uint32_t J = uint32_t(nv - 1) / K;  // cosets k j, j = 1..J <= 7 (nv <= n <= 8 k)
  uint32_t cur = __builtin_amdgcn_readfirstlane(*slot);

  // This lane's 4 x 16 payload bytes of tile (b, i): pieces i * TILE + WP wave
  // + 4 g + u (g = lane >> (M - 3)), bytes 16 q .. 16 q + 15 of each (q = lane
  // & QM), zero past plen; issued in the previous tile's last coset.
  v4u d[4];
  State nxt;
  const auto fetch = [&](uint64_t fb, uint64_t fi) __attribute__((always_inline)) {
    const uint8_t *FP = payloads + fb * pstride;
    const uint64_t pw = fi * G::TILE + G::WP * wave_s;  // this wave's first piece (uniform)
    uint32_t ftid = tid0;
    asm volatile("" : "+v"(ftid));
    const uint32_t lane = ftid & 63, g = lane >> (M - 3), q = lane & G::QM;
    if ((pw + G::WP) * 2 * K <= plen) {  // the wave's pieces inside the payload
      const uint8_t *src = FP + (pw + 4 * g) * 2 * K + 16 * q;
#pragma unroll
      for (int u = 0; u < 4; ++u) d[u] = *reinterpret_cast<const v4u *>(src + u * 2 * K);
    } else if (pw < npieces) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint64_t off = (pw + 4 * g + u) * 2 * K + 16 * q;
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
    // encode_k256w's lane roles: q5 = position bits 3..7 in layout A (the
    // group bits above p(M-1) read as positions), inst = lane bit 5
    const uint32_t q5 = lane & 31, i0 = lane >> 5;
    const uint32_t reg0 = XCH0 + wave * XCH_BYTES;
    XBase xb;
    xb.a = reg0 | mswz(ulaneA(q5, i0));
    xb.b = reg0 | mswz(ulaneB(q5, i0));
    xb.c = reg0 | mswz(ulaneC(q5, i0));
    const uint64_t b = cur / tiles_pp, piece0 = uint64_t(cur % tiles_pp) * G::TILE;
    uint32_t taken = 0;
    if (tid0 == 0) taken = tick ? atomicAdd(tick, 1u) : cur + gridDim.x;
    uint32_t next = 0;
    uint8_t *SH = shards + b * uint64_t(nv) * sstride;
    // every store phase of this tile but possibly the last coset's takes the
    // fast path (4 stores per lane), or none does
    [[maybe_unused]] const bool fast = store_fast<M>(SH, sstride, 0, nv, piece0, npieces);
    // k = 256, n = 2048: coset j's extension image (10 x 1 KB) -> LDS, chunk i by
    // wave i % 8, issued after the previous coset's rows-staged barrier
    [[maybe_unused]] const auto dma_ext = [&](uint32_t j) __attribute__((always_inline)) {
      const uint8_t *src = eimg + (j - 4) * kEImg256Bytes + 16 * lane;
      for (uint32_t i = wave_s; i < kEImg256Bytes / 1024; i += WAVES)
        lds_dma16(EXT8 + 1024 * i, src + 1024 * i);
    };
    const auto fetch_next = [&]() __attribute__((always_inline)) {
      next = __builtin_amdgcn_readfirstlane(*slot);
      fetch(next < total ? next / tiles_pp : 0, next < total ? next % tiles_pp : tiles_pp);
    };
    const auto rsync = [&]() __attribute__((always_inline)) { lds_barrier(); };
    const auto store = [&](uint32_t s0, bool last) __attribute__((always_inline)) {
      __builtin_amdgcn_s_setprio(1);
      if (last)
        store_own<M>(SH, sstride, s0, nv, piece0, npieces, wave_s, lane,
                     [&]() __attribute__((always_inline)) { to_state(d, nxt); });
      else
        store_own<M>(SH, sstride, s0, nv, piece0, npieces, wave_s, lane, [] {});
      __builtin_amdgcn_s_setprio(0);
    };
    const auto store_sys = [&]() __attribute__((always_inline)) {
      __builtin_amdgcn_s_setprio(1);
      store_own<M>(SH, sstride, 0, nv, piece0, npieces, wave_s, lane, [&]() __attribute__((always_inline)) {
        if (tid0 == 0) *slot = taken;
      });
      __builtin_amdgcn_s_setprio(0);
    };

    // a wave none of whose pieces exist (the payload's last, partial tile)
    // takes part only in the barriers and the row stores (uniform)
    if (piece0 + G::WP * wave_s >= npieces) {
      rsync();  // tile start
      rsync();  // systematic rows staged
      store_sys();
      rsync();  // after IFFT pass A
      for (uint32_t j = 1;; ++j) {
        if constexpr (M == 8) {
          if (j >= 4 && fast) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
          else if (j >= 4) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        rsync();  // previous rows read out
        if (j == J) {
          fetch_next();
          rsync();  // rows staged
          store(K * j, true);
          break;
        }
        rsync();  // rows staged
        if constexpr (M == 8)
          if (j >= 3) dma_ext(j + 1);
        store(K * j, false);
        __builtin_amdgcn_sched_barrier(0);
      }
      cur = next;
      continue;
    }

    State s = nxt;
    const uint32_t q = lane & G::QM, g = lane >> (M - 3);
    // ---- systematic shards 0..k-1 = the data symbols (poly_encoder.hpp:239)
    rsync();  // the other waves are done reading the regions (last tile)
    stage_own<M>(s, q, g, wave);
    rsync();
    store_sys();
    __builtin_amdgcn_sched_barrier(0);
    {  // into tower coordinates
      const TowerK tk = tower_k();
#pragma unroll
      for (int r = 0; r < 8; ++r) s.l[0][r] = tower_lo(s.l[0][r], s.h[0][r], tk);
    }

    // ---- IFFT_k (index 0): pass A (bits 0-2), then pass B (bits 3..M-1;
    // M = 7: 3-5, then stage 6 in layout C).  Lane parts of the positions
    // (group bits excluded): A 8 q, B (M = 7) posB(q5, 0) & 127
    const uint32_t baseA = 8 * q, baseB = posB(q5, 0) & (K - 1);
    ipass<0>(s, baseA);
    rsync();  // systematic rows read out of the regions
    xchg<LA, LB>(s, xb);
    if constexpr (M == 8) {
      ipass<3>(s, baseB);
      xchg<LB, LC>(s, xb);
      ipassC8(s);
    } else if constexpr (M == 7) {
      ipass<3>(s, baseB);
      xchg<LB, LC>(s, xb);
#pragma unroll
      for (int r = 0; r < 8; r += 2) bxor(s, r, r + 1);  // stage 6, x = 0 (additive_fft.hpp:110-112)
    } else {
      ipassB_u<M>(s);
    }
    State coef = s;

    // ---- FFT_k at each coset k j (encodeLow, poly_encoder.hpp:229-237).
    // Kinds (x = (pos + off) >> (m + 1)): M = 7: stage 0 subfield (j = 1), F9
    // (2, 3), general (4..7), stage 1 subfield (j <= 3), F9 above; M = 6:
    // stage 0 subfield (j <= 3), F9 above; everything else subfield.
    const auto coset = [&](auto t2, auto t1, auto t0, const uint32_t j) __attribute__((always_inline)) {
      using T2 = decltype(t2);
      using T1 = decltype(t1);
      using T0 = decltype(t0);
      const uint32_t off = K * j;
      uint32_t bA = baseA, bB = baseB;
      asm volatile("" : "+v"(bA), "+v"(bB));  // table addresses formed per coset, not hoisted
#pragma unroll
      for (int r = 0; r < 8; ++r) asm volatile("" : "+v"(coef.l[0][r]), "+v"(coef.h[0][r]));
      if constexpr (M == 8) {
        fpassC8(s, coef, off);
        // previous coset's rows read out; from coset 4 on, also this coset's
        // extension image landed in every wave (issued before the previous
        // coset's store phase: 4 stores per lane after it on the fast path)
        if (j >= 4 && fast) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else if (j >= 4) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        rsync();
        xchg<LC, LB>(s, xb);
        fpass<3, SubTab, SubTab, SubTab>(s, bB, off);
      } else if constexpr (M == 7) {
        {  // stage 6, x = off >> 7, from the coefficients
          SubTab T6;
          ctab(0u, cimg_lin(off >> 7), T6);
#pragma unroll
          for (int r = 0; r < 8; r += 2) fbfly_from(s, coef, r, r + 1, T6);
        }
        rsync();  // previous coset's rows read out
        xchg<LC, LB>(s, xb);
        fpass<3, SubTab, SubTab, SubTab>(s, bB, off);
      } else {
        fpassB_u<M>(s, coef, off);
        rsync();  // previous coset's rows read out
      }
      xchg<LB, LA>(s, xb);
      fpass<0, T2, T1, T0>(s, bA, off);
      {  // back to symbol coordinates
        const TowerK tk = tower_k();
#pragma unroll
        for (int r = 0; r < 8; ++r) s.l[0][r] = tower_lo(s.l[0][r], s.h[0][r], tk);
      }
      stage_own<M>(s, q, g, wave);
    };
    // the cosets in a loop (a body per table-kind class); the last one leaves
    // it, so the next tile's payload (d, nxt) is live in that one only
    for (uint32_t j = 1;; ++j) {
      if constexpr (M == 8) {  // n = 2048: stage 0 of cosets 4..7 from the extension image
        if (j == 1) coset(SubTab(), SubTab(), F9Tab(), j);
        else if (j <= 3) coset(SubTab(), F9Tab(), Tab(), j);
        else coset(F9Tab(), Tab(), Ext0(), j);
      } else if constexpr (M == 7) {
        if (j == 1) coset(SubTab(), SubTab(), SubTab(), j);
        else if (j <= 3) coset(SubTab(), SubTab(), F9Tab(), j);
        else coset(SubTab(), F9Tab(), Tab(), j);
      } else if constexpr (M == 6) {
        if (j <= 3) coset(SubTab(), SubTab(), SubTab(), j);
        else coset(SubTab(), SubTab(), F9Tab(), j);
      } else {
        coset(SubTab(), SubTab(), SubTab(), j);
      }
      if (j == J) {
        fetch_next();  // coef and s are dead here
        rsync();       // rows staged
        store(K * j, true);
        break;
      }
      rsync();  // rows staged; every wave is past this coset's tables
      if constexpr (M == 8)
        if (j >= 3) dma_ext(j + 1);
      store(K * j, false);
      __builtin_amdgcn_sched_barrier(0);
    }
    cur = next;
  }
  if constexpr (M == 8) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA outlives the workgroup
}

bool kw_applicable(const CodeParams &p) {
  return (p.k >= 16 && p.k <= 128 && (p.k & (p.k - 1)) == 0 && p.n > p.k && p.n <= 8 * p.k) ||
         (p.k == 256 && p.n == 2048);
}

size_t kw_scratch_bytes(const CodeParams &p) { return kw_applicable(p) ? 256 : 0; }

template <int M>
static hipError_t launch_m(const CodeParams &p, const DevTables &t, const uint8_t *d_payloads, size_t plen,
                           size_t pstride, size_t batch, uint8_t *d_shards, size_t sstride, void *scratch,
                           hipStream_t s) {
  int cus = 0;
  if (const hipError_t e = prepare_kernel(reinterpret_cast<const void *>(&encode_kw<M>), lds_bytes<M>(), &cus);
      e != hipSuccess)
    return e;
  const size_t sl = shard_len(p.k, plen);
  const size_t tiles = (sl / 2 + Geo<M>::TILE - 1) / Geo<M>::TILE * batch;
  if (tiles >= (size_t(1) << 32) - size_t(4) * cus) return hipErrorInvalidValue;
  uint32_t *tick = static_cast<uint32_t *>(scratch);  // none: the static schedule
  if (tick)
    if (const hipError_t e = launch_zero_counters(tick, sizeof(uint32_t), s); e != hipSuccess) return e;
  const size_t slots = 2 * size_t(cus);  // two workgroups per CU
  const unsigned grid = unsigned(tiles < slots ? tiles : slots);
  hipLaunchKernelGGL(encode_kw<M>, dim3(grid), dim3(THREADS), lds_bytes<M>(), s, d_payloads, uint64_t(plen),
                     uint64_t(pstride), d_shards, uint64_t(sl), uint64_t(sstride), int(p.nv),
                     uint32_t(batch), t.cimg, t.eimg256, tick);
  return hipGetLastError();
}

hipError_t launch_encode_kw(const CodeParams &p, const DevTables &t, const uint8_t *d_payloads,
                            size_t plen, size_t pstride, size_t batch, uint8_t *d_shards,
                            size_t sstride, void *scratch, hipStream_t s) {
  if (!t.cimg || !kw_applicable(p) || p.nv <= p.k || p.nv > p.n) return hipErrorInvalidValue;
  if (p.k == 256 && (!t.eimg256 || p.nv <= 4 * p.k)) return hipErrorInvalidValue;  // cosets 4.. exist (n = 2048)
  switch (p.k) {
    case 16: return launch_m<4>(p, t, d_payloads, plen, pstride, batch, d_shards, sstride, scratch, s);
    case 32: return launch_m<5>(p, t, d_payloads, plen, pstride, batch, d_shards, sstride, scratch, s);
    case 64: return launch_m<6>(p, t, d_payloads, plen, pstride, batch, d_shards, sstride, scratch, s);
    case 128: return launch_m<7>(p, t, d_payloads, plen, pstride, batch, d_shards, sstride, scratch, s);
    default: return launch_m<8>(p, t, d_payloads, plen, pstride, batch, d_shards, sstride, scratch, s);
  }
}

}  // namespace ecamd
