// enc_k256w.hip — encode for k = 256, n = 1024 (n_validators 766..1024, the
// BASELINE headline), two 8-wave workgroups per CU.
//
// The transforms are those of encode_k256 (enc_k256.hip):
// per piece IFFT_256 at index 0, then FFT_256 at the cosets 256, 512, 768
// (encodeLow, poly_encoder.hpp:217-240), radix-8 register passes with
// wave-private LDS exchanges, tower coordinates with subfield / F9 / general
// multiplies.  What differs:
//  * the multiply tables are the 32 KB element-indexed compact image
//    (ec_kernels.hpp kCImg*, DevTables::cimg) instead of the 80 KB skew-slot
//    image, so a workgroup needs 64 KB of LDS and TWO are resident per CU.
//    Each workgroup still synchronises its waves at every staging step, but
//    while one waits at a barrier, for its payload loads or for its row
//    stores to issue, the other one's waves compute on the same SIMDs
//    (phase stamps of the 16-wave form: 30% of wave time at barriers, 9% in
//    the payload loads, 9% in the stores);
//  * the tile is 64 pieces (8 waves x 8), each shard row a 128-B segment.
#include <hip/hip_runtime.h>

#include "ec_device.hpp"
#include "ec_kernels.hpp"
#include "cimg.hpp"
#include "enc_k256_common.hpp"

namespace ecamd {
namespace {

constexpr int K = 256;
constexpr int WAVES = 8;
constexpr int THREADS = 64 * WAVES;
constexpr int TILE = 8 * WAVES;  // pieces per tile
constexpr uint32_t XCH_BYTES = 256 * 16;   // per-wave exchange / staging region
constexpr uint32_t XCH0 = kCImgBytes;      // the regions follow the tables
constexpr uint32_t SLOT = XCH0 + WAVES * XCH_BYTES;  // the next tile's index (dynamic schedule)
constexpr int LDS_BYTES = int(SLOT + 16);
static_assert(2 * LDS_BYTES <= 160 * 1024, "two workgroups per CU");
static_assert(kCImgBytes % (16 * THREADS) == 0, "whole image chunks per thread");

// Element index of a stage-m butterfly whose a-position is pos, in a transform
// at index off (a multiple of 256): x = (pos + off) >> (m + 1) (ec_kernels.hpp).
// A radix-8 pass over position bits b0..b0+2 held in registers (pos = base |
// r << b0, base without those bits): stage b0 block rr (registers 2rr, 2rr+1)
// x = base >> (b0+1) | rr; stage b0+1 block hh (registers 4hh + {0,1}, + 2)
// x = base >> (b0+2) | hh; stage b0+2: x = base >> (b0+3); each | off >> (m+1).
// Lane parts l0..l2 = cimg_lin of the three base shifts (3 VGPRs per pass).
struct XLanes {
  uint32_t l0, l1, l2;
};
template <int B0>
__device__ __forceinline__ XLanes xlanes(uint32_t base) {
  return {cimg_lin(base >> (B0 + 1)), cimg_lin(base >> (B0 + 2)), cimg_lin(base >> (B0 + 3))};
}

// inverse pass, index 0 (IFFT_256): every element < 128 (subfield)
template <int B0>
__device__ __forceinline__ void ipass3w(State &s, uint32_t base) {
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

// forward pass at index off: stages b0+2, b0+1, b0 with table types T2, T1, T0
// (the elements' kinds, known per coset: DESIGN.md §5.1)
template <int B0, typename T2, typename T1, typename T0>
__device__ __forceinline__ void fpass3w(State &s, uint32_t base, uint32_t off) {
  const XLanes x = xlanes<B0>(base);
  // uniform parts (scalar for a run-time coset): cimg_lin(off >> (m + 1))
  const uint32_t u0 = cimg_lin(off >> (B0 + 1)), u1 = cimg_lin(off >> (B0 + 2)), u2 = cimg_lin(off >> (B0 + 3));
  T2 Ta2;
  T1 Ta1, Tb1;
  T0 Ta0, Tb0;
  ctab(x.l2, u2, Ta2);
  ctab(x.l1, u1, Tb1);
#pragma unroll
  for (int r = 0; r < 4; ++r) fbfly(s, r, r + 4, Ta2);
  ctab(x.l1, u1 ^ cimg_lin(1), Ta1);
  fbfly(s, 0, 2, Tb1);
  fbfly(s, 1, 3, Tb1);
  ctab(x.l0, u0, Tb0);
  fbfly(s, 4, 6, Ta1);
  fbfly(s, 5, 7, Ta1);
  ctab(x.l0, u0 ^ cimg_lin(1), Ta0);
  fbfly(s, 0, 1, Tb0);
  ctab(x.l0, u0 ^ cimg_lin(2), Tb0);
  fbfly(s, 2, 3, Ta0);
  ctab(x.l0, u0 ^ cimg_lin(3), Ta0);
  fbfly(s, 4, 5, Tb0);
  fbfly(s, 6, 7, Ta0);
}

// layout C (register bit0 = p6, bit1 = p7, bit2 = p5): the elements of stages
// 6, 7 are lane-uniform.  IFFT at index 0: stage 7 (x = 0) and stage 6's
// p7 = 0 block (x = 0) are b ^= a only (the skew 0xFFFF of additive_fft.hpp:
// 110-112); stage 6's p7 = 1 block has x = 1.
__device__ __forceinline__ void ipassC0w(State &s) {
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

// FFT stages 7, 6 at index off, reading the IFFT coefficients c and writing s:
// stage 7 x = off >> 8, stage 6 x = off >> 7 | p7
__device__ __forceinline__ void fpassCw(State &s, const State &c, uint32_t off) {
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

// ---- own-region staging: wave w stages its 8 pieces x 256 rows in its own
// 4 KB region, 16 B per row (half = instance); row v in 256-B block v >> 4 at
// 16-B slot (v ^ (v >> 4) ^ 2w) & 15.  The row reads (lane = row-in-8 << 3 |
// source wave c) hit 16 distinct slots in every ds_read_b128 lane group; the
// layout-A writes are 2-way (the minimum for 8-B writes of one instance).
__host__ __device__ constexpr uint32_t soff8(uint32_t v, uint32_t w) {
  return ((v >> 4) << 8) | (((v ^ (v >> 4) ^ (w << 1)) & 15) << 4);
}

__device__ __forceinline__ void stage_own8(const State &s, uint8_t *xch, uint32_t q, uint32_t inst,
                                           uint32_t wave) {
#pragma unroll
  for (int r = 0; r < 8; ++r)
    *reinterpret_cast<uint2 *>(xch + soff8(posA(q, r), wave) + 8 * inst) = to_be(s.l[0][r], s.h[0][r]);
}

// all waves: rows [s0, s0 + 256) from the 8 regions -> shards.  Lane = (row in
// 8, source wave c = 16-B chunk of pieces [8c, 8c + 8)); row v = it * 64 +
// wave * 8 + lane / 8.  Fast path (uniform): 16-B aligned rows, the whole tile
// inside the payload, all 256 rows below n_validators -- one streaming 16-B
// store per lane and row, 8 lanes per 128-B row segment.
__device__ __forceinline__ bool store_fast(const uint8_t *SH, uint64_t sstride, uint32_t s0, int nv,
                                           uint64_t piece0, uint64_t npieces) {
  return ((sstride | reinterpret_cast<uintptr_t>(SH)) & 15) == 0 && piece0 + TILE <= npieces &&
         int(s0) + 256 <= nv;
}

// `then` runs at the end of each path: code that waits for a load issued
// before the stores is placed there, so the compiler's wait on the fast path
// counts its 4 stores (vmcnt(4)) instead of the minimum over every path.
template <typename Then>
__device__ __forceinline__ void store_own8(uint8_t *SH, uint64_t sstride, uint32_t s0, int nv,
                                           uint64_t piece0, uint64_t npieces, uint32_t wave,
                                           uint32_t lane, Then &&then) {
  asm volatile("" : "+v"(lane));  // recomputed here, not kept live across the FFTs
  const uint32_t c = lane & 7;
  const uint32_t v0 = wave * 8 + (lane >> 3);
  const uint32_t sa = XCH0 + c * XCH_BYTES + soff8(v0, c);
  if (store_fast(SH, sstride, s0, nv, piece0, npieces)) {
    uint8_t *dst = SH + uint64_t(s0 + v0) * sstride + 2 * (piece0 + 8 * c);
    const uint64_t dstep = uint64_t(8 * WAVES) * sstride;
#pragma unroll
    for (int it = 0; it < 256 / (8 * WAVES); ++it) {  // soff8 is GF(2)-linear in v = it * 64 | v0
      const v4u val = lds_r128(sa ^ soff8(uint32_t(it) * 8 * WAVES, 0));
      __builtin_nontemporal_store(val, reinterpret_cast<v4u *>(dst + it * dstep));  // written once
    }
    then();
    asm volatile("; store_own8 fast path end" ::: "memory");  // distinct tails: `then` is not merged
    return;
  }
  const uint64_t p = piece0 + 8 * c;
  const bool wide = ((sstride | reinterpret_cast<uintptr_t>(SH)) & 15) == 0;
#pragma unroll
  for (int it = 0; it < 256 / (8 * WAVES); ++it) {
    const uint32_t v = uint32_t(it) * 8 * WAVES + v0;
    const v4u val = lds_r128(sa ^ soff8(uint32_t(it) * 8 * WAVES, 0));
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
  asm volatile("; store_own8 slow path end" ::: "memory");
}

// 4 x 16 payload bytes (4 pieces, positions 8q..8q+7) -> byte-planar State:
// 4x4 byte transposes, dword j of each piece = (hi_{2j}, lo_{2j}, hi_{2j+1}, lo_{2j+1})
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

__global__ void __launch_bounds__(THREADS, 4) encode_k256w(const uint8_t *__restrict__ payloads,
                                                           uint64_t plen, uint64_t pstride,
                                                           uint8_t *__restrict__ shards, uint64_t slen,
                                                           uint64_t sstride, int nv, uint32_t batch,
                                                           const uint8_t *__restrict__ cimg,
                                                           uint32_t *__restrict__ tick) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const uint32_t tid0 = threadIdx.x;
  auto *slot = reinterpret_cast<__attribute__((address_space(3))) volatile uint32_t *>(uintptr_t(SLOT));
  // this workgroup's first tile; without a counter (no scratch) a static
  // grid stride (slower: the two workgroups of a CU drift apart, below)
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
  const uint32_t tiles_pp = uint32_t((npieces + TILE - 1) / TILE);
  const uint32_t total = tiles_pp * batch;  // < 2^32 (launch_encode_k256w)
  const uint32_t wave_s = __builtin_amdgcn_readfirstlane(tid0 >> 6);
  // Dynamic schedule: tiles are taken from the launch's counter (`tick`,
  // zeroed before the launch) one tile ahead, so the two workgroups of a CU,
  // which the issue arbiter serves at unequal rates (the older one's waves win
  // ties), finish together.  With a static grid-stride split the faster one
  // ended up to 2.8 ms before the slower one of a 7 ms launch, which then ran
  // alone (scripts/variants/clk_run.py).
  // Thread 0 takes tile t + 1 at the start of tile t and publishes it in the
  // LDS slot after the tile's systematic stores; every wave reads it after the
  // barrier that follows IFFT pass A; the slot is rewritten only after the
  // next tile-start barrier, by which every wave has read it.
  uint32_t cur = __builtin_amdgcn_readfirstlane(*slot);

  // This lane's 4 x 16 payload bytes of tile (b, i): pieces i * TILE + 8 wave +
  // 4 inst + u, bytes 16 q .. 16 q + 15 of each, zero past plen.  A tile's loads
  // are issued at the end of the previous tile, before its last row stores, and
  // turned into the next State right after those stores (store_own8's `then`).
  // vmcnt counts loads and stores together in issue order: loads issued after
  // a store phase (the tile start) wait for those stores to complete.
  v4u d[4];
  State nxt;  // the next tile's data, byte-planar, symbol coordinates
  const auto fetch = [&](uint64_t fb, uint64_t fi) __attribute__((always_inline)) {
    const uint8_t *FP = payloads + fb * pstride;
    const uint64_t pw = fi * TILE + 8 * wave_s;  // this wave's first piece (uniform)
    uint32_t ftid = tid0;
    asm volatile("" : "+v"(ftid));  // per-lane addresses recomputed here, not hoisted and spilled
    const uint32_t lane = ftid & 63, inst = lane >> 5, q = lane & 31;
    if ((pw + 8) * 2 * K <= plen) {  // the wave's 8 pieces inside the payload: 4 loads in flight
      const uint8_t *src = FP + (pw + 4 * inst) * 2 * K + 16 * q;
#pragma unroll
      for (int u = 0; u < 4; ++u) d[u] = *reinterpret_cast<const v4u *>(src + u * 2 * K);
    } else if (pw < npieces) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint64_t off = (pw + 4 * inst + u) * 2 * K + 16 * q;
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
    } else {  // every path assigns d: the old value is never carried across a tile
#pragma unroll
      for (int u = 0; u < 4; ++u) d[u] = v4u{0, 0, 0, 0};
    }
  };
  if (cur < total) {
    fetch(cur / tiles_pp, cur % tiles_pp);
    to_state(d, nxt);
  }

  while (cur < total) {
    // lane ids made opaque per tile: per-lane LDS addresses are recomputed in
    // the loop instead of being hoisted out of it and spilled
    uint32_t tid = tid0;
    asm volatile("" : "+v"(tid));
    const uint32_t lane = tid & 63, wave = tid >> 6;
    const uint32_t inst = lane >> 5, q = lane & 31;
    uint8_t *xch = lds + XCH0 + wave * XCH_BYTES;
    XBase xb;
    xb.a = mswz(ulaneA(q, inst));
    xb.b = mswz(ulaneB(q, inst));
    xb.c = mswz(ulaneC(q, inst));
    const uint64_t b = cur / tiles_pp, piece0 = uint64_t(cur % tiles_pp) * TILE;
    uint32_t taken = 0;  // thread 0: the tile taken for after this one
    if (tid0 == 0) taken = tick ? atomicAdd(tick, 1u) : cur + gridDim.x;
    uint32_t next = 0;   // every wave: that tile, read from the slot
    uint8_t *SH = shards + b * uint64_t(nv) * sstride;
    // the last coset of this n_validators (uniform), after whose staging the
    // next tile's payload is fetched
    const uint32_t last_sh = nv > 768 ? 768u : 512u;  // nv > 512 (launch_encode_k256w)
    const auto fetch_next = [&]() __attribute__((always_inline)) {
      next = __builtin_amdgcn_readfirstlane(*slot);
      // past the end: the zero path, no loads
      fetch(next < total ? next / tiles_pp : 0, next < total ? next % tiles_pp : tiles_pp);
    };
    const auto rsync = [&]() __attribute__((always_inline)) { lds_barrier(); };
    const auto store = [&](uint32_t s0) __attribute__((always_inline)) {
      // the row stores (LDS reads + global stores) at raised issue priority
      __builtin_amdgcn_s_setprio(1);
      store_own8(SH, sstride, s0, nv, piece0, npieces, wave_s, lane, [] {});
      __builtin_amdgcn_s_setprio(0);
    };
    // the systematic rows' store phase; thread 0 then publishes the tile it
    // took (the wait for the atomic's return then counts only the stores
    // issued after it on the fast path, store_own8)
    const auto store_sys = [&]() __attribute__((always_inline)) {
      __builtin_amdgcn_s_setprio(1);
      store_own8(SH, sstride, 0, nv, piece0, npieces, wave_s, lane, [&]() __attribute__((always_inline)) {
        if (tid0 == 0) *slot = taken;
      });
      __builtin_amdgcn_s_setprio(0);
    };
    // the last store phase of the tile, then the next tile's State
    const auto store_last = [&](uint32_t s0) __attribute__((always_inline)) {
      __builtin_amdgcn_s_setprio(1);
      store_own8(SH, sstride, s0, nv, piece0, npieces, wave_s, lane,
                 [&]() __attribute__((always_inline)) { to_state(d, nxt); });
      __builtin_amdgcn_s_setprio(0);
    };

    // A wave none of whose 8 pieces exist (the last, partial tile of a payload:
    // 1 MB is 1954 pieces, its 31st tile has 34) skips the transforms and only
    // takes part in the barriers and the row stores of the others, in the same
    // order as below (wave-uniform branch)
    if (piece0 + 8 * wave_s >= npieces) {
      rsync();  // tile start
      rsync();  // systematic rows staged
      store(0);
      rsync();  // after IFFT pass A
      for (uint32_t sh = K; sh < 1024u && int(sh) < nv; sh += K) {
        rsync();  // after pass C
        rsync();  // rows staged
        if (sh == last_sh) {
          fetch_next();
          store_last(sh);
        } else {
          store(sh);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      cur = next;
      continue;
    }

    // ---- 8 pieces x 16 bytes (positions 8q..8q+7), fetched by the previous tile
    State s = nxt;

    // ---- systematic shards 0..255 = the data symbols (poly_encoder.hpp:239)
    rsync();  // the other waves are done reading this region (last tile)
    stage_own8(s, xch, q, inst, wave);
    rsync();
    store_sys();
    __builtin_amdgcn_sched_barrier(0);
    {  // into tower coordinates
      const TowerK tk = tower_k();
#pragma unroll
      for (int r = 0; r < 8; ++r) s.l[0][r] = tower_lo(s.l[0][r], s.h[0][r], tk);
    }

    // ---- IFFT_256 (index 0): passes A (bits 0-2), B (3-5), C (6-7)
    ipass3w<0>(s, posA(q, 0));
    rsync();  // systematic rows read out of the regions
    exchange<LA, LB>(s, xch, xb);
    ipass3w<3>(s, posB(q, 0));
    exchange<LB, LC>(s, xch, xb);
    ipassC0w(s);
    State coef = s;

    // ---- FFT_256 at each coset shift (encodeLow, poly_encoder.hpp:229-237).
    // Kinds of pass A's stages 2 / 1 / 0 by coset: 256: sub / sub / F9;
    // 512, 768: sub / F9 / general (x = (pos + off) >> (m + 1), ec_kernels.hpp)
    const auto coset = [&](auto t1, auto t0, const uint32_t off, auto last) __attribute__((always_inline)) {
      using T1 = decltype(t1);
      using T0 = decltype(t0);
      // coef made opaque in place (no copy): keeps the compiler from hoisting
      // the first stage's selector masks out of the coset loop
#pragma unroll
      for (int r = 0; r < 8; ++r) asm volatile("" : "+v"(coef.l[0][r]), "+v"(coef.h[0][r]));
      fpassCw(s, coef, off);
      rsync();  // previous coset's rows read out
      exchange<LC, LB>(s, xch, xb);
      fpass3w<3, SubTab, SubTab, SubTab>(s, posB(q, 0), off);
      exchange<LB, LA>(s, xch, xb);
      fpass3w<0, SubTab, T1, T0>(s, posA(q, 0), off);
      {  // back to symbol coordinates
        const TowerK tk = tower_k();
#pragma unroll
        for (int r = 0; r < 8; ++r) s.l[0][r] = tower_lo(s.l[0][r], s.h[0][r], tk);
      }
      stage_own8(s, xch, q, inst, wave);
      if constexpr (decltype(last)::value) fetch_next();  // coef and s are dead here
      rsync();
      if constexpr (decltype(last)::value)
        store_last(off);
      else
        store(off);
      __builtin_amdgcn_sched_barrier(0);
    };
    // n_validators 766..1024 (k = 256, n = 1024): cosets 256, 512 and, above
    // 768, 768; the last one has its own body (it fetches the next tile)
    coset(SubTab(), F9Tab(), K, std::false_type());
    if (last_sh == 3 * K) coset(F9Tab(), Tab(), 2 * K, std::false_type());
    coset(F9Tab(), Tab(), last_sh, std::true_type());
    cur = next;
  }
}

hipError_t launch_encode_k256w(const CodeParams &p, const DevTables &t, const uint8_t *d_payloads,
                               size_t plen, size_t pstride, size_t batch, uint8_t *d_shards,
                               size_t sstride, void *scratch, hipStream_t s) {
  int cus = 0;
  if (!t.cimg) return hipErrorInvalidValue;
  if (const hipError_t e = prepare_kernel(reinterpret_cast<const void *>(&encode_k256w), LDS_BYTES, &cus);
      e != hipSuccess)
    return e;
  if (p.nv <= 2 * K || p.nv > 1024) return hipErrorInvalidValue;  // cosets 256, 512 (, 768)
  const size_t sl = shard_len(p.k, plen);
  const size_t tiles = (sl / 2 + TILE - 1) / TILE * batch;
  if (tiles >= (size_t(1) << 32) - size_t(4) * cus) return hipErrorInvalidValue;
  // the tile counter (k256_scratch_bytes), zeroed in stream order; no
  // scratch: the static schedule (a missing counter costs speed,
  // not an error)
  uint32_t *tick = static_cast<uint32_t *>(scratch);
  if (tick)
    if (const hipError_t e = launch_zero_counters(tick, sizeof(uint32_t), s); e != hipSuccess) return e;
  const size_t slots = 2 * size_t(cus);  // two workgroups per CU
  const unsigned grid = unsigned(tiles < slots ? tiles : slots);
  hipLaunchKernelGGL(encode_k256w, dim3(grid), dim3(THREADS), LDS_BYTES, s, d_payloads, uint64_t(plen),
                     uint64_t(pstride), d_shards, uint64_t(sl), uint64_t(sstride), int(p.nv),
                     uint32_t(batch), t.cimg, tick);
  return hipGetLastError();
}

}  // namespace ecamd
