// enc_k256.hip — encode kernel specialised for k = 256, n = 1024
// (n_validators 766..1024, the BASELINE headline configuration).
//
// Work decomposition:
//  * persistent: one 1024-thread workgroup (16 waves, 4 per SIMD) per CU,
//    looping over tiles of 128 consecutive pieces (piece = 512 payload bytes
//    = 256 GF(2^16) symbols);
//  * wave w owns pieces [8w, 8w+8) of the tile: 2 "instances" (lanes 0-31 /
//    32-63) x 1 byte-planar group (registers) x 4 pieces;
//  * within an instance, lane q holds 8 of the 256 positions in registers:
//    every radix-8 pass runs 3 butterfly stages in registers, then the wave
//    re-distributes positions through its private LDS region;
//  * multiplies: v_perm tables (ec_device.hpp) for every skew the k=256 /
//    n=1024 code uses (1023 x 80 B) are resident in LDS for the whole kernel;
//  * shard stores: each wave stages its 8 pieces x 256 rows in its own LDS
//    region; all waves then write 256-byte contiguous row segments
//    (global_store_dwordx4, 16 B per lane).
// Butterflies, skew indices and the encodeLow structure follow
// include/ec-cpp/additive_fft.hpp:99-141 and poly_encoder.hpp:217-240.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "ec_device.hpp"
#include "ec_kernels.hpp"
#include "enc_k256_common.hpp"

namespace ecamd {
namespace {

constexpr int K = 256;
// one byte-planar group per lane (GP = 1) and 16 waves: 4 waves/SIMD (<= 128
// VGPRs) for latency hiding; the tile is 128 pieces
constexpr int WAVES = 16 / GP;
constexpr int THREADS = 64 * WAVES;
constexpr int TILE = 8 * GP * WAVES;  // pieces per tile
using Tabs = LdsTabs<1024>;
constexpr int TAB_REGION = Tabs::kBytes;  // skew idx 0..1022
constexpr int XCH_BYTES = 256 * 16 * GP;   // per-wave exchange region
constexpr int LDS_BYTES = TAB_REGION + WAVES * XCH_BYTES;
static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
static_assert(TILE == 128 && 256 * 256 <= WAVES * XCH_BYTES, "staging fits the exchange regions");

// GF(2)-linear part of the swizzled table address (LdsTabs::addr without the
// plane term): tlin(a | b) = tlin(a) ^ tlin(b) for disjoint a, b.  A table index
// is (lane part) | (uniform part), so its address is one v_xor of a per-lane
// base with a wave-uniform value.
__host__ __device__ constexpr uint32_t tlin(uint32_t idx) {
  return ((idx >> 4) << 8) | (((idx ^ (idx >> 4) ^ (idx >> 8)) & 15) << 4);
}

__device__ __forceinline__ void lds_tab_at(const uint8_t *lds, uint32_t lin, Tab &T) {
#pragma unroll
  for (int q = 4; q >= 0; --q) {  // plane 0 (first used) last: one wait per table
    const uint4 v = *reinterpret_cast<const uint4 *>(lds + q * Tabs::kPlane + lin);
    T.t[4 * q] = v.x;
    T.t[4 * q + 1] = v.y;
    T.t[4 * q + 2] = v.z;
    T.t[4 * q + 3] = v.w;
  }
}

// subfield table (tower image): plane 0 and dword 0 of plane 1
__device__ __forceinline__ void lds_tab_at(const uint8_t *lds, uint32_t lin, SubTab &T) {
  T.t[4] = *reinterpret_cast<const uint32_t *>(lds + Tabs::kPlane + lin);
  const uint4 v = *reinterpret_cast<const uint4 *>(lds + lin);
  T.t[0] = v.x;
  T.t[1] = v.y;
  T.t[2] = v.z;
  T.t[3] = v.w;
}
// table type of stage m in a tower image whose subfield stages start at SM
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
// F9 tables (F9 image kind 1) where F is set
template <int M, int SM, bool F>
using TabAtF = std::conditional_t<F, F9Tab, TabAt<M, SM>>;
constexpr bool kF9 = true;

__device__ __forceinline__ void lds_tab_at(const uint8_t *lds, uint32_t lin, F9Tab &T) {
#pragma unroll
  for (int q = 3; q >= 0; --q) {
    const uint4 v = *reinterpret_cast<const uint4 *>(lds + q * Tabs::kPlane + lin);
    T.t[4 * q] = v.x;
    T.t[4 * q + 1] = v.y;
    T.t[4 * q + 2] = v.z;
    T.t[4 * q + 3] = v.w;
  }
}

// skew index of the block holding position pos_a at stage m (additive_fft.hpp:108,126)
__device__ __forceinline__ uint32_t skew_idx(uint32_t pos_a, int m, uint32_t offset) {
  const uint32_t d = 1u << m;
  return (pos_a & ~(2 * d - 1)) + d - 1 + offset;
}

// Table loads are software-pipelined: the next butterfly group's table is
// requested before the current group's multiplies, so a wave keeps one 80-B
// table load in flight instead of stalling on each (2 x 20 VGPRs).
// radix-8 pass over 3 consecutive position bits b0..b0+2 held in registers:
// pos(r) = base | (r << b0).  Inverse: stages b0, b0+1, b0+2.
// Stages >= SM (the tower image's subfield stages) multiply with SubTab, and
// so do stages SL <= m < SM, whose skews the caller knows to be subfield too:
// those read the stage-2 slot of the same element, 2 ((off | pos) >> (m + 1))
// (alias index ((off | pos) >> (m + 1)) << 3 | 3).
template <int b0, int SM, int SL>
struct PassIdx {
  static constexpr bool A0 = b0 < SM && b0 >= SL, A1 = b0 + 1 < SM && b0 + 1 >= SL;
  uint32_t lb, la0, la1, off;
  __device__ __forceinline__ PassIdx(uint32_t base, uint32_t off_) : off(off_) {
    lb = tlin(base & ~((2u << b0) - 1));  // lane part of every index below
    la0 = A0 ? tlin(((base | off) >> (b0 + 1)) << 3) : 0u;
    la1 = A1 ? tlin(((base | off) >> (b0 + 2)) << 3) : 0u;
  }
  __device__ __forceinline__ uint32_t i0(int rr) const {
    return A0 ? la0 ^ tlin((uint32_t(rr) << 3) | 3u) : lb ^ tlin(skew_idx(uint32_t(2 * rr) << b0, b0, off));
  }
  __device__ __forceinline__ uint32_t i1(int hh) const {
    return A1 ? la1 ^ tlin((uint32_t(hh) << 3) | 3u) : lb ^ tlin(skew_idx(uint32_t(4 * hh) << b0, b0 + 1, off));
  }
  __device__ __forceinline__ uint32_t i2() const { return lb ^ tlin(skew_idx(0, b0 + 2, off)); }
};

template <int b0, int SM, int SL = SM>
__device__ __forceinline__ void ipass3(State &s, const uint8_t *tabs, uint32_t base, uint32_t off) {
  {
    TabAt<b0, SL> Ta0, Tb0;
    TabAt<b0 + 1, SL> Ta1, Tb1;
    TabAt<b0 + 2, SL> Ta2;
    const PassIdx<b0, SM, SL> ix(base, off);
    const auto i0 = [&](int rr) { return ix.i0(rr); };
    const auto i1 = [&](int hh) { return ix.i1(hh); };
    const uint32_t i2 = ix.i2();
    lds_tab_at(tabs, i0(0), Ta0);
    lds_tab_at(tabs, i0(1), Tb0);
    ibfly(s, 0, 1, Ta0);
    lds_tab_at(tabs, i0(2), Ta0);
    ibfly(s, 2, 3, Tb0);
    lds_tab_at(tabs, i0(3), Tb0);
    ibfly(s, 4, 5, Ta0);
    lds_tab_at(tabs, i1(0), Ta1);
    ibfly(s, 6, 7, Tb0);
    lds_tab_at(tabs, i1(1), Tb1);
    ibfly(s, 0, 2, Ta1);
    ibfly(s, 1, 3, Ta1);
    lds_tab_at(tabs, i2, Ta2);
    ibfly(s, 4, 6, Tb1);
    ibfly(s, 5, 7, Tb1);
#pragma unroll
    for (int r = 0; r < 4; ++r) ibfly(s, r, r + 4, Ta2);
  }
}

// forward: stages b0+2, b0+1, b0 (F0 / F1: stage b0 / b0 + 1 with F9 tables)
template <int b0, int SM, int SL = SM, bool F0 = false, bool F1 = false>
__device__ __forceinline__ void fpass3(State &s, const uint8_t *tabs, uint32_t base, uint32_t off) {
  {
    TabAtF<b0, SL, F0> Ta0, Tb0;
    TabAtF<b0 + 1, SL, F1> Ta1, Tb1;
    TabAt<b0 + 2, SL> Ta2;
    const PassIdx<b0, SM, SL> ix(base, off);
    const auto i0 = [&](int rr) { return ix.i0(rr); };
    const auto i1 = [&](int hh) { return ix.i1(hh); };
    const uint32_t i2 = ix.i2();
    lds_tab_at(tabs, i2, Ta2);
    lds_tab_at(tabs, i1(0), Tb1);
#pragma unroll
    for (int r = 0; r < 4; ++r) fbfly(s, r, r + 4, Ta2);
    lds_tab_at(tabs, i1(1), Ta1);
    fbfly(s, 0, 2, Tb1);
    fbfly(s, 1, 3, Tb1);
    lds_tab_at(tabs, i0(0), Tb0);
    fbfly(s, 4, 6, Ta1);
    fbfly(s, 5, 7, Ta1);
    lds_tab_at(tabs, i0(1), Ta0);
    fbfly(s, 0, 1, Tb0);
    lds_tab_at(tabs, i0(2), Tb0);
    fbfly(s, 2, 3, Ta0);
    lds_tab_at(tabs, i0(3), Ta0);
    fbfly(s, 4, 5, Tb0);
    fbfly(s, 6, 7, Ta0);
  }
}

// layout C: register bit0 = p6, bit1 = p7, bit2 = p5 (passenger); stages 6, 7
// have lane-uniform skews.  Only the IFFT at index 0 runs here, where the
// block at j = d of a stage has skew skews[d - 1] = 0xFFFF (inverse_afft skips
// the multiply): stage 7 (j = 128) and stage 6's first block (j = 64) are
// b ^= a only.
__device__ __forceinline__ void ipassC0(State &s, const uint8_t *tabs) {
  SubTab Tb;  // stage 6 >= tower_sub_min(0)
  lds_tab_at(tabs, tlin(skew_idx(1u << 7, 6, 0)), Tb);
  bxor(s, 0, 1);  // stage 6, j = 64
  bxor(s, 4, 5);
  ibfly(s, 2, 3, Tb);  // stage 6, j = 192
  ibfly(s, 6, 7, Tb);
  bxor(s, 0, 2);  // stage 7, j = 128
  bxor(s, 1, 3);
  bxor(s, 4, 6);
  bxor(s, 5, 7);
}

__device__ __forceinline__ void fpassC(State &s, const State &c, const uint8_t *tabs, uint32_t off) {
  SubTab Ta, Tb;  // stages 7, 6 >= tower_sub_min(0), tower_sub_min(1)
  lds_tab_at(tabs, tlin(skew_idx(0, 7, off)), Ta);
  lds_tab_at(tabs, tlin(skew_idx(0, 6, off)), Tb);
  fbfly_from(s, c, 0, 2, Ta);
  fbfly_from(s, c, 1, 3, Ta);
  fbfly_from(s, c, 4, 6, Ta);
  fbfly_from(s, c, 5, 7, Ta);
  lds_tab_at(tabs, tlin(skew_idx(1u << 7, 6, off)), Ta);
  fbfly(s, 0, 1, Tb);
  fbfly(s, 4, 5, Tb);
  fbfly(s, 2, 3, Ta);
  fbfly(s, 6, 7, Ta);
}

// ---- own-region staging: wave w stages its 8 pieces x 256 rows in
// its own 4 KB exchange region, 16 B per row (half = inst).  Row v sits in
// 256-byte block v >> 4 at 16-B slot (v ^ (v >> 4) ^ w) & 15: the 16 lanes that
// read one row from the 16 regions hit 16 distinct slots (conflict free) and
// the layout-A writes are 2-way.  A wave only ever writes its own region, so
// the next write needs a barrier only after the other waves' row reads.
__host__ __device__ constexpr uint32_t soff(uint32_t v, uint32_t w) {
  return ((v >> 4) << 8) | (((v ^ (v >> 4) ^ w) & 15) << 4);
}

__device__ __forceinline__ void stage_own(const State &s, uint8_t *xch, uint32_t q,
                                          uint32_t inst, uint32_t wave) {
#pragma unroll
  for (int r = 0; r < 8; ++r)
    *reinterpret_cast<uint2 *>(xch + soff(posA(q, r), wave) + 8 * inst) =
        to_be(s.l[0][r], s.h[0][r]);
}

// one 16-B chunk (8 pieces) of a shard row at any even address: the widest
// stores the address allows, 2-B stores for a partial chunk (packed batches
// with tight, unaligned row pitches)
__device__ __forceinline__ void store_chunk_any(uint8_t *dst, const uint4 val, uint64_t nvalid) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(dst);
  if (nvalid >= 8) {
    if ((a & 15) == 0) {
      *reinterpret_cast<uint4 *>(dst) = val;
      return;
    }
    if ((a & 7) == 0) {
      reinterpret_cast<uint2 *>(dst)[0] = make_uint2(val.x, val.y);
      reinterpret_cast<uint2 *>(dst)[1] = make_uint2(val.z, val.w);
      return;
    }
    if ((a & 3) == 0) {
      reinterpret_cast<uint32_t *>(dst)[0] = val.x;
      reinterpret_cast<uint32_t *>(dst)[1] = val.y;
      reinterpret_cast<uint32_t *>(dst)[2] = val.z;
      reinterpret_cast<uint32_t *>(dst)[3] = val.w;
      return;
    }
  }
  const uint32_t w[4] = {val.x, val.y, val.z, val.w};
#pragma unroll
  for (int e = 0; e < 8; ++e)
    if (uint64_t(e) < nvalid) *reinterpret_cast<uint16_t *>(dst + 2 * e) = uint16_t(w[e >> 1] >> (16 * (e & 1)));
}

// all waves: rows [s0, s0 + 256) from the 16 regions -> shards; lane =
// (row-in-4, source wave c = 16-B chunk of pieces [8c, 8c + 8)): pieces
// piece0 + 8c of the tile's payload (SH), or, packed, pieces [pc, pc + 8) of
// the payload bc that owns flattened slot tile * TILE + 8c (computed here, not
// kept live across the FFTs)
// The common case of store_own, decided once (uniform): 16-B aligned rows, the
// whole tile inside the payload and all 256 rows below n_validators -- one
// aligned 16-B streaming store per lane and row, addresses stepped, no
// per-lane tests (the general form made the compiler merge its two store
// shapes into a 4-B + a misaligned 12-B store per chunk)
__device__ __forceinline__ bool rows_fast_ok(const uint8_t *SH, uint64_t sstride, uint32_t s0, int nv,
                                             uint64_t piece0, uint64_t npieces) {
  return ((sstride | reinterpret_cast<uintptr_t>(SH)) & 15) == 0 && piece0 + TILE <= npieces &&
         int(s0) + 256 <= nv;
}
__device__ __forceinline__ void store_rows_fast(const uint8_t *xbase, uint8_t *SH, uint64_t sstride,
                                                uint32_t s0, uint64_t piece0, uint32_t wave, uint32_t lane) {
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  const uint32_t c = lane & 15;
  const uint32_t v0 = wave * 4 + (lane >> 4);
  const uint32_t sa = lds_addr(xbase + c * XCH_BYTES) + soff(v0, c);
  uint8_t *dst = SH + uint64_t(s0 + v0) * sstride + 2 * (piece0 + 8 * c);
  const uint64_t dstep = uint64_t(4 * WAVES) * sstride;
#pragma unroll
  for (int it = 0; it < 256 / (4 * WAVES); ++it) {  // soff is GF(2)-linear in v = it * 4 WAVES | v0
    const v4u val = *(const __attribute__((address_space(3))) v4u *)(uintptr_t(sa ^ soff(uint32_t(it) * 4 * WAVES, 0)));
    // streaming (non-temporal): rows are written once, not re-read
    __builtin_nontemporal_store(val, reinterpret_cast<v4u *>(dst + it * dstep));
  }
}

template <bool PACKED>
__device__ __forceinline__ void store_own(const uint8_t *xbase, uint8_t *SH, uint64_t sstride,
                                          uint32_t s0, int nv, uint64_t piece0, uint64_t npieces,
                                          uint32_t wave, uint32_t lane, uint64_t tile, uint32_t npp8,
                                          uint32_t batch) {
  asm volatile("" : "+v"(lane));  // recomputed here, not kept live across the FFTs
  if constexpr (!PACKED) {
    if (rows_fast_ok(SH, sstride, s0, nv, piece0, npieces)) {
      store_rows_fast(xbase, SH, sstride, s0, piece0, wave, lane);
      return;
    }
  }
  const uint32_t c = lane & 15;
  uint64_t p = piece0 + 8 * c;
  if constexpr (PACKED) {
    const uint32_t gc = uint32_t(tile) * TILE + 8 * c, bc = gc / npp8;
    p = bc < batch ? gc % npp8 : npieces;  // past the batch: nothing to store
    SH += uint64_t(bc < batch ? bc : 0) * uint64_t(nv) * sstride;
  }
  const bool wide = ((sstride | reinterpret_cast<uintptr_t>(SH)) & 15) == 0;  // 16-B aligned rows
  const uint8_t *src = xbase + c * XCH_BYTES;
#pragma unroll
  for (int it = 0; it < 256 / (4 * WAVES); ++it) {
    const uint32_t v = uint32_t(it) * 4 * WAVES + wave * 4 + (lane >> 4);
    const uint4 val = *reinterpret_cast<const uint4 *>(src + soff(v, c));
    const uint32_t shard = s0 + v;
    if (int(shard) >= nv) continue;
    uint8_t *dst = SH + uint64_t(shard) * sstride + 2 * p;
    if constexpr (PACKED) {
      if (p < npieces) store_chunk_any(dst, val, npieces - p);
    } else if (p + 8 <= npieces) {
      if (wide) {
        *reinterpret_cast<uint4 *>(dst) = val;
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
}

// packed waves (PK = 2): this wave's 8 staged pieces x 256 rows [s0, s0 + 256)
// -> shards, lane = (piece e = lane & 7, rows lane / 8 + 8 k); piece e of the
// task is flattened piece 8 task + e, i.e. piece p of payload b (each piece
// its own payload when payloads are one piece long): 2-B stores
__device__ __forceinline__ void store_wave(const uint8_t *xch, uint8_t *shards, uint64_t sstride,
                                           uint32_t s0, int nv, uint32_t task, uint32_t npp,
                                           uint32_t batch, uint32_t wave, uint32_t lane) {
  asm volatile("" : "+v"(lane));
  const uint32_t e = lane & 7, g = 8 * task + e, b = g / npp, p = g % npp;
  if (b >= batch) return;
  uint8_t *dst = shards + uint64_t(b) * uint64_t(nv) * sstride + 2 * uint64_t(p);
#pragma unroll 8
  for (int k = 0; k < 32; ++k) {
    const uint32_t v = (lane >> 3) + 8 * k, shard = s0 + v;
    if (int(shard) >= nv) break;  // rows increase with k
    *reinterpret_cast<uint16_t *>(dst + uint64_t(shard) * sstride) =
        *reinterpret_cast<const uint16_t *>(xch + soff(v, wave) + 2 * e);
  }
}

}  // namespace

// N = n: 1024 (n_validators 766..1024) or 2048 (1025..1533); the cosets at
// 1024 and above use LDS table image 1 (skews 1024 .. 2046, DevTables::timg)
// at offset sh - 1024, reloaded by LDS-DMA between the two coset loops
// PK = 1, packed tiles (n = 2048 with small payloads, or payload / shard
// pitches the 16-B path cannot take): tiles run over the flattened piece space
// of the batch, payload b owning slots [b * npp8, b * npp8 + npieces) with
// npp8 = pieces rounded up to 8, so a wave's 8 pieces (and each 16-B chunk of
// a staged row) belong to one payload; loads and stores take any alignment.
// PK = 2, packed waves (n = 1024, same cases): the waves run independently
// over tasks of 8 consecutive pieces of the exactly flattened piece space
// (payload b owns pieces [b * npp, (b + 1) * npp)), each staging and storing
// its own rows (2-B stores, any payload per piece), no workgroup barrier in the
// loop: 4096 one-piece payloads are 512 wave tasks (about 2 per CU) instead of
// 4096 tiles (or 256 tiles of 8x-rounded slots).
template <int N, int PK>
__global__ void __launch_bounds__(THREADS) encode_k256(const uint8_t *__restrict__ payloads,
                                                       uint64_t plen, uint64_t pstride,
                                                       uint8_t *__restrict__ shards, uint64_t slen,
                                                       uint64_t sstride, int nv, uint32_t batch,
                                                       uint32_t npp8, DevTables t) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  uint8_t *tabs = lds;
  const uint32_t tid0 = threadIdx.x;
  uint8_t *stg = lds + TAB_REGION;

  // resident multiply tables for skew indices 0..1022 (all FFTs of k=256, n=1024)
  // multiply tables for skew indices 0..1022: the prebuilt LDS image 0
  // (DevTables::timg), one coalesced 80 KB copy instead of a 1023-entry gather
  // through the skews (that gather was ~10 us of every launch; small calls pay it)
  // the tower images: the transforms run in tower coordinates
  // (image 0 as its F9 variant kind 1: DESIGN.md §2.8)
  const uint8_t *const img0 = kF9 ? t.timg_f9 + kTabImageBytes : t.timg_t;
  Tabs::copy_image<THREADS>(tabs, img0, tid0);
  __syncthreads();
  [[maybe_unused]] int img = 0;
  [[maybe_unused]] const auto load_image = [&](int q) {  // LDS-DMA: no VGPRs (the kernel is at 128)
    lds_barrier();  // every wave is done with the current tables
    Tabs::dma_image<THREADS>(tabs, q == 0 ? img0 : t.timg_t + q * kTabImageBytes, tid0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
  };

  constexpr bool PACKED = PK == 1;
  const uint64_t npieces = slen / 2;
  const uint32_t tiles_pp = uint32_t((npieces + TILE - 1) / TILE);
  const uint64_t total = PK == 2   ? (npieces * batch + 7) / 8
                         : PACKED ? (uint64_t(npp8) * batch + TILE - 1) / TILE
                                  : uint64_t(tiles_pp) * batch;
  // PK = 2: "tile" = this wave's task (a wave-uniform, scalar index)
  const uint32_t wave_s = __builtin_amdgcn_readfirstlane(tid0 >> 6);
  // (task t on workgroup t % grid, wave t / grid: a small batch spreads over
  // every CU instead of filling the first ones' waves; a wave's latency, not
  // the CU's throughput, bounds it)
  const uint64_t first = PK == 2 ? uint64_t(wave_s) * gridDim.x + blockIdx.x : blockIdx.x;
  const uint64_t step = PK == 2 ? uint64_t(gridDim.x) * WAVES : gridDim.x;
  // region hand-over: a workgroup barrier (other waves read this wave's staged
  // rows), or in PK = 2 the wave's own program order
  const auto rsync = [&]() __attribute__((always_inline)) {
    if constexpr (PK == 2) {
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
    } else {
      lds_barrier();
    }
  };
  TileWalk walk(first, step, tiles_pp);  // PK = 0: payload and tile of `tile`
  for (uint64_t tile = first; tile < total; tile += step, walk.advance()) {
    // lane ids made opaque per tile: per-lane LDS addresses are recomputed in the
    // loop instead of being hoisted out of it and spilled
    uint32_t tid = tid0;
    asm volatile("" : "+v"(tid));
    const uint32_t lane = tid & 63, wave = tid >> 6;
    const uint32_t inst = lane >> 5, q = lane & 31;
    uint8_t *xch = lds + TAB_REGION + wave * XCH_BYTES;
    XBase xb;
    xb.a = mswz(ulaneA(q, inst));
    xb.b = mswz(ulaneB(q, inst));
    xb.c = mswz(ulaneC(q, inst));
    // unpacked: the tile is pieces [piece0, piece0 + 128) of payload b;
    // packed: wave w's 8 pieces are pieces [pw, pw + 8) of payload bw (uniform),
    // and the chunk a lane stores (source wave c) is pieces [pc, pc + 8) of bc
    uint64_t b, piece0, bw = 0, pw = 0;
    if constexpr (PACKED) {
      const uint32_t gw = uint32_t(tile) * TILE + 8 * wave;  // < 2^32 (launch check)
      bw = gw / npp8;
      pw = gw % npp8;
      b = bw;
      piece0 = pw;
    } else {
      b = walk.b;
      piece0 = walk.i * TILE;
    }
    const uint8_t *P = payloads + b * pstride;
    uint8_t *SH = PACKED ? shards : shards + b * uint64_t(nv) * sstride;  // packed: per chunk

    const auto store = [&](uint32_t s0) __attribute__((always_inline)) {
      // the row stores (LDS reads + global stores) at raised issue priority:
      // a wave's stores leave before the other waves' next transform
      // (B = 4096 encode 7.58 -> 7.39 ms; priority 3 the same)
      __builtin_amdgcn_s_setprio(1);
      if constexpr (PK == 2)
        store_wave(xch, shards, sstride, s0, nv, uint32_t(tile), uint32_t(npieces), batch, wave, lane);
      else
        store_own<PACKED>(stg, SH, sstride, s0, nv, piece0, npieces, wave, lane, tile, npp8, batch);
      __builtin_amdgcn_s_setprio(0);
    };

    // A wave none of whose 8 pieces exist (the last, partial tile of a payload:
    // 1 MB is 1954 pieces, its 16th tile has 34) skips the transforms and only
    // takes part in the barriers, the image loads and the row stores of the
    // others, in the same order as below (wave-uniform branch)
    if constexpr (PK == 0) {
      if (piece0 + 8 * wave_s >= npieces) {
        rsync();  // tile start
        rsync();  // systematic rows staged
        store(0);
        if constexpr (N > 1024) {
          if (img != 0) {
            load_image(0);
            img = 0;
          }
        }
        rsync();  // after IFFT pass A
        const auto coset_idle = [&](uint32_t sh) __attribute__((always_inline)) {
          rsync();  // after pass C
          rsync();  // rows staged
          store(sh);
          __builtin_amdgcn_sched_barrier(0);
        };
        coset_idle(K);
        for (uint32_t sh = 2 * K; sh < 1024u && int(sh) < nv; sh += K) coset_idle(sh);
        if constexpr (N > 1024) {
          for (uint32_t sh = 1024u; sh < uint32_t(N) && int(sh) < nv; sh += K) {
            if (sh == 1024u) {
              load_image(1);
              img = 1;
            }
            coset_idle(sh);
          }
        }
        continue;
      }
    }

    // ---- load 8 pieces x 16 bytes (positions 8q..8q+7), zero past plen
    State s;
#pragma unroll
    for (int g = 0; g < GP; ++g) {
      uint4 d[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if constexpr (PK == 2) {
          const uint32_t gp = uint32_t(tile) * 8 + inst * 4 * GP + g * 4 + u;  // < 2^32 (launch check)
          const uint32_t pb = gp / uint32_t(npieces), piece = gp % uint32_t(npieces);
          const uint64_t off = uint64_t(piece) * 2 * K + 16 * q;
          const bool ok = pb < batch && off < plen;
          d[u] = load16_any(payloads + uint64_t(ok ? pb : 0) * pstride + (ok ? off : 0), ok ? plen - off : 0);
        } else if constexpr (PACKED) {
          const uint64_t piece = pw + inst * 4 * GP + g * 4 + u;
          const uint64_t off = piece * 2 * K + 16 * q;
          const bool ok = bw < batch && piece < npieces && off < plen;
          d[u] = load16_any(P + (ok ? off : 0), ok ? plen - off : 0);
        } else {
          const uint64_t piece = piece0 + wave * 8 * GP + inst * 4 * GP + g * 4 + u;
          const uint64_t off = piece * 2 * K + 16 * q;
          if (off + 16 <= plen) {
            d[u] = *reinterpret_cast<const uint4 *>(P + off);
          } else {
            uint32_t w[4] = {0, 0, 0, 0};
            for (uint64_t e = off; e < plen && e < off + 16; ++e)
              w[(e - off) >> 2] |= uint32_t(P[e]) << (8 * ((e - off) & 3));
            d[u] = make_uint4(w[0], w[1], w[2], w[3]);
          }
        }
      }
      // 4x4 byte transposes: dword j of each piece = (hi_{2j}, lo_{2j}, hi_{2j+1}, lo_{2j+1})
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t D0 = (&d[0].x)[j], D1 = (&d[1].x)[j], D2 = (&d[2].x)[j], D3 = (&d[3].x)[j];
        const uint32_t t0 = vperm(D1, D0, 0x05010400u), t1 = vperm(D1, D0, 0x07030602u);
        const uint32_t u0 = vperm(D3, D2, 0x05010400u), u1 = vperm(D3, D2, 0x07030602u);
        s.h[g][2 * j] = vperm(u0, t0, 0x05040100u);
        s.l[g][2 * j] = vperm(u0, t0, 0x07060302u);
        s.h[g][2 * j + 1] = vperm(u1, t1, 0x05040100u);
        s.l[g][2 * j + 1] = vperm(u1, t1, 0x07060302u);
      }
    }

    // ---- systematic shards 0..255 = the data symbols (poly_encoder.hpp:239)
    rsync();  // the other waves are done reading this region (last tile)
    stage_own(s, xch, q, inst, wave);
    rsync();
    store(0);
    __builtin_amdgcn_sched_barrier(0);
    {  // into tower coordinates
      const TowerK tk = tower_k();
#pragma unroll
      for (int r = 0; r < 8; ++r) s.l[0][r] = tower_lo(s.l[0][r], s.h[0][r], tk);
    }

    // ---- IFFT_256 (index 0): passes A (bits 0-2), B (3-5), C (6-7)
    if constexpr (N > 1024) {
      if (img != 0) {  // the previous tile ended on image 1
        load_image(0);
        img = 0;
      }
    }
    // index 0, positions < 256: every skew is subfield (stages 0, 1 by alias)
    ipass3<0, tower_sub_min(0), 0>(s, tabs, posA(q, 0), 0);
    rsync();  // systematic rows read out of the regions
    exchange<LA, LB>(s, xch, xb);
    ipass3<3, tower_sub_min(0)>(s, tabs, posB(q, 0), 0);
    exchange<LB, LC>(s, xch, xb);
    ipassC0(s, tabs);
    State coef = s;

    // ---- FFT_256 at each coset shift (encodeLow, poly_encoder.hpp:229-237)
    // sm: the tower image's first subfield stage (std::integral_constant)
    // sl: first subfield stage of this coset's pass A (<= SM: aliased stages)
    // f0 / f1: pass A's stage 0 / 1 with F9 tables (std::integral_constant)
    const auto coset = [&](auto sm, auto sl, auto f0, auto f1, const uint32_t sh, const uint32_t off)
                           __attribute__((always_inline)) {
      constexpr int SM = decltype(sm)::value, SL = decltype(sl)::value;
      constexpr bool F0 = decltype(f0)::value, F1 = decltype(f1)::value;
      // coef made opaque in place (no copy): keeps the compiler from hoisting
      // the first stage's selector masks out of the coset loop (that costs ~50
      // VGPRs and forces spills); pass C's stage 7 reads it and writes s
#pragma unroll
      for (int r = 0; r < 8; ++r) asm volatile("" : "+v"(coef.l[0][r]), "+v"(coef.h[0][r]));
      fpassC(s, coef, tabs, off);
      rsync();  // previous coset's rows read out
      exchange<LC, LB>(s, xch, xb);
      fpass3<3, SM>(s, tabs, posB(q, 0), off);
      exchange<LB, LA>(s, xch, xb);
      fpass3<0, SM, SL, F0, F1>(s, tabs, posA(q, 0), off);
      {  // back to symbol coordinates
        const TowerK tk = tower_k();
#pragma unroll
        for (int r = 0; r < 8; ++r) s.l[0][r] = tower_lo(s.l[0][r], s.h[0][r], tk);
      }
      stage_own(s, xch, q, inst, wave);
      rsync();
      store(sh);
      __builtin_amdgcn_sched_barrier(0);
    };
    using Sub0 = std::integral_constant<int, tower_sub_min(0)>;
    using Sub1 = std::integral_constant<int, tower_sub_min(1)>;
    using F9on = std::integral_constant<bool, kF9>;
    using F9off = std::integral_constant<bool, false>;
    // coset 1 (index 256): stage 1 skews are 128 + 2 (pos >> 2), subfield;
    // stage 0's elements 256..510 take F9 tables
    coset(Sub0(), std::integral_constant<int, 1>(), F9on(), F9off(), K, K);  // (nv > 256 for k = 256)
    // cosets 2, 3: stage 1's elements 256..510 take F9 tables
    for (uint32_t sh = 2 * K; sh < 1024u && int(sh) < nv; sh += K) coset(Sub0(), Sub0(), F9off(), F9on(), sh, sh);
    if constexpr (N > 1024) {
      for (uint32_t sh = 1024u; sh < uint32_t(N) && int(sh) < nv; sh += K) {
        if (sh == 1024u) {
          load_image(1);
          img = 1;
        }
        coset(Sub1(), Sub1(), F9off(), F9off(), sh, sh & 1023u);
      }
    }
  }
}

bool k256_applicable(const CodeParams &p) { return p.k == 256 && (p.n == 1024 || p.n == 2048); }

// packed tiles: pieces per payload below one tile, or pitches / bases the
// unpacked kernel's 16-B loads and 8-B stores cannot take (any even shard
// pitch and shard base, any payload pitch and base)
bool k256_packed(size_t plen, size_t pstride, size_t batch, uintptr_t pay, uintptr_t sh, size_t sstride) {
  const size_t npp = (plen + 2 * K - 1) / (2 * K);
  const bool aligned = pay % 16 == 0 && sh % 8 == 0 && (batch == 1 || pstride % 16 == 0) && sstride % 8 == 0;
  return !aligned || npp < size_t(TILE);
}

bool k256_packed_ok(size_t plen, size_t batch, uintptr_t sh, size_t sstride) {
  const size_t npp8 = ((plen + 2 * K - 1) / (2 * K) + 7) / 8 * 8;
  return sh % 2 == 0 && sstride % 2 == 0 && npp8 * batch + TILE < (size_t(1) << 32);
}  // (npp8 >= npp: also bounds the exactly flattened piece space of PK = 2)

size_t k256_scratch_bytes(const CodeParams &) { return 256; }  // the unpacked kernels' tile counter

hipError_t launch_encode_k256(const CodeParams &p, const DevTables &t, const uint8_t *d_payloads,
                              size_t plen, size_t pstride, size_t batch, uint8_t *d_shards,
                              size_t sstride, void *scratch, hipStream_t s) {
  int cus = 0;
  const bool packed = k256_packed(plen, pstride, batch, reinterpret_cast<uintptr_t>(d_payloads),
                                  reinterpret_cast<uintptr_t>(d_shards), sstride);
  if (p.n == 1024 && !packed)
    return launch_encode_k256w(p, t, d_payloads, plen, pstride, batch, d_shards, sstride, scratch, s);
  if (p.n == 2048 && !packed)  // round 6: the two-workgroups-per-CU model (enc_kw.hip)
    return launch_encode_kw(p, t, d_payloads, plen, pstride, batch, d_shards, sstride, scratch, s);
  if (packed && !k256_packed_ok(plen, batch, reinterpret_cast<uintptr_t>(d_shards), sstride))
    return hipErrorInvalidValue;
  const void *fn = p.n == 1024 ? reinterpret_cast<const void *>(&encode_k256<1024, 2>)
                               : (packed ? reinterpret_cast<const void *>(&encode_k256<2048, 1>)
                                         : reinterpret_cast<const void *>(&encode_k256<2048, 0>));
  if (const hipError_t e = prepare_kernel(fn, LDS_BYTES, &cus); e != hipSuccess) return e;
  const size_t sl = shard_len(p.k, plen);
  const size_t npp8 = (sl / 2 + 7) / 8 * 8;
  const size_t tiles = !packed       ? (sl / 2 + TILE - 1) / TILE * batch
                       : p.n == 1024 ? ((sl / 2) * batch + 7) / 8  // wave tasks, spread over the CUs
                                     : (npp8 * batch + TILE - 1) / TILE;
  const unsigned grid = unsigned(tiles < size_t(cus) ? tiles : size_t(cus));
#define ECAMD_K256(NN, PK)                                                                       \
  hipLaunchKernelGGL((encode_k256<NN, PK>), dim3(grid), dim3(THREADS), LDS_BYTES, s, d_payloads,   \
                     uint64_t(plen), uint64_t(pstride), d_shards, uint64_t(sl), uint64_t(sstride), \
                     int(p.nv), uint32_t(batch), uint32_t(npp8), t)
  if (p.n == 1024) {
    ECAMD_K256(1024, 2);  // (packed: the unpacked n = 1024 case is encode_k256w)
  } else {
    if (packed) ECAMD_K256(2048, 1);
    else ECAMD_K256(2048, 0);
  }
#undef ECAMD_K256
  return hipGetLastError();
}

}  // namespace ecamd
