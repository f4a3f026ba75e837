// enc_k1024.hip — encode specialised for k = 1024, n = 4096 (n_validators
// 3070..4096; BASELINE config 4).
//
// encodeLow (poly_encoder.hpp:217-240) for k = 1024 is one IFFT_1024 and up to
// three FFT_1024 at coset shifts 1024 / 2048 / 3072, each with its own 1023
// skews (80 KB of multiply tables).  All 4095 tables do not fit LDS next to the
// exchange regions, so one persistent launch cycles the four table sets
// through LDS per tile (LDS-DMA, hidden behind shard stores; see the kernel).
//
// Tile = 32 consecutive pieces (piece = 2048 payload bytes = 1024 symbols);
// wave w owns pieces [4w, 4w + 4) as ONE byte-planar group, run through
// tf1024.hpp's register passes.  The IFFT coefficients stay in registers for
// every coset (round 5: until then two groups per wave and a 64-piece tile,
// with the coefficients of cosets 2 and 3 read back from a per-workgroup L2
// scratch slot: 1.59x the algorithmic HBM traffic).
// Shard rows (64 B per row per tile) are staged in the waves' own regions,
// 8 B per row, and stored as 16 B per lane from two adjacent regions.
// Tiles are taken from a per-launch counter (dynamic schedule: the static
// grid-stride split gave every 8th workgroup all the payloads' partial last
// tiles, so they ended ~10% apart).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>

#include "ec_kernels.hpp"
#include "tf1024.hpp"

namespace ecamd {
namespace {

using namespace tf;
constexpr int K = 1024;
constexpr int WAVES = 8;
constexpr int THREADS = 64 * WAVES;
constexpr int TILE = 4 * WAVES;  // pieces: one byte-planar group per wave
constexpr uint32_t SLOT = Tabs::kBytes + WAVES * REG_BYTES;  // the next tile's index
constexpr int LDS_BYTES = int(SLOT + 16);
static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");

// global stores per lane of store_rows' fast path: the hand-written
// s_waitcnt vmcnt(kStoreIts) in the kernel rely on it (tests/test_asm_checks.py
// counts them in the built code)
constexpr int kStoreIts = 1024 / (16 * WAVES);
static_assert(kStoreIts == 8, "the vmcnt(8) waits below");

// own-region staging slot of row v (0..1023), 8 B: the store reads (lane =
// row-in-16 << 2 | 16-B chunk c = regions 2c, 2c + 1) spread over the banks
__host__ __device__ constexpr uint32_t soff(uint32_t v) {
  return ((v >> 5) << 8) | (((v ^ (v >> 5)) & 31) << 3);
}

// row v of this wave's group -> own region (8 B, big-endian symbols of its 4 pieces)
__device__ __forceinline__ void stage_rows(const S16 &g, uint8_t *my, uint32_t lane) {
  // layout A: position 16 lane + r
  const uint32_t a = lds_addr(my);
#pragma unroll
  for (int r = 0; r < 16; ++r) lds_st2(a + soff(16 * lane + uint32_t(r)), to_be(g.l[r], g.h[r]));
}

// all waves: the 1024 staged rows -> shards row0 + v (rows >= nv skipped);
// lane = (row-in-16, chunk c): 16 B = the 8 B of regions 2c and 2c + 1
__device__ __forceinline__ void store_rows(const uint8_t *regions, uint8_t *SH, uint64_t sstride,
                                           uint32_t row0, int nv, uint64_t piece0,
                                           uint64_t npieces, uint32_t wave, uint32_t lane) {
  asm volatile("" : "+v"(lane));  // recomputed here, not kept live across the FFTs
  const uint32_t c = lane & 3, vl = wave * 16 + (lane >> 2);
  const uint32_t ra = lds_addr(regions) + 2 * c * REG_BYTES;
  const uint64_t p = piece0 + 8 * c;
  const bool wide = ((sstride | reinterpret_cast<uintptr_t>(SH)) & 15) == 0;  // 16-B aligned rows
  // the common case, decided once (uniform): aligned rows, the whole tile inside
  // the payload, all 1024 rows below n_validators
  if (wide && piece0 + TILE <= npieces && int(row0) + 1024 <= nv) {
    uint8_t *dst = SH + uint64_t(row0 + vl) * sstride + 2 * p;
    const uint64_t dstep = uint64_t(16 * WAVES) * sstride;
#pragma unroll
    for (int it = 0; it < 1024 / (16 * WAVES); ++it) {  // soff is GF(2)-linear in v = it * 128 | vl
      const uint32_t o = soff(uint32_t(it) * 16 * WAVES) ^ soff(vl);
      const uint2 x = lds_ld2(ra + o), y = lds_ld2(ra + REG_BYTES + o);
      typedef uint32_t v4u __attribute__((ext_vector_type(4)));
      // streaming (non-temporal): rows are written once, not re-read
      __builtin_nontemporal_store(v4u{x.x, x.y, y.x, y.y}, reinterpret_cast<v4u *>(dst + it * dstep));
    }
    return;
  }
#pragma unroll 2
  for (int it = 0; it < 1024 / (16 * WAVES); ++it) {
    const uint32_t v = uint32_t(it) * 16 * WAVES + vl;
    const uint2 x = lds_ld2(ra + soff(v)), y = lds_ld2(ra + REG_BYTES + soff(v));
    const uint32_t shard = row0 + v;
    if (int(shard) >= nv) continue;
    uint8_t *dst = SH + uint64_t(shard) * sstride + 2 * p;
    const uint32_t w[4] = {x.x, x.y, y.x, y.y};
    if (p + 8 <= npieces) {
      if (wide) {
        *reinterpret_cast<uint4 *>(dst) = make_uint4(w[0], w[1], w[2], w[3]);
      } else {
        reinterpret_cast<uint2 *>(dst)[0] = make_uint2(w[0], w[1]);
        reinterpret_cast<uint2 *>(dst)[1] = make_uint2(w[2], w[3]);
      }
    } else if (p < npieces) {
      for (uint64_t e = 0; e < npieces - p; ++e)
        *reinterpret_cast<uint16_t *>(dst + 2 * e) = uint16_t(w[e >> 1] >> (16 * (e & 1)));
    }
  }
}

// 4 pieces piece_0 .. piece_0 + 3 -> layout A byte-planar (zero past plen):
// lane reads positions 16 lane .. 16 lane + 15 (32 B) of each piece
__device__ __forceinline__ void load_group(S16 &s, const uint8_t *P, uint64_t plen,
                                           uint64_t piece_0, uint32_t lane) {
  uint32_t D[4][8];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const uint64_t off = (piece_0 + u) * 2 * K + 32 * lane;
    if (off + 32 <= plen) {
      const uint4 a = *reinterpret_cast<const uint4 *>(P + off);
      const uint4 b = *reinterpret_cast<const uint4 *>(P + off + 16);
      D[u][0] = a.x; D[u][1] = a.y; D[u][2] = a.z; D[u][3] = a.w;
      D[u][4] = b.x; D[u][5] = b.y; D[u][6] = b.z; D[u][7] = b.w;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) D[u][j] = 0;
      for (uint64_t e = off; e < plen && e < off + 32; ++e)
        D[u][(e - off) >> 2] |= uint32_t(P[e]) << (8 * ((e - off) & 3));
    }
  }
  // dword j of each piece = (hi_{2j}, lo_{2j}, hi_{2j+1}, lo_{2j+1}) -> registers 2j, 2j+1
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t t0 = vperm(D[1][j], D[0][j], 0x05010400u), t1 = vperm(D[1][j], D[0][j], 0x07030602u);
    const uint32_t u0 = vperm(D[3][j], D[2][j], 0x05010400u), u1 = vperm(D[3][j], D[2][j], 0x07030602u);
    s.h[2 * j] = vperm(u0, t0, 0x05040100u);
    s.l[2 * j] = vperm(u0, t0, 0x07060302u);
    s.h[2 * j + 1] = vperm(u1, t1, 0x05040100u);
    s.l[2 * j + 1] = vperm(u1, t1, 0x07060302u);
  }
}

// symbol <-> tower coordinates (an involution)
__device__ __forceinline__ void to_tower(S16 &g) {
  const TowerK tk = tower_k();
#pragma unroll
  for (int r = 0; r < 16; ++r) g.l[r] = tower_lo(g.l[r], g.h[r], tk);
}

// One persistent launch for all four transforms.  The four 80 KB table sets
// take turns in LDS, loaded by LDS-DMA: each coset's set and the next tile's
// index-0 set as soon as every wave is past the previous transform, behind
// that coset's shard stores.
__global__ void __launch_bounds__(THREADS)
    encode_k1024_fused(const uint8_t *__restrict__ payloads, uint64_t plen, uint64_t pstride,
                       uint8_t *__restrict__ shards, uint64_t slen, uint64_t sstride, int nv,
                       uint32_t batch, uint32_t *__restrict__ tick, DevTables t) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  uint8_t *tabs = lds;
  uint8_t *regions = lds + Tabs::kBytes;
  const uint32_t tid0 = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid0 >> 6);
  uint8_t *my = regions + wave * REG_BYTES;
  auto *slot = reinterpret_cast<__attribute__((address_space(3))) volatile uint32_t *>(uintptr_t(SLOT));
  // this workgroup's first tile (no counter: a static grid stride)
  if (tid0 == 0) *slot = tick ? atomicAdd(tick, 1u) : blockIdx.x;
  // cosets 1 .. ncos - 1 start below n_validators (poly_encoder.hpp:229-236)
  const uint32_t ncos = uint32_t(nv + K - 1) / K;

  // tower images: the transforms run in tower coordinates
  Tabs::copy_image<THREADS>(tabs, t.timg_t, tid0);  // index 0 (the IFFT)
  __syncthreads();

  const uint64_t npieces = slen / 2;
  const uint32_t tiles_pp = uint32_t((npieces + TILE - 1) / TILE);
  const uint32_t total = tiles_pp * batch;  // < 2^32 (launch_encode_k1024)
  // thread 0 takes the tile after this one at the tile start and publishes it
  // in the slot after the first barrier that follows its return; every wave
  // reads it after the next barrier; the slot is rewritten only in the next
  // tile, after its start barrier
  uint32_t cur = __builtin_amdgcn_readfirstlane(*slot);
  while (cur < total) {
    uint32_t tid = tid0;
    asm volatile("" : "+v"(tid));
    const uint32_t lane = tid & 63;
    const uint64_t b = cur / tiles_pp;
    const uint64_t piece0 = uint64_t(cur % tiles_pp) * TILE;
    uint32_t taken = 0;
    if (tid0 == 0) taken = tick ? atomicAdd(tick, 1u) : cur + gridDim.x;
    uint8_t *SH = shards + b * uint64_t(nv) * sstride;
    const uint8_t *P = payloads + b * pstride;
    S16 g, coef;
    // a wave none of whose 4 pieces exist (the payload's last, partial tile:
    // 1 MB is 489 pieces, its 16th tile has 9) skips its transforms and only
    // joins the barriers, the table DMAs and the row stores (uniform)
    const bool idle = piece0 + 4 * wave >= npieces;
    if (!idle) load_group(g, P, plen, piece0 + 4 * wave, lane);
    // systematic shards 0..1023 = the data symbols (poly_encoder.hpp:239)
    lds_barrier();  // the other waves are done reading the regions
    if (!idle) stage_rows(g, my, lane);
    lds_barrier();
    store_rows(regions, SH, sstride, 0, nv, piece0, npieces, wave, lane);
    // the index-0 tables (the last tile's DMA, issued before the systematic
    // stores just made: 8 per lane on the fast path, kStoreIts) landed; the
    // regions are free
    const bool fast_rows = ((sstride | reinterpret_cast<uintptr_t>(SH)) & 15) == 0 && piece0 + TILE <= npieces;
    if (fast_rows && K <= nv)
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
    if (!idle) {
      to_tower(g);
      ifft1024<true, tower_sub_min(0)>(g, tabs, my, lane);
#pragma unroll
      for (int r = 0; r < 16; ++r) {  // the coefficients of every coset, kept in registers
        coef.l[r] = g.l[r];
        coef.h[r] = g.h[r];
      }
    }
    if (tid0 == 0) *slot = taken;  // (issued at the tile start: long returned)
    lds_barrier();  // every wave is done with the index-0 tables
    const uint32_t next = __builtin_amdgcn_readfirstlane(*slot);
    // the compiler's own LDS-DMA here (HIDDEN = false, ec_device.hpp
    // lds_dma16): with it hidden this kernel read 3% slower in an in-process
    // A/B (profiles/r06/NOTES.md), the other DMA users 1-3% faster
    Tabs::dma_image<THREADS, false>(tabs, t.timg_t + kTabImageBytes, tid);
    // cs: std::integral_constant coset number (its image's subfield stages)
    const auto coset = [&](auto cs) __attribute__((always_inline)) {
      constexpr uint32_t s = decltype(cs)::value;
      // coset s's tables landed (all waves' slices; issued before the previous
      // coset's row stores, 8 per lane on the fast path) and the regions are free
      if (s > 1 && fast_rows && int(s * K) <= nv) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lds_barrier();
      if (!idle) {
        if constexpr (s > 1) {
          // coef made opaque: copied here, not re-associated into the FFT
#pragma unroll
          for (int r = 0; r < 16; ++r) asm volatile("" : "+v"(coef.l[r]), "+v"(coef.h[r]));
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            g.l[r] = coef.l[r];
            g.h[r] = coef.h[r];
          }
        }
        fft1024<false, tower_sub_min(int(s))>(g, tabs, my, lane);
        to_tower(g);  // back to symbol coordinates
        stage_rows(g, my, lane);
      }
      lds_barrier();  // every wave is past its FFT and staged: the next set (index 0 after the last coset)
      Tabs::dma_image<THREADS, false>(tabs, t.timg_t + (s + 1 < ncos ? s + 1 : 0) * kTabImageBytes, tid);
      store_rows(regions, SH, sstride, s * K, nv, piece0, npieces, wave, lane);
    };
    coset(std::integral_constant<uint32_t, 1>());
    coset(std::integral_constant<uint32_t, 2>());
    if (ncos > 3) coset(std::integral_constant<uint32_t, 3>());
    cur = next;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA outlives the workgroup
}

}  // namespace

bool k1024_applicable(const CodeParams &p) { return p.k == 1024 && p.n == 4096; }

size_t k1024_scratch_bytes(size_t, size_t) { return 256; }  // the tile counter

hipError_t launch_encode_k1024(const CodeParams &p, const DevTables &t, const uint8_t *d_payloads,
                               size_t plen, size_t pstride, size_t batch, uint8_t *d_shards,
                               size_t sstride, void *scratch, hipStream_t s) {
  int cus = 0;
  const size_t sl = shard_len(p.k, plen);
  const size_t tiles = (sl / 2 + TILE - 1) / TILE * batch;
  if (const hipError_t e = prepare_kernel(reinterpret_cast<const void *>(&encode_k1024_fused), LDS_BYTES, &cus);
      e != hipSuccess)
    return e;
  if (tiles >= (size_t(1) << 32) - size_t(2) * cus) return hipErrorInvalidValue;
  // the tile counter (k1024_scratch_bytes); none: the static schedule
  uint32_t *tick = static_cast<uint32_t *>(scratch);
  if (tick)
    if (const hipError_t e = launch_zero_counters(tick, sizeof(uint32_t), s); e != hipSuccess) return e;
  const unsigned grid = unsigned(std::min(tiles, size_t(cus)));
  hipLaunchKernelGGL(encode_k1024_fused, dim3(grid), dim3(THREADS), LDS_BYTES, s, d_payloads,
                     uint64_t(plen), uint64_t(pstride), d_shards, uint64_t(sl), uint64_t(sstride),
                     int(p.nv), uint32_t(batch), tick, t);
  return hipGetLastError();
}

}  // namespace ecamd
