// enc_k1024.hip — encode specialised for k = 1024, n = 4096 (n_validators
// 3070..4096; BASELINE config 4).
//
// encodeLow (poly_encoder.hpp:217-240) for k = 1024 is one IFFT_1024 and up to
// three FFT_1024 at coset shifts 1024 / 2048 / 3072, each with its own 1023
// skews (80 KB of multiply tables).  All 4095 tables do not fit LDS next to the
// exchange regions, so one persistent launch cycles the four table sets
// through LDS per tile (LDS-DMA, hidden behind shard stores; see the kernel).
// (Until round 3: one launch per transform with the coefficients round-tripped
// through HBM)
//
// Tile = 64 consecutive pieces (piece = 2048 payload bytes = 1024 symbols);
// wave w owns pieces [8w, 8w + 8) as two byte-planar groups of 4, each run
// through tf1024.hpp's register passes.  Shard rows (128 B per row per tile)
// are staged in two halves of 512 rows through the waves' own regions and
// stored as 16 B per lane, 128-B row segments.
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
constexpr int TILE = 8 * WAVES;  // pieces
constexpr int LDS_BYTES = Tabs::kBytes + WAVES * REG_BYTES;
static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
constexpr size_t SCRATCH_PER_WG = size_t(WAVES) * 2 * 16 * 64 * sizeof(uint2);  // a tile's coefficients
constexpr size_t kMaxGrid = 1024;  // workgroups of the launch (>= the CU count)

// own-region staging slot of row v (0..511) of wave w: the 8 lanes reading one
// row from the 8 regions hit 8 distinct 16-B slots
__host__ __device__ constexpr uint32_t soff(uint32_t v, uint32_t w) {
  return ((v >> 4) << 8) | (((v ^ (v >> 4) ^ w) & 15) << 4);
}

// rows 16 (lane & 31) + r of the lanes of half hf -> own region (16 B: groups 0, 1)
__device__ __forceinline__ void stage_half(const S16 &g0, const S16 &g1, uint8_t *my,
                                           uint32_t lane, uint32_t wave, uint32_t hf) {
  if ((lane >> 5) != hf) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const uint2 a = to_be(g0.l[r], g0.h[r]), b = to_be(g1.l[r], g1.h[r]);
    *reinterpret_cast<uint4 *>(my + soff(16 * (lane & 31) + uint32_t(r), wave)) =
        make_uint4(a.x, a.y, b.x, b.y);
  }
}

// all waves: 512 staged rows -> shards row0 + v; lane = (row-in-8, source wave c)
__device__ __forceinline__ void store_half(const uint8_t *regions, uint8_t *SH, uint64_t sstride,
                                           uint32_t row0, int nv, uint64_t piece0,
                                           uint64_t npieces, uint32_t wave, uint32_t lane) {
  const uint32_t c = lane & 7;
  const uint64_t p = piece0 + 8 * c;
  const bool wide = ((sstride | reinterpret_cast<uintptr_t>(SH)) & 15) == 0;  // 16-B aligned rows
  const uint8_t *src = regions + c * REG_BYTES;
  // the common case, decided once (uniform): aligned rows, the whole tile inside
  // the payload, all 512 rows below n_validators -- one aligned 16-B store per
  // lane and row, no per-lane tests (the general loop below compiles to a 4-B +
  // a misaligned 12-B store per chunk)
  if (wide && piece0 + TILE <= npieces && int(row0) + 512 <= nv) {
    const uint32_t v0 = wave * 8 + (lane >> 3);
    const uint32_t sa = lds_addr(src) + soff(v0, c);
    uint8_t *dst = SH + uint64_t(row0 + v0) * sstride + 2 * p;
    const uint64_t dstep = uint64_t(8 * WAVES) * sstride;
#pragma unroll
    for (int it = 0; it < 512 / (8 * WAVES); ++it) {  // soff is GF(2)-linear in v = it * 8 WAVES | v0
      typedef uint32_t v4u __attribute__((ext_vector_type(4)));
      const v4u val = *(const __attribute__((address_space(3))) v4u *)(uintptr_t(sa ^ soff(uint32_t(it) * 8 * WAVES, 0)));
      // streaming (non-temporal): rows are written once, not re-read
      __builtin_nontemporal_store(val, reinterpret_cast<v4u *>(dst + it * dstep));
    }
    return;
  }
#pragma unroll 2
  for (int it = 0; it < 512 / (8 * WAVES); ++it) {
    const uint32_t v = uint32_t(it) * 8 * WAVES + wave * 8 + (lane >> 3);
    const uint4 val = *reinterpret_cast<const uint4 *>(src + soff(v, c));
    const uint32_t shard = row0 + v;
    if (int(shard) >= nv) continue;
    uint8_t *dst = SH + uint64_t(shard) * sstride + 2 * p;
    if (p + 8 <= npieces) {
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

// symbol <-> tower coordinates of both groups (an involution)
__device__ __forceinline__ void to_tower(S16 &g0, S16 &g1) {
  const TowerK tk = tower_k();
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    g0.l[r] = tower_lo(g0.l[r], g0.h[r], tk);
    g1.l[r] = tower_lo(g1.l[r], g1.h[r], tk);
  }
}

// workgroup wg's coefficient slot, wave w, group g: 16 registers x 64 lanes
__device__ __forceinline__ uint2 *coef_at(uint2 *scratch, uint64_t wg, uint32_t wave, int g) {
  return scratch + ((wg * WAVES + wave) * 2 + uint64_t(g)) * (16 * 64);
}

// One persistent launch for all four transforms.  The four 80 KB table sets
// take turns in LDS, loaded by LDS-DMA: coset 2's, coset 3's and the next
// tile's index-0 set behind the previous coset's shard stores (its tables are
// no longer read by then), coset 1's right after the IFFT.  Coset 1 takes the
// IFFT coefficients from the registers; cosets 2 and 3 read them back from a
// per-workgroup scratch slot (128 KB, rewritten every tile, so it stays in L2
// / the memory-side cache).  (Prefetching them behind the previous coset's
// stores needs 64 more VGPRs at the 256 limit: 15 spills, 7.61 vs 6.95 ms.)
__global__ void __launch_bounds__(THREADS)
    encode_k1024_fused(const uint8_t *__restrict__ payloads, uint64_t plen, uint64_t pstride,
                       uint8_t *__restrict__ shards, uint64_t slen, uint64_t sstride, int nv,
                       uint32_t batch, uint2 *__restrict__ coef, DevTables t) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  uint8_t *tabs = lds;
  uint8_t *regions = lds + Tabs::kBytes;
  const uint32_t tid0 = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid0 >> 6);
  uint8_t *my = regions + wave * REG_BYTES;
  // cosets 1 .. ncos - 1 start below n_validators (poly_encoder.hpp:229-236)
  const uint32_t ncos = uint32_t(nv + K - 1) / K;
  uint2 *const cw0 = coef_at(coef, blockIdx.x, wave, 0), *const cw1 = coef_at(coef, blockIdx.x, wave, 1);

  // tower images: the transforms run in tower coordinates
  Tabs::copy_image<THREADS>(tabs, t.timg_t, tid0);  // index 0 (the IFFT)
  __syncthreads();

  const uint64_t npieces = slen / 2;
  const uint32_t tiles_pp = uint32_t((npieces + TILE - 1) / TILE);
  const uint64_t total = uint64_t(tiles_pp) * batch;
  for (uint64_t tile = blockIdx.x; tile < total; tile += gridDim.x) {
    uint32_t tid = tid0;
    asm volatile("" : "+v"(tid));
    const uint32_t lane = tid & 63;
    const uint64_t b = tile / tiles_pp;
    const uint64_t piece0 = (tile % tiles_pp) * TILE;
    uint8_t *SH = shards + b * uint64_t(nv) * sstride;
    const uint8_t *P = payloads + b * pstride;
    S16 g0, g1;
    // a wave none of whose 8 pieces exist (the payload's last, partial tile:
    // 1 MB is 489 pieces, its 8th tile has 41) skips its transforms and only
    // joins the barriers, the table DMAs and the row stores (uniform)
    const bool idle = piece0 + 8 * wave >= npieces;
    const auto load_coef = [&]() __attribute__((always_inline)) {
      // opaque addresses: the values stored after the IFFT must be read back,
      // not forwarded from the registers (which would stay live meanwhile)
      const uint2 *r0 = cw0, *r1 = cw1;
      asm volatile("" : "+s"(r0), "+s"(r1));
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const uint2 x = r0[r * 64 + lane], y = r1[r * 64 + lane];
        g0.l[r] = x.x;
        g0.h[r] = x.y;
        g1.l[r] = y.x;
        g1.h[r] = y.y;
      }
    };
    if (!idle) {
      load_group(g0, P, plen, piece0 + 8 * wave, lane);
      load_group(g1, P, plen, piece0 + 8 * wave + 4, lane);
    }
    // systematic shards 0..1023 = the data symbols (poly_encoder.hpp:239)
#pragma unroll
    for (uint32_t hf = 0; hf < 2; ++hf) {
      lds_barrier();  // the other waves are done reading the regions
      if (!idle) stage_half(g0, g1, my, lane, wave, hf);
      lds_barrier();
      store_half(regions, SH, sstride, 512 * hf, nv, piece0, npieces, wave, lane);
    }
    // the index-0 tables (the last tile's DMA, issued before the 16 fast-form
    // systematic stores just made) landed; the regions are free
    if (((sstride | reinterpret_cast<uintptr_t>(SH)) & 15) == 0 && piece0 + TILE <= npieces)
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
    if (!idle) {
      to_tower(g0, g1);
      ifft1024<true, tower_sub_min(0)>(g0, tabs, my, lane);
      ifft1024<true, tower_sub_min(0)>(g1, tabs, my, lane);
#pragma unroll
      for (int r = 0; r < 16; ++r) {  // read back by cosets 2 and 3 (coset 1 uses the registers)
        cw0[r * 64 + lane] = make_uint2(g0.l[r], g0.h[r]);
        cw1[r * 64 + lane] = make_uint2(g1.l[r], g1.h[r]);
      }
    }
    lds_barrier();  // every wave is done with the index-0 tables
    Tabs::dma_image<THREADS>(tabs, t.timg_t + kTabImageBytes, tid);
    // cs: std::integral_constant coset number (its image's subfield stages)
    const bool fast_rows = ((sstride | reinterpret_cast<uintptr_t>(SH)) & 15) == 0 && piece0 + TILE <= npieces;
    const auto coset = [&](auto cs) __attribute__((always_inline)) {
      constexpr uint32_t s = decltype(cs)::value;
      if (s > 1 && fast_rows && int(s * K) <= nv) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // coset s's tables and coefficients landed
      lds_barrier();  // (all waves' slices) and the regions are free
      if (!idle) {
        fft1024<false, tower_sub_min(int(s))>(g0, tabs, my, lane);
        fft1024<false, tower_sub_min(int(s))>(g1, tabs, my, lane);
        to_tower(g0, g1);  // back to symbol coordinates
      }
#pragma unroll
      for (uint32_t hf = 0; hf < 2; ++hf) {
        if (hf) lds_barrier();
        if (!idle) stage_half(g0, g1, my, lane, wave, hf);
        lds_barrier();
        if (hf == 0)  // every wave is past its FFT: the next set (index 0 after the last coset)
          Tabs::dma_image<THREADS>(tabs, t.timg_t + (s + 1 < ncos ? s + 1 : 0) * kTabImageBytes, tid);
        if (hf == 1 && s + 1 < ncos && !idle) load_coef();  // g0 / g1 are staged
        store_half(regions, SH, sstride, s * K + 512 * hf, nv, piece0, npieces, wave, lane);
      }
    };
    coset(std::integral_constant<uint32_t, 1>());
    coset(std::integral_constant<uint32_t, 2>());
    if (ncos > 3) coset(std::integral_constant<uint32_t, 3>());
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA outlives the workgroup
}

}  // namespace

bool k1024_applicable(const CodeParams &p) { return p.k == 1024 && p.n == 4096; }

size_t k1024_scratch_bytes(size_t plen, size_t batch) {
  const size_t tiles = (shard_len(K, plen) / 2 + TILE - 1) / TILE * batch;
  return std::min(tiles, kMaxGrid) * SCRATCH_PER_WG;  // one coefficient slot per workgroup
}

hipError_t launch_encode_k1024(const CodeParams &p, const DevTables &t, const uint8_t *d_payloads,
                               size_t plen, size_t pstride, size_t batch, uint8_t *d_shards,
                               size_t sstride, void *scratch, hipStream_t s) {
  int cus = 0;
  const size_t sl = shard_len(p.k, plen);
  const size_t tiles = (sl / 2 + TILE - 1) / TILE * batch;
  if (const hipError_t e = prepare_kernel(reinterpret_cast<const void *>(&encode_k1024_fused), LDS_BYTES, &cus);
      e != hipSuccess)
    return e;
  const unsigned grid = unsigned(std::min({tiles, size_t(cus), kMaxGrid}));
  if (!scratch) return hipErrorInvalidValue;
  hipLaunchKernelGGL(encode_k1024_fused, dim3(grid), dim3(THREADS), LDS_BYTES, s, d_payloads,
                     uint64_t(plen), uint64_t(pstride), d_shards, uint64_t(sl), uint64_t(sstride),
                     int(p.nv), uint32_t(batch), static_cast<uint2 *>(scratch), t);
  return hipGetLastError();
}

}  // namespace ecamd
