// dec_n1024x.hip — reconstruct for n = 1024, k = 256 (n_validators 766..1024,
// the BASELINE headline) with 12 waves per CU: three per SIMD instead of the
// two of reconstruct_n1024 (dec_n1024.hip), for the latency the 2-wave form
// leaves exposed (31% of wave time waiting to issue, the
// VALU ~57% busy at 2 waves per SIMD).
//
// The per-wave work is reconstruct_n1024's (one byte-planar group of 4 shard
// columns per wave; gather + E[v] scaling, IFFT_1024 in radix-16 register
// passes with wave-private LDS exchanges, the closed-form derivative and the
// FFT restricted to the k outputs, phase 5: erased outputs times E[y]).  What
// it takes to fit 12 waves in one CU:
//  * LDS = the 32 KB element-indexed compact image (DevTables::cimg, the
//    headline encode's; since round 6: layouts whose element kinds are
//    register-indexed, below) + 12 x 8 KB exchange regions = 128 KB.  Until
//    round 6 a 64 KB reduced skew-slot image (every stage-0 table in the
//    general form, because the kinds varied across the lanes).
//  * phase 5's received data rows y < k: the gather copies each present
//    row's raw 96-B segment into LDS beside the regions (24 KB of the 32 KB
//    the compact image freed; until round 6 they were re-read from the
//    shards into registers held across the IFFT: 10.58 -> 10.54 ms at
//    nv = 1024, 10.23 -> 10.12 at nv = 800, profiles/r06/ab/rec_stage/).
//  * <= 168 VGPRs: the output tables E[y] are requested after IFFT pass C,
//    not before the transform.
// Tile = 48 shard columns (12 waves x 4); 1 MB at n_validators 1024 is 1954
// columns, 41 tiles per payload.
#include <hip/hip_runtime.h>

#include "dec_n1024_common.hpp"
#include "ec_device.hpp"
#include "ec_kernels.hpp"
#include "cimg.hpp"

namespace ecamd {
namespace {
using namespace n1024;
constexpr int WAVES = 12;
constexpr int THREADS = 64 * WAVES;
constexpr int COLS = 4 * WAVES;  // shard columns per tile
constexpr int TAB_REGION = int(kCImgBytes);  // the element-indexed compact image
static_assert(TAB_REGION % 8192 == 0, "regions 8 KB aligned: region addresses are base | rz");
// the tile schedule's LDS word, after the regions
// phase 5's received rows y < 256: row slot (y & 3) << 6 | y >> 2 at a 112-B
// pitch, so that its reads (y = 4 lane + q) are at most 2-way
constexpr uint32_t STG = uint32_t(TAB_REGION + WAVES * REG_BYTES);
constexpr uint32_t STG_PITCH = 112;
__device__ __forceinline__ uint32_t stg_row(uint32_t y) { return STG + (((y & 3) << 6) | (y >> 2)) * STG_PITCH; }
constexpr uint32_t SLOT = STG + 256 * STG_PITCH;
constexpr int LDS_BYTES = int(SLOT + 16);
static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
constexpr int ROW_WORDS = COLS / 2;  // dwords of a row segment (96 B)

// Region address of position v (8-byte cells, GF(2)-linear): conflict-free
// for the reads (2 x 32 lanes) and writes (4 x 16 lanes) of the three layouts
// below (scripts/search_raddr.py's condition; raddr, dec_n1024_common.hpp,
// is 2-way on layout A' reads)
__host__ __device__ constexpr uint32_t rz(uint32_t v) {
  return ((v >> 5) << 8) | (((v ^ (v >> 4) ^ (v >> 5)) & 31) << 3);
}

// The IFFT's three register layouts (lane bits / register bits -> position bits):
//  A' lane = p2..p7, r = (p0, p1, p8, p9): stages 0, 1.  The element of a
//     butterfly, x = pos >> (m + 1) (its table: the compact image entry x,
//     cimg.hpp), has its kind bits (x >= 128: F9, x >= 256: general) in p8,
//     p9, i.e. in the register index: every multiply takes the cheapest form
//     its element allows (stage 0: 2 subfield + 2 F9 + 4 general per lane,
//     stage 1: 4 subfield + 4 F9), where the round-5 layout (p0..p3 in
//     registers) had p8, p9 in the lane and used the general form for all of
//     stage 0 and the F9 form for all of stage 1.
//  B' lane = (p0, p1, p6..p9), r = p2..p5: stages 2-5 (subfield).
//  C  lane = p0..p5, r = (p8, p9, p6, p7): stages 6-9, every element
//     wave-uniform (x = 0: b ^= a only), then the derivative and the FFT.
__device__ __forceinline__ uint32_t posA2_reg(int r) { return uint32_t(r & 3) | (uint32_t(r >> 2) << 8); }
__device__ __forceinline__ uint32_t posB2_lane(uint32_t lane) { return (lane & 3) | ((lane >> 2) << 6); }
__device__ __forceinline__ uint32_t posC_reg(int r) {
  return (uint32_t((r >> 2) & 3) << 6) | (uint32_t(r & 3) << 8);
}

// IFFT stages 0 and 1 in layout A'
__device__ __forceinline__ void ipassA2(S16 &s, uint32_t lane) {
  const uint32_t l0 = cimg_lin(lane << 1), l1 = cimg_lin(lane);
  SubTab S0, S1;
  F9Tab F0, F1;
  Tab G0, G1;
  // stage 0, pair (r, r + 1): x = ((r >> 1) & 1) | lane << 1 | (r >> 2) << 7
  ctab(l0, cimg_lin(0), S0);
  ctab(l0, cimg_lin(1), S1);
  ctab(l0, cimg_lin(128), F0);
  ib(s, 0, 1, S0);
  ctab(l0, cimg_lin(129), F1);
  ib(s, 2, 3, S1);
  ctab(l0, cimg_lin(256), G0);
  ib(s, 4, 5, F0);
  ctab(l0, cimg_lin(257), G1);
  ib(s, 6, 7, F1);
  ib(s, 8, 9, G0);
  ctab(l0, cimg_lin(384), G0);
  ib(s, 10, 11, G1);
  ctab(l0, cimg_lin(385), G1);
  ctab(l1, cimg_lin(0), S0);
  ib(s, 12, 13, G0);
  ctab(l1, cimg_lin(64), S1);
  ib(s, 14, 15, G1);
  // stage 1, pair (r, r + 2): x = lane | (r >> 2) << 6
  ctab(l1, cimg_lin(128), F0);
  ib(s, 0, 2, S0);
  ib(s, 1, 3, S0);
  ctab(l1, cimg_lin(192), F1);
  ib(s, 4, 6, S1);
  ib(s, 5, 7, S1);
  ib(s, 8, 10, F0);
  ib(s, 9, 11, F0);
  ib(s, 12, 14, F1);
  ib(s, 13, 15, F1);
}

// IFFT stages 2-5 in layout B': radix 16 over r = p2..p5, 15 subfield tables
// (stage 2 + t, block blk: x = lane part >> (3 + t) | blk >> (1 + t)) through
// a ring of R slots, table k requested R - 1 tables ahead of its use
constexpr int tk(int k) { return k < 8 ? 0 : k < 12 ? 1 : k < 14 ? 2 : 3; }
constexpr int bk(int k) { return k < 8 ? 2 * k : k < 12 ? 4 * (k - 8) : k < 14 ? 8 * (k - 12) : 0; }
constexpr int RING_B = 3;
__device__ __forceinline__ void ipassB2(S16 &s, uint32_t lane) {
  const uint32_t ph = (lane >> 2) << 6;  // p6..p9 of the lane part
  const uint32_t lt[4] = {cimg_lin(ph >> 3), cimg_lin(ph >> 4), cimg_lin(ph >> 5), cimg_lin(ph >> 6)};
  SubTab ring[RING_B];
  const auto fetch = [&](int k, SubTab &U) __attribute__((always_inline)) {
    ctab(lt[tk(k)], cimg_lin(uint32_t(bk(k)) >> (1 + tk(k))), U);
  };
#pragma unroll
  for (int k = 0; k < RING_B - 1; ++k) fetch(k, ring[k]);
#pragma unroll
  for (int k = 0; k < 15; ++k) {
    if (k + RING_B - 1 < 15) fetch(k + RING_B - 1, ring[(k + RING_B - 1) % RING_B]);
    const int blk = bk(k), d = 1 << tk(k);
#pragma unroll
    for (int i = 0; i < d; ++i) ib(s, blk + i, blk + i + d, ring[k % RING_B]);
  }
}

// IFFT stages 6-9 in layout C (r bit 0 = p8, 1 = p9, 2 = p6, 3 = p7): the
// elements are wave-uniform (broadcast table reads); x = 0 is b ^= a only
// (the skew 0xFFFF, additive_fft.hpp:110-112)
__device__ __forceinline__ void bx(S16 &s, int a, int b) {
  s.l[b] ^= s.l[a];
  s.h[b] ^= s.h[a];
}
__device__ __forceinline__ void ipassC2(S16 &s) {
  SubTab X1, X2, X3, X4;
  ctab(0u, cimg_lin(1), X1);
  ctab(0u, cimg_lin(2), X2);
  ctab(0u, cimg_lin(3), X3);
  ctab(0u, cimg_lin(4), X4);
  // stage 6, pair (r, r | 4): x = p7 | p8 << 1 | p9 << 2
  bx(s, 0, 4);
  ib(s, 8, 12, X1);
  ib(s, 1, 5, X2);
  ib(s, 9, 13, X3);
  ib(s, 2, 6, X4);
  ctab(0u, cimg_lin(5), X4);
  ib(s, 10, 14, X4);
  ctab(0u, cimg_lin(6), X4);
  ib(s, 3, 7, X4);
  ctab(0u, cimg_lin(7), X4);
  ib(s, 11, 15, X4);
  // stage 7, pair (r, r | 8): x = p8 | p9 << 1
  bx(s, 0, 8);
  bx(s, 4, 12);
  ib(s, 1, 9, X1);
  ib(s, 5, 13, X1);
  ib(s, 2, 10, X2);
  ib(s, 6, 14, X2);
  ib(s, 3, 11, X3);
  ib(s, 7, 15, X3);
  // stage 8, pair (r, r | 1): x = p9
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    bx(s, 4 * q, 4 * q + 1);
    ib(s, 4 * q + 2, 4 * q + 3, X1);
  }
  // stage 9, pair (r, r | 2): x = 0
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    bx(s, 4 * q, 4 * q + 2);
    bx(s, 4 * q + 1, 4 * q + 3);
  }
}

// bytes [0, avail) (avail < 96) of a 16-B aligned row slice into w[24], zero
// beyond: whole dwords at immediate offsets under a uniform count, the last
// one masked (an aligned dword holding a wanted byte never crosses a page)
__device__ __forceinline__ void load_row_tail96(const uint8_t *row, uint32_t avail, uint32_t (&w)[ROW_WORDS]) {
  const uint32_t nw = (avail + 3) / 4;  // wave-uniform
  const uint32_t last = (avail & 3) ? (1u << (8 * (avail & 3))) - 1 : ~0u;
  const uint32_t *r = reinterpret_cast<const uint32_t *>(row);
#pragma unroll
  for (int j = 0; j < ROW_WORDS; ++j) {
    w[j] = 0;
    if (uint32_t(j) < nw) w[j] = r[j] & (uint32_t(j) + 1 == nw ? last : ~0u);
  }
}

}  // namespace

__global__ void __launch_bounds__(THREADS) reconstruct_n1024x(
    const uint8_t *__restrict__ shards, uint64_t slen, uint64_t sstride,
    const uint8_t *__restrict__ present, const uint16_t *__restrict__ elog,
    const uint32_t *__restrict__ pattern, const uint32_t *__restrict__ order,
    uint8_t *__restrict__ out, uint64_t ostride, int nv, uint32_t batch, uint32_t *tick, DevTables t) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  uint8_t *regions = lds + TAB_REGION;
  // Tiles are handed out dynamically: a workgroup's first tile is blockIdx.x,
  // every later one gridDim.x + a ticket from the counter *tick (zeroed by
  // the launcher).  The ticket for the tile after next is taken by thread 0
  // during a tile and published in the LDS word SLOT at its end (one tile of
  // notice: the next tile's metadata is loaded a tile ahead).  A static
  // grid stride left the workgroups' end times ~3.5% of the launch apart.
  volatile uint32_t *slot = reinterpret_cast<volatile uint32_t *>(lds + SLOT);
  const uint32_t tid0 = threadIdx.x, wave = tid0 >> 6;
  uint32_t taken = 0;
  if (tid0 == 0) taken = gridDim.x + atomicAdd(tick, 1u);
  uint8_t *my = regions + wave * REG_BYTES;

  // the 32 KB compact image (DevTables::cimg), every load issued before the first store
  {
    constexpr int kPer = (TAB_REGION / 16 + THREADS - 1) / THREADS;
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    v4u v[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const uint32_t i = tid0 + k * THREADS;
      if (i < uint32_t(TAB_REGION / 16)) v[k] = reinterpret_cast<const v4u *>(t.cimg)[i];
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const uint32_t i = tid0 + k * THREADS;
      if (i < uint32_t(TAB_REGION / 16)) reinterpret_cast<v4u *>(lds)[i] = v[k];
    }
  }
  __syncthreads();
  if (tid0 == 0) *slot = taken;  // read after the first tile's region barrier

  const uint64_t ncols = slen / 2;
  const uint32_t tiles_pp = uint32_t((ncols + COLS - 1) / COLS);
  const uint64_t total = uint64_t(tiles_pp) * batch;
  const uint32_t wave_s = __builtin_amdgcn_readfirstlane(tid0 >> 6);
  // m[0], m[1]: this thread's gather slots (gather_order: present rows first;
  // slot tid and 768 + tid, the latter only below 1024): row << 16 |
  // mul_index(E[row]), low half 0xFFFF = absent.  m[2], m[3]: the output rows
  // y = 4 lane + q of phase 5, 16 bits each: 0xFFFF = present, else
  // mul_index(E[y]).  Loaded one tile ahead.
  const auto load_meta = [&](uint64_t bw, uint32_t tid, uint32_t (&m)[4]) {
    const uint64_t pt = pattern ? pattern[bw] : bw;
    m[0] = order[bw * N + tid];
    m[1] = tid + THREADS < uint32_t(N) ? order[bw * N + THREADS + tid] : 0xFFFFu;
    const uint32_t y0 = 4 * (tid & 63);
    const uint32_t p4 = *reinterpret_cast<const uint32_t *>(present + pt * N + y0);
    const uint2 e4 = *reinterpret_cast<const uint2 *>(elog + pt * N + y0);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t e = ((q < 2 ? e4.x : e4.y) >> (16 * (q & 1))) & 0xFFFFu;
      const uint32_t f = ((p4 >> (8 * q)) & 0xFFu) ? 0xFFFFu : mul_index(e);
      if (q & 1) m[2 + (q >> 1)] |= f << 16;
      else m[2 + (q >> 1)] = f;
    }
  };
  uint32_t meta[4] = {0, 0, 0, 0}, meta_next[4] = {0, 0, 0, 0};
  uint32_t cur = blockIdx.x;  // (total < 2^32: launcher)
  if (cur < total) load_meta(cur / tiles_pp, tid0, meta);
  while (cur < total) {
    // lane-derived addresses recomputed per tile (not hoisted and spilled)
    uint32_t tid = tid0;
    asm volatile("" : "+v"(tid));
    const uint32_t lane = tid & 63;
    const uint32_t bq = cur / tiles_pp;
    const uint64_t b = bq, col0 = uint64_t(cur - bq * tiles_pp) * COLS;
    const uint8_t *SH = shards + b * uint64_t(nv) * sstride;
    uint8_t *O = out + b * ostride;

    uint32_t nxt;  // the next tile (SLOT)
    // ---- phase 1: gather + scale this thread's slots' rows (decode_main:
    // 174-177), 12 groups of 4 columns each into the groups' regions; absent
    // rows as 0.  The first slot's row and E[v] table are requested before
    // the tile barrier.
    {
      uint32_t w[ROW_WORDS] = {};  // (defined on every path: not carried across tiles)
      Tab RT = {};
      const uint64_t avail = slen - 2 * col0;  // bytes of a row inside the tile
      const auto load_row = [&](int half) __attribute__((always_inline)) {
        const uint8_t *row = SH + uint64_t(meta[half] >> 16) * sstride + 2 * col0;
        if (avail >= 2 * COLS) {
#pragma unroll
          for (int q = 0; q < ROW_WORDS / 4; ++q) {
            const uint4 d = reinterpret_cast<const uint4 *>(row)[q];
            w[4 * q] = d.x;
            w[4 * q + 1] = d.y;
            w[4 * q + 2] = d.z;
            w[4 * q + 3] = d.w;
          }
        } else {  // the payload's last tile
          load_row_tail96(row, uint32_t(avail), w);
        }
        load_tab(t.mtab_tin, meta[half] & 0xffffu, RT);  // scaled into tower coordinates
      };
      if ((meta[0] & 0xffffu) != 0xffffu) load_row(0);
      lds_barrier();  // the previous tile's readers of the regions are done
      nxt = __builtin_amdgcn_readfirstlane(*slot);
      if (tid0 == 0) taken = gridDim.x + atomicAdd(tick, 1u);  // the tile after nxt
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        if (half == 1 && tid >= uint32_t(N - THREADS)) break;  // (uniform per wave)
        const uint32_t v = meta[half] >> 16;
        const bool on = (meta[half] & 0xffffu) != 0xffffu;
        if (half == 1 && on) load_row(1);
        uint32_t l[WAVES], h[WAVES];
#pragma unroll
        for (int g = 0; g < WAVES; ++g) l[g] = h[g] = 0;
        if (on) {  // one divergent branch for the 12 groups
          if (v < uint32_t(K)) {  // phase 5's copy of a received data row
#pragma unroll
            for (int j = 0; j < ROW_WORDS / 4; ++j)
              *reinterpret_cast<__attribute__((address_space(3))) v4u *>(uintptr_t(stg_row(v) + 16 * j)) =
                  v4u{w[4 * j], w[4 * j + 1], w[4 * j + 2], w[4 * j + 3]};
          }
#pragma unroll
          for (int g = 0; g < WAVES; ++g) {  // columns 4g..4g+3: words (h0 l0 h1 l1)(h2 l2 h3 l3)
            const uint32_t a = w[2 * g], c = w[2 * g + 1];
            const uint32_t xh = vperm(c, a, 0x06040200u), xl = vperm(c, a, 0x07050301u);
            mul_acc(xl, xh, RT, l[g], h[g]);
          }
        }
#pragma unroll
        for (int g = 0; g < WAVES; ++g)
          *reinterpret_cast<uint2 *>(regions + g * REG_BYTES + rz(v)) = make_uint2(l[g], h[g]);
      }
    }
    if (nxt < total) load_meta(nxt / tiles_pp, tid, meta_next);
    __syncthreads();  // (every wave has read SLOT)
    const uint64_t cbase = col0 + 4 * uint64_t(wave_s);  // wave-uniform
    // a group past the payload's last column (the last, partial tile: 1 MB is
    // 1954 columns, the 41st tile has 34): phases 2-5 are this wave's alone
    if (cbase >= ncols) {
#pragma unroll
      for (int i = 0; i < 4; ++i) meta[i] = meta_next[i];
      cur = nxt;
      continue;
    }

    S16 s;
    // ---- phase 2: IFFT_1024 on this wave's group: layouts A', B', C (above)
    {
      const uint32_t la = lds_addr(my) | rz(lane << 2);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const uint2 x = lds_ld2(la ^ rz(posA2_reg(r)));
        s.l[r] = x.x;
        s.h[r] = x.y;
      }
      ipassA2(s, lane);
#pragma unroll
      for (int r = 0; r < 16; ++r) lds_st2(la ^ rz(posA2_reg(r)), make_uint2(s.l[r], s.h[r]));
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
    {
      const uint32_t lb = lds_addr(my) | rz(posB2_lane(lane));
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const uint2 x = lds_ld2(lb ^ rz(uint32_t(r) << 2));
        s.l[r] = x.x;
        s.h[r] = x.y;
      }
      ipassB2(s, lane);
#pragma unroll
      for (int r = 0; r < 16; ++r) lds_st2(lb ^ rz(uint32_t(r) << 2), make_uint2(s.l[r], s.h[r]));
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
    // layout C: r bit0 = p8, bit1 = p9, bit2 = p6, bit3 = p7; lane = p0..p5
    const uint32_t lc = lds_addr(my) | rz(lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const uint2 x = lds_ld2(lc ^ rz(posC_reg(r)));
      s.l[r] = x.x;
      s.h[r] = x.y;
    }
    ipassC2(s);

    // phase-5 operands requested now, consumed after the derivative and the
    // FFT: E[y] of this lane's erased output rows y = 4 lane + q (and the
    // received ones)
    Tab T5[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t m = (meta[2 + (q >> 1)] >> (16 * (q & 1))) & 0xFFFFu;
      // defined on every path (a table read only where used would be carried
      // across the tile loop, and spilled, by the compiler)
      load_tab(t.mtab_tout, m != 0xFFFFu ? m : 0u, T5[q]);  // tower in, symbols out
    }

    // ---- phases 3 + 4: the closed-form derivative at y < 256 and the FFT
    // restricted to y < 256 (dec_n1024.hip, the same steps)
    uint32_t ql[4], qh[4];
    {
      const uint32_t keep0 = ((lane ^ (lane >> 1)) & 1) ? 0u : 0xffffffffu;
      const uint32_t m4 = ((lane >> 4) & 1) ? 0u : 0xffffffffu;
      const uint32_t m5 = ((lane >> 5) & 1) ? 0u : 0xffffffffu;
      const auto lane_terms = [&](uint32_t c0, uint32_t acc) {
        acc ^= uint32_t(__builtin_amdgcn_update_dpp(0, int(c0), 0xF5, 0xf, 0xf, false));  // quad [1,1,3,3]
        acc ^= uint32_t(__builtin_amdgcn_update_dpp(0, int(c0), 0xEE, 0xf, 0xf, false));  // quad [2,3,2,3]
        acc ^= uint32_t(__builtin_amdgcn_update_dpp(0, int(c0), 0x104, 0xf, 0x5, false));  // row_shl:4, banks 0, 2
        acc ^= uint32_t(__builtin_amdgcn_update_dpp(0, int(c0), 0x108, 0xf, 0x3, false));  // row_shl:8, banks 0, 1
        acc = __builtin_amdgcn_bitop3_b32(acc, from_upper(c0, 4), m4, 0x78);  // acc ^ (x & m)
        acc = __builtin_amdgcn_bitop3_b32(acc, from_upper(c0, 5), m5, 0x78);
        return __builtin_amdgcn_bitop3_b32(acc, c0, keep0, 0x78);
      };
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint32_t al = s.l[4 * q + 1] ^ s.l[4 * q + 2], ah = s.h[4 * q + 1] ^ s.h[4 * q + 2];
        if (!(q & 1)) {  // p6 = 0
          al ^= s.l[4 * (q | 1)];
          ah ^= s.h[4 * (q | 1)];
        }
        if (!(q & 2)) {  // p7 = 0
          al ^= s.l[4 * (q | 2)];
          ah ^= s.h[4 * (q | 2)];
        }
        ql[q] = lane_terms(s.l[4 * q], al);
        qh[q] = lane_terms(s.h[4 * q], ah);
      }
    }
    {
      auto fb = [&](int a, int bb, const SubTab &T) {  // every stage >= SUB for y < 256
        mul_acc_sub(ql[bb], qh[bb], T, ql[a], qh[a]);
        ql[bb] ^= ql[a];
        qh[bb] ^= qh[a];
      };
      const uint32_t hi67 = ((lane >> 4) & 3) << 6, lo = lane & 15;
      const uint32_t hi47 = ((lane >> 2) & 15) << 4, lo01 = lane & 3;
      const uint32_t hi27 = lane << 2;
      // the restricted FFT's elements x = pos >> (m + 1) (compact image entries)
      auto L = [&](int i) -> uint32_t {
        switch (i) {
          case 2: return cimg_lin(1);                         // stage 6, p7 = 1
          case 3: return cimg_lin((hi67 | lo) >> 6);          // stage 5
          case 4: return cimg_lin((hi67 | lo) >> 5);          // stage 4
          case 5: return cimg_lin((hi67 | 32u | lo) >> 5);
          case 6: return cimg_lin((hi47 | lo01) >> 4);        // stage 3
          case 7: return cimg_lin((hi47 | lo01) >> 3);        // stage 2
          case 8: return cimg_lin((hi47 | 8u | lo01) >> 3);
          case 9: return cimg_lin(hi27 >> 2);                 // stage 1
          case 10: return cimg_lin(hi27 >> 1);                // stage 0
          default: return cimg_lin((hi27 | 2u) >> 1);
        }
      };
      const auto fx = [&](int a, int bb) {
        ql[bb] ^= ql[a];
        qh[bb] ^= qh[a];
      };
      SubTab T[2];
      ctab(0u, L(2), T[0]);
      ctab(0u, L(3), T[1]);
      fx(0, 2);  // stage 7
      fx(1, 3);
      fx(0, 1);  // stage 6
      fb(2, 3, T[0]);
      ctab(0u, L(4), T[0]);
      swap_bit(ql[0], ql[1], 4, false);
      swap_bit(qh[0], qh[1], 4, false);
      swap_bit(ql[2], ql[3], 4, false);
      swap_bit(qh[2], qh[3], 4, false);
      swap_bit(ql[0], ql[2], 5, false);
      swap_bit(qh[0], qh[2], 5, false);
      swap_bit(ql[1], ql[3], 5, false);
      swap_bit(qh[1], qh[3], 5, false);
      fb(0, 2, T[1]);  // stage 5
      fb(1, 3, T[1]);
      ctab(0u, L(5), T[1]);
      fb(0, 1, T[0]);  // stage 4
      ctab(0u, L(6), T[0]);
      fb(2, 3, T[1]);
      ctab(0u, L(7), T[1]);
      const bool l2 = (lane >> 2) & 1, l3 = (lane >> 3) & 1;
      swap_bit(ql[0], ql[1], 2, l2);
      swap_bit(qh[0], qh[1], 2, l2);
      swap_bit(ql[2], ql[3], 2, l2);
      swap_bit(qh[2], qh[3], 2, l2);
      swap_bit(ql[0], ql[2], 3, l3);
      swap_bit(qh[0], qh[2], 3, l3);
      swap_bit(ql[1], ql[3], 3, l3);
      swap_bit(qh[1], qh[3], 3, l3);
      fb(0, 2, T[0]);  // stage 3
      fb(1, 3, T[0]);
      ctab(0u, L(8), T[0]);
      fb(0, 1, T[1]);  // stage 2
      ctab(0u, L(9), T[1]);
      fb(2, 3, T[0]);
      ctab(0u, L(10), T[0]);
      const bool l0 = lane & 1, l1 = (lane >> 1) & 1;
      swap_bit(ql[0], ql[1], 0, l0);
      swap_bit(qh[0], qh[1], 0, l0);
      swap_bit(ql[2], ql[3], 0, l0);
      swap_bit(qh[2], qh[3], 0, l0);
      swap_bit(ql[0], ql[2], 1, l1);
      swap_bit(qh[0], qh[2], 1, l1);
      swap_bit(ql[1], ql[3], 1, l1);
      swap_bit(qh[1], qh[3], 1, l1);
      fb(0, 2, T[1]);  // stage 1
      fb(1, 3, T[1]);
      ctab(0u, L(11), T[1]);
      fb(0, 1, T[0]);  // stage 0
      fb(2, 3, T[1]);
    }

    // ---- phase 5: y = 4*lane + q; columns cbase + c (decode_main:185-188,
    // reconstructSub:138-149)
    {
      uint32_t ol[4], oh[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t m = (meta[2 + (q >> 1)] >> (16 * (q & 1))) & 0xFFFFu;
        ol[q] = oh[q] = 0;
        if (m != 0xFFFFu) {
          mul_acc(ql[q], qh[q], T5[q], ol[q], oh[q]);
        } else {
          const uint2 rv = lds_ld2(stg_row(4 * lane + uint32_t(q)) + 8 * wave_s);
          oh[q] = vperm(rv.y, rv.x, 0x06040200u);
          ol[q] = vperm(rv.y, rv.x, 0x07050301u);
        }
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const uint64_t col = cbase + c;
        if (col >= ncols) break;
        const uint32_t w0 = vperm(ol[0], oh[0], 0x0c0c0400u + 0x0101u * c) |
                            (vperm(ol[1], oh[1], 0x0c0c0400u + 0x0101u * c) << 16);
        const uint32_t w1 = vperm(ol[2], oh[2], 0x0c0c0400u + 0x0101u * c) |
                            (vperm(ol[3], oh[3], 0x0c0c0400u + 0x0101u * c) << 16);
        *reinterpret_cast<uint2 *>(O + (col * K + 4 * lane) * 2) = make_uint2(w0, w1);
      }
    }
    // thread 0 (wave 0 never idles: its columns start the tile) publishes the
    // tile after next; the atomic returned during the transform
    if (tid0 == 0) *slot = taken;
#pragma unroll
    for (int i = 0; i < 4; ++i) meta[i] = meta_next[i];
    cur = nxt;
  }
}

// scratch of the n = 1024 reconstructs: the gather order, then the tile
// counter of reconstruct_n1024x (256 B apart)
size_t n1024_tick_offset(const CodeParams &p, size_t batch) { return (gather_order_bytes(p, batch) + 255) / 256 * 256; }
size_t n1024_scratch_bytes(const CodeParams &p, size_t batch) { return n1024_tick_offset(p, batch) + 256; }

hipError_t launch_reconstruct_n1024x(const CodeParams &p, const DevTables &t,
                                     const uint8_t *d_shards, size_t slen, size_t sstride,
                                     const uint8_t *d_present, const uint16_t *d_err_log,
                                     const uint32_t *d_pattern, size_t batch, uint8_t *d_out,
                                     size_t ostride, void *scratch, hipStream_t s) {
  int cus = 0;
  if (!t.cimg || !scratch || slen / 2 < size_t(COLS)) return hipErrorInvalidValue;
  if (const hipError_t e = prepare_kernel(reinterpret_cast<const void *>(&reconstruct_n1024x), LDS_BYTES, &cus);
      e != hipSuccess)
    return e;
  const size_t tiles = (slen / 2 + COLS - 1) / COLS * batch;
  if (tiles + 4096 >= (size_t(1) << 32)) return hipErrorInvalidValue;  // 32-bit tile tickets
  uint32_t *order = static_cast<uint32_t *>(scratch);  // n1024_scratch_bytes(p, batch)
  uint32_t *tick = reinterpret_cast<uint32_t *>(static_cast<uint8_t *>(scratch) + n1024_tick_offset(p, batch));
  if (const hipError_t e = launch_gather_order(p, d_present, d_err_log, d_pattern, batch, order, s);
      e != hipSuccess)
    return e;
  if (const hipError_t e = launch_zero_counters(tick, sizeof(uint32_t), s); e != hipSuccess) return e;
  const unsigned grid = unsigned(tiles < size_t(cus) ? tiles : size_t(cus));
  hipLaunchKernelGGL(reconstruct_n1024x, dim3(grid), dim3(THREADS), LDS_BYTES, s, d_shards, uint64_t(slen),
                     uint64_t(sstride), d_present, d_err_log, d_pattern, order, d_out, uint64_t(ostride),
                     int(p.nv), uint32_t(batch), tick, t);
  return hipGetLastError();
}

}  // namespace ecamd
