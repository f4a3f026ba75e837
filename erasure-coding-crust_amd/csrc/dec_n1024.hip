// dec_n1024.hip — reconstruct kernel specialised for n = 1024, k = 256
// (n_validators 683..1024; BASELINE configs 2 and 3).
//
// Per workgroup tile: 32 shard columns (= 32 codewords of 1024 symbols,
// poly_encoder.hpp:164-189), 8 waves, one byte-planar group of 4 columns per
// wave.  Phases:
//  1. gather+scale: thread v loads 64 B of shard row v and multiplies by the
//     locator E[v] (one v_perm table per row, reused for 8 groups), writing
//     each group into that group's wave-private LDS region;
//  2. IFFT_1024: radix-16 register passes A (bits 0-3), B (4-7) and a radix-4
//     pass C (8-9) with the exchanges going through the wave's region;
//  3. formal derivative in closed form, c'[j] = c[j] ^ XOR_{b: j_b=0} c[j|2^b],
//     register bits in place, lane bits via DPP / permlane swaps;
//  4. FFT_1024 restricted to the k outputs that are read: stage 9 keeps
//     v < 512, stage 8 keeps v < 256, then stages 7..0 on 4 registers per lane
//     with register<->lane bit swaps by DPP / permlane (no LDS);
//  5. output: erased y < k scaled by E[y]; present y copied from the shard;
//     each lane writes 8 contiguous bytes of a 512-byte output row.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "dec_n1024_common.hpp"
#include "ec_device.hpp"
#include "ec_kernels.hpp"

namespace ecamd {
namespace {
using namespace n1024;
constexpr int WAVES = 8;
constexpr int THREADS = 64 * WAVES;
constexpr int COLS = 4 * WAVES;  // shard positions per tile
using OutTabs = LdsTabs<256>;  // output multiply tables E[y], y < 256 (in the regions)
constexpr int TAB_REGION = Tabs::kBytes;
// received rows y < K of the tile as read (the present ones): phase 5 copies
// them to the output instead of re-reading them from HBM
constexpr int STAGE_BYTES = K * COLS * 2;
constexpr int LDS_BYTES = TAB_REGION + WAVES * REG_BYTES + STAGE_BYTES;
static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
static_assert(OutTabs::kBytes <= WAVES * REG_BYTES, "output tables fit the regions");

// staging address of (row y < K, group g): the 8 bytes of columns 4g..4g+3 in
// 32-byte chunks of 4 rows; chunk g of 4-row block y/4 is swizzled by (y/4) & 7
// so the phase-5 reads (lane = y/4, 32 B each, fixed g) cover all banks
__device__ __forceinline__ uint32_t stage_addr(uint32_t y, uint32_t g) {
  return ((y >> 2) << 8) | ((g ^ ((y >> 2) & 7)) << 5) | ((y & 3) << 3);
}
}  // namespace

// Gather order of a payload's received rows (its erasure pattern), per
// 1024-row quarter (n = 1024: one; reconstruct_n4096: n / 1024; n < 1024:
// the n rows, reconstruct_gen): the present
// rows first, then the absent ones, dealt wave-major (slot s of each half ->
// wave s / 64, lane s % 64; waves w and w + 4 share a SIMD), stored in the
// order threads read it: entry [(b * Q + q) * 1024 + half * 512 + tid] =
// (row in quarter << 16) | mul_index(E[row]) for a present row, | 0xFFFF for
// an absent one.  A wave whose slots of a half are all absent skips that
// half's multiplies (uniform branch): with 342 of 1024 rows present
// (threshold) every second half and waves 6, 7 of the first; with k = 256
// present also waves 4, 5, so no SIMD multiplies more than one wave's rows
// (the natural row order multiplied in every wave and half).
__global__ void __launch_bounds__(1024) gather_order(const uint8_t *__restrict__ present,
                                                     const uint16_t *__restrict__ elog,
                                                     const uint32_t *__restrict__ pattern, int nv,
                                                     uint32_t n, uint32_t rows, uint32_t nq,
                                                     uint32_t *__restrict__ order) {
  __shared__ uint32_t cnt[16];
  const uint32_t b = blockIdx.x / nq, q = blockIdx.x % nq;
  const uint32_t v = threadIdx.x, lane = v & 63, w = v >> 6, row = 1024 * q + v;
  const uint64_t pt = pattern ? pattern[b] : b;
  // rows of the block: 1024, or n < 1024 (threads v >= n are absent and, being
  // last in thread order, take slots >= n, which are not written)
  const bool f = v < rows && int(row) < nv && present[pt * n + row] != 0;
  const uint64_t m = __ballot(f);
  const uint32_t below = __popcll(m & ((1ull << lane) - 1));
  if (lane == 0) cnt[w] = uint32_t(__popcll(m));
  __syncthreads();
  uint32_t pw = 0, c = 0;  // present rows in earlier waves, and in all
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    pw += i < int(w) ? cnt[i] : 0u;
    c += cnt[i];
  }
  // slot: present rows in row order, then absent rows in row order; slot s
  // of the quarter is read by thread s % 512 in half s / 512
  const uint32_t slot = f ? pw + below : c + (64 * w - pw) + (lane - below);
  if (v < rows)
    order[uint64_t(b) * n + 1024 * q + slot] = (v << 16) | (f ? mul_index(elog[pt * n + row]) : 0xFFFFu);
}

hipError_t launch_gather_order(const CodeParams &p, const uint8_t *d_present,
                               const uint16_t *d_err_log, const uint32_t *d_pattern, size_t batch,
                               uint32_t *order, hipStream_t s) {
  if (p.n > 1024 && p.n % 1024 != 0) return hipErrorInvalidValue;
  const uint32_t rows = p.n < 1024 ? p.n : 1024, nq = p.n / rows;
  hipLaunchKernelGGL(gather_order, dim3(unsigned(batch * nq)), dim3(1024), 0, s, d_present, d_err_log,
                     d_pattern, int(p.nv), uint32_t(p.n), rows, nq, order);
  return hipGetLastError();
}

size_t gather_order_bytes(const CodeParams &p, size_t batch) { return batch * p.n * sizeof(uint32_t); }

// PACKED (payloads of fewer than 32 columns, or shard pitches the 16-B row
// loads cannot take): the waves run independently over the flattened space
// of byte-planar groups, payload b owning groups [b * ncols4 / 4, (b + 1) *
// ncols4 / 4) (ncols4 = columns rounded up to 4), one group (4 codewords) per
// wave and step.  Lane l gathers rows 16 l .. 16 l + 15 straight into the
// IFFT's layout-A registers (its flags and E[v] in three coalesced loads, the
// absent rows multiplied by the zero table), so there is no LDS gather, no
// gather order and no workgroup barrier: 4096 one-column payloads are 4096
// wave steps (2 per wave on 256 CUs) instead of 4096 workgroup tiles.
template <bool PACKED>
__global__ void __launch_bounds__(THREADS) reconstruct_n1024(
    const uint8_t *__restrict__ shards, uint64_t slen, uint64_t sstride,
    const uint8_t *__restrict__ present, const uint16_t *__restrict__ elog,
    const uint32_t *__restrict__ pattern, const uint32_t *__restrict__ order,
    uint8_t *__restrict__ out, uint64_t ostride, int nv, uint32_t batch, uint32_t ncols4,
    DevTables t) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  uint8_t *tabs = lds;
  uint8_t *regions = lds + TAB_REGION;
  uint8_t *stage = regions + WAVES * REG_BYTES;
  const uint32_t tid0 = threadIdx.x, wave = tid0 >> 6;
  uint8_t *my = regions + wave * REG_BYTES;

  // multiply tables for skew indices 0..1022: the prebuilt LDS image 0
  // (DevTables::timg), one coalesced 80 KB copy instead of a 1023-entry gather
  // through the skews (that gather was ~10 us of every launch; small calls pay it)
  Tabs::copy_image<THREADS>(tabs, kF9 ? t.timg_f9 : t.timg_t, tid0);  // F9 kind 0
  __syncthreads();

  const uint64_t ncols = slen / 2;
  const uint32_t tiles_pp = uint32_t((ncols + COLS - 1) / COLS);
  const uint32_t gpp = ncols4 / 4;  // packed: groups per payload
  // packed: "tile" = this wave's group, stepping over the grid's waves
  const uint64_t total = PACKED ? uint64_t(gpp) * batch : uint64_t(tiles_pp) * batch;
  // the wave index as a wave-uniform (scalar) value: the packed loop and every
  // address derived from its group stay in SGPRs
  const uint32_t wave_s = __builtin_amdgcn_readfirstlane(tid0 >> 6);
  // (group g on workgroup g % grid, wave g / grid: a small batch spreads over
  // every CU)
  // big batches: a workgroup's 8 waves take 8 adjacent groups (one payload's
  // tables shared in L1); small ones: spread, so each CU gets work
  const bool spread = PACKED && total < uint64_t(2) * gridDim.x * WAVES;
  const uint64_t first = !PACKED ? uint64_t(blockIdx.x)
                         : spread ? uint64_t(wave_s) * gridDim.x + blockIdx.x
                                  : uint64_t(blockIdx.x) * WAVES + wave_s;
  const uint64_t step = PACKED ? uint64_t(gridDim.x) * WAVES : gridDim.x;
  // m[0], m[1]: this thread's two gather slots (gather_order): row << 16 |
  // mul_index(E[row]), low half 0xFFFF = absent.  Loaded one tile ahead so the
  // gather's table loads wait on one global latency instead of two.
  // m[2], m[3]: the output rows y = 4 lane + q (q = 0..3) of phase 5, 16 bits
  // each: 0xFFFF = present (copied from the staged row), else mul_index(E[y]) (the
  // erased value is scaled by E[y]; y < 256 < nv always holds for n = 1024).
  TileWalk walk(first, step, tiles_pp);  // !PACKED: payload and tile of `tile`
  // bb: the payload of tile tl (!PACKED: from the walk, no division)
  auto load_meta = [&](uint64_t tl, uint64_t bw, uint32_t tid, uint32_t (&m)[4]) {
    const uint64_t bb = PACKED ? uint64_t(uint32_t(tl) / gpp) : bw;
    const uint64_t pt = pattern ? pattern[bb] : bb;
    if constexpr (!PACKED) {
#pragma unroll
      for (int half = 0; half < 2; ++half) m[half] = order[bb * N + half * THREADS + tid];
    }
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
  if (first < total) load_meta(first, walk.b, tid0, meta);
  for (uint64_t tile = first; tile < total; tile += step, walk.advance()) {
    // lane-derived addresses are recomputed per tile from an opaque copy of
    // the thread id (hoisted out of the loop they were kept live, and spilled,
    // across the whole tile)
    uint32_t tid = tid0;
    asm volatile("" : "+v"(tid));
    const uint32_t lane = tid & 63;
    uint64_t b, col0;
    if constexpr (PACKED) {  // this wave's group: columns [cbase, cbase + 4) of payload b
      b = uint32_t(tile) / gpp;  // < 2^32 groups (launch check)
      col0 = 4 * uint64_t(uint32_t(tile) % gpp) - 4 * uint64_t(wave_s);  // cbase below = col0 + 4 * wave (mod 2^64)
    } else {
      b = walk.b;
      col0 = walk.i * COLS;
    }
    const uint8_t *SH = shards + b * uint64_t(nv) * sstride;
    uint8_t *O = out + b * ostride;
    S16 s;

    if constexpr (PACKED) {
      // ---- phase 1, packed: this wave's group only (decode_main:174-177).
      // The present rows (flag set, v < nv) of the payload's pattern are
      // compacted into a list in the wave's own region (lane l reads the flags
      // and E[v] of rows 16 l .. 16 l + 15 with three coalesced loads, a wave
      // prefix sum places them), so the wave multiplies ceil(present / 64)
      // rows per lane instead of 16; then the region is zeroed (absent rows)
      // and each list entry's product is written at its row.
      const uint64_t pt = pattern ? pattern[b] : b;
      const uint32_t v0 = 16 * lane;
      const uint4 f16 = *reinterpret_cast<const uint4 *>(present + pt * N + v0);
      const uint4 e0 = *reinterpret_cast<const uint4 *>(elog + pt * N + v0);
      const uint4 e1 = *reinterpret_cast<const uint4 *>(elog + pt * N + v0 + 8);
      const uint32_t fw[4] = {f16.x, f16.y, f16.z, f16.w};
      const uint32_t ew[8] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w};
      uint32_t mask = 0;
#pragma unroll
      for (int r = 0; r < 16; ++r)
        mask |= uint32_t(((fw[r >> 2] >> (8 * (r & 3))) & 0xFFu) != 0 && int(v0) + r < nv) << r;
      const uint32_t cnt = __builtin_popcount(mask);
      uint32_t incl = cnt;  // inclusive prefix sum of the counts over the lanes
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = uint32_t(__shfl_up(int(incl), d));
        if (lane >= uint32_t(d)) incl += o;
      }
      const uint32_t total = uint32_t(__shfl(int(incl), 63));  // wave-uniform
      uint32_t at = incl - cnt;
      const uint32_t lbase = lds_addr(my);
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if ((mask >> r) & 1) {  // list entry: row << 16 | mul_index(E[row])
          const uint32_t e = (ew[r >> 1] >> (16 * (r & 1))) & 0xFFFFu;
          *(__attribute__((address_space(3))) uint32_t *)(uintptr_t(lbase + 4 * at)) =
              ((v0 + r) << 16) | mul_index(e);
          ++at;
        }
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
      const uint32_t nj = (total + 63) / 64;  // list entries per lane (uniform)
      uint32_t ent[16];
#pragma unroll
      for (int j = 0; j < 16; ++j)
        ent[j] = uint32_t(j) < nj && lane + 64 * j < total
                     ? *(const __attribute__((address_space(3))) uint32_t *)(uintptr_t(lbase + 4 * (lane + 64 * j)))
                     : 0xFFFFu;  // no entry: the zero table, no bytes read
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int r = 0; r < 16; ++r) lds_st2(lbase | raddr(v0 + r), make_uint2(0, 0));  // absent rows
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
      const uint64_t cg = 4 * uint64_t(uint32_t(tile) % gpp);
      const uint64_t have = ncols - cg;  // columns of the group inside the payload
      const uint32_t avail = have >= 4 ? 8u : uint32_t(2 * have);
      const uint8_t *colp = SH + 2 * cg;
      // rows 8-B aligned and the group whole: one 8-B load per row (uniform)
      const bool wide = avail == 8 && ((sstride | reinterpret_cast<uintptr_t>(colp)) & 7) == 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {  // 4 entries at a time: 4 tables + 4 rows in flight
        if (uint32_t(4 * q) >= nj) break;  // uniform
        Tab T[4];
        uint2 d[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t m = ent[4 * q + i], v = m >> 16;
          const bool on = (m & 0xFFFFu) != 0xFFFFu;
          load_tab(t.mtab_tin, on ? (m & 0xFFFFu) : 65535u, T[i]);  // [65535] = * 0; tower out
          d[i] = make_uint2(0, 0);
          if (on) d[i] = wide ? *reinterpret_cast<const uint2 *>(colp + uint64_t(v) * sstride)
                              : load8_any(colp + uint64_t(v) * sstride, avail);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t m = ent[4 * q + i], v = m >> 16;
          if ((m & 0xFFFFu) == 0xFFFFu) continue;
          if (v < uint32_t(K)) *reinterpret_cast<uint2 *>(stage + stage_addr(v, wave)) = d[i];
          const uint32_t xh = vperm(d[i].y, d[i].x, 0x06040200u), xl = vperm(d[i].y, d[i].x, 0x07050301u);
          uint32_t l = 0, h = 0;
          mul_acc(xl, xh, T[i], l, h);
          lds_st2(lbase | raddr(v), make_uint2(l, h));  // layout A, read back below
        }
        __builtin_amdgcn_sched_barrier(0);  // one batch of tables live at a time
      }
    } else {
    // ---- phase 1: gather + scale this thread's two slots' rows (present rows
    // first, gather_order; decode_main:174-177); absent rows are written as 0.
    // The first slot's row and E[v] table are requested before the barrier
    // (they only land in registers), so their latency overlaps the wait for
    // the other waves' previous tile; the second slot (mostly absent rows:
    // present rows come first) is loaded after it.
    uint32_t w[2][16];
    Tab RT[2];
    const uint64_t avail = slen - 2 * col0;  // bytes of a row inside the tile
    const auto load_row = [&](int half) __attribute__((always_inline)) {
      const uint8_t *row = SH + uint64_t(meta[half] >> 16) * sstride + 2 * col0;
      if (avail >= 64) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint4 d = reinterpret_cast<const uint4 *>(row)[q];
          w[half][4 * q] = d.x;
          w[half][4 * q + 1] = d.y;
          w[half][4 * q + 2] = d.z;
          w[half][4 * q + 3] = d.w;
        }
      } else {  // the payload's last tile: whole dwords, then bytes (rows 16-B aligned here)
        load_row_tail64(row, avail, w[half]);
      }
      load_tab(t.mtab_tin, meta[half] & 0xffffu, RT[half]);  // scaled into tower coordinates
    };
    if ((meta[0] & 0xffffu) != 0xffffu) load_row(0);
    lds_barrier();  // previous tile's readers of the regions are done (LDS only)
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const uint32_t v = meta[half] >> 16;
      uint32_t l[8], h[8];
#pragma unroll
      for (int g = 0; g < 8; ++g) l[g] = h[g] = 0;
      if ((meta[half] & 0xffffu) != 0xffffu) {
        if (half == 1) load_row(1);
        if (v < uint32_t(K)) {  // a present data row: kept for phase 5
#pragma unroll
          for (int g = 0; g < 8; ++g)
            *reinterpret_cast<uint2 *>(stage + stage_addr(v, g)) = make_uint2(w[half][2 * g], w[half][2 * g + 1]);
        }
#pragma unroll
        for (int g = 0; g < 8; ++g) {  // columns 4g..4g+3: words (h0 l0 h1 l1)(h2 l2 h3 l3)
          const uint32_t a = w[half][2 * g], c = w[half][2 * g + 1];
          const uint32_t xh = vperm(c, a, 0x06040200u), xl = vperm(c, a, 0x07050301u);
          mul_acc(xl, xh, RT[half], l[g], h[g]);
        }
      }
#pragma unroll
      for (int g = 0; g < 8; ++g)
        *reinterpret_cast<uint2 *>(regions + g * REG_BYTES + raddr(v)) = make_uint2(l[g], h[g]);
    }
    }
    if (tile + step < total) {
      uint64_t nb, ni;
      walk.next_of(nb, ni);
      load_meta(tile + step, nb, tid, meta_next);
    }
    if constexpr (!PACKED) __syncthreads();  // packed: the wave's own region and staging only
    const uint64_t cbase = col0 + 4 * uint64_t(wave_s);  // wave-uniform: phase 5's column tests stay scalar
    if constexpr (!PACKED) {
      // a group past the payload's last column (its last, partial tile: 1 MB
      // shards are 1954 columns, the 62nd tile has 2): phases 2-5 are this
      // wave's alone, so it goes straight to the next tile's barrier
      if (col0 + 4 * uint64_t(wave_s) >= ncols) {
#pragma unroll
        for (int i = 0; i < 4; ++i) meta[i] = meta_next[i];
        continue;
      }
    }
    // phase-5 tables requested now, consumed after the transform (latency
    // hidden behind it): E[y] of this lane's erased output rows y = 4 lane + q
    // (its present ones are in the staging area)
    Tab T5[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t m = (meta[2 + (q >> 1)] >> (16 * (q & 1))) & 0xFFFFu;
      // tower coordinates in, symbols out
      if constexpr (PACKED) load_tab(t.mtab_tout, m != 0xFFFFu ? m : 0u, T5[q]);  // defined on every path
      else if (m != 0xFFFFu) load_tab(t.mtab_tout, m, T5[q]);
    }

    // ---- phase 2: IFFT_1024 on this wave's group
    {  // layout A: v = 16*lane + r
      const uint32_t la = lds_addr(my) | raddr(16 * lane);
      if constexpr (PACKED) {  // the wave's own writes above: a wave barrier orders them
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const uint2 x = lds_ld2(la ^ raddr(r));
        s.l[r] = x.x;
        s.h[r] = x.y;
      }
      prio_lead(wave_s & 4);
      ipass4<0>(s, tabs, tlin(16 * lane));
#pragma unroll
      for (int r = 0; r < 16; ++r) lds_st2(la ^ raddr(r), make_uint2(s.l[r], s.h[r]));
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
    const uint32_t baseB = (lane & 15) | ((lane >> 4) << 8);  // layout B: bits 4-7 in registers
    {
      const uint32_t lb = lds_addr(my) | raddr(baseB);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const uint2 x = lds_ld2(lb ^ raddr(uint32_t(r) << 4));
        s.l[r] = x.x;
        s.h[r] = x.y;
      }
      prio_lead(!(wave_s & 4));
      ipass4<4>(s, tabs, tlin((lane >> 4) << 8));
#pragma unroll
      for (int r = 0; r < 16; ++r) lds_st2(lb ^ raddr(uint32_t(r) << 4), make_uint2(s.l[r], s.h[r]));
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
    // layout C: r bit0 = p8, bit1 = p9, bit2 = p6, bit3 = p7; lane = p0..p5
    const uint32_t lc = lds_addr(my) | raddr(lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const uint2 x = lds_ld2(lc ^ raddr((uint32_t((r >> 2) & 3) << 6) | (uint32_t(r & 3) << 8)));
      s.l[r] = x.x;
      s.h[r] = x.y;
    }
    // IFFT stages 8 and 9 (inverse_afft, additive_fft.hpp:99-119, index 0).  A
    // stage's block at j = d has skew skews[d - 1] = 0xFFFF, i.e. no multiply:
    // stage 9 is b ^= a only, stage 8 multiplies in its p9 = 1 block only.  The
    // p8 = p9 = 1 registers (4 hi + 3) are not needed past stage 8.
    {
      SubTab Tb;
      tab_at(tabs, tlin(skew_idx(1u << 9, 8)), Tb);
#pragma unroll
      for (int hi = 0; hi < 4; ++hi) {
        s.l[4 * hi + 1] ^= s.l[4 * hi];  // stage 8, p9 = 0 block
        s.h[4 * hi + 1] ^= s.h[4 * hi];
      }
#pragma unroll
      for (int hi = 0; hi < 4; ++hi) ib(s, 4 * hi + 2, 4 * hi + 3, Tb);  // stage 8, p9 = 1 block
#pragma unroll
      for (int hi = 0; hi < 4; ++hi) {
        s.l[4 * hi + 2] ^= s.l[4 * hi];  // stage 9
        s.h[4 * hi + 2] ^= s.h[4 * hi];
      }
    }

    prio_lead(wave_s & 4);
    // ---- phases 3 + 4a: formal derivative (poly_encoder.hpp:195-215) and FFT
    // stages 9, 8 (afft, additive_fft.hpp:121-141) for the outputs y < 256 only.
    // Those FFT stages keep the block at j = d, whose skew skews[d - 1] is
    // 0xFFFF: a ^= b * skew is a no-op, so they pass c'[y] through for y < 256,
    // and the derivative is needed at y < 256 only.  Its closed form
    // c'[y] = c[y] ^ XOR_{b: y_b = 0} c[y | 2^b] there reads
    //   c'[y] = c0[y] ^ c1[y] ^ c2[y] ^ XOR_{b < 8, y_b = 0} c0[y | 2^b]
    // with c0 / c1 / c2 = registers 4 q / 4 q + 1 / 4 q + 2 (p8 p9 = 00 / 10 /
    // 01), q bit 0 = p6, bit 1 = p7, lane bits = p0..p5.
    // Lane-bit terms (lanes with p_b = 0 add the value of lane + 2^b): p2, p3
    // by one row_shl DPP xor each whose bank mask leaves the p_b = 1 lanes
    // untouched; p0, p1 by quad_perm DPP xors that hand the p_b = 1 lanes
    // their own c0 instead of 0 (corrected once: c0 is kept where p0 ^ p1 = 0
    // rather than xor'ed twice); p4, p5 by permlane swaps, masked.
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
      // q bit0 = p6, bit1 = p7; lane bits = p0..p5.  Positions < 256 only.
      auto fb = [&](int a, int bb, const SubTab &T) {  // every stage >= SUB for y < 256
        mul_acc_sub(ql[bb], qh[bb], T, ql[a], qh[a]);
        ql[bb] ^= ql[a];
        qh[bb] ^= qh[a];
      };
      // table addresses in order of use (lane bits after each swap stage below)
      const uint32_t hi67 = ((lane >> 4) & 3) << 6, lo = lane & 15;
      const uint32_t hi47 = ((lane >> 2) & 15) << 4, lo01 = lane & 3;
      const uint32_t hi27 = lane << 2;
      auto L = [&](int i) -> uint32_t {
        switch (i) {
          case 2: return tlin(skew_idx(1u << 7, 6));
          case 3: return tlin(skew_idx(hi67 | lo, 5));
          case 4: return tlin(skew_idx(hi67 | lo, 4));
          case 5: return tlin(skew_idx(hi67 | 32u | lo, 4));
          case 6: return tlin(skew_idx(hi47 | lo01, 3));
          case 7: return tlin(skew_idx(hi47 | lo01, 2));
          case 8: return tlin(skew_idx(hi47 | 8u | lo01, 2));
          // stages 1, 0: their image slots hold general tables; the stage-2
          // slot of the same (subfield) skew element instead (sub_alias)
          case 9: return tlin(sub_alias(hi27, 1));
          case 10: return tlin(sub_alias(hi27, 0));
          default: return tlin(sub_alias(hi27 | 2u, 0));
        }
      };
      // stage 7 (block j = 128) and stage 6's first block (j = 64) have the
      // skew 0xFFFF at index 0 (additive_fft.hpp:129): b ^= a only
      const auto fx = [&](int a, int bb) {
        ql[bb] ^= ql[a];
        qh[bb] ^= qh[a];
      };
      SubTab T[2];
      tab_at(tabs, L(2), T[0]);
      tab_at(tabs, L(3), T[1]);
      fx(0, 2);  // stage 7
      fx(1, 3);
      fx(0, 1);  // stage 6
      fb(2, 3, T[0]);
      tab_at(tabs, L(4), T[0]);
      // q (p6, p7) <-> lane bits 4, 5 (p4, p5)
      swap_bit(ql[0], ql[1], 4, false);
      swap_bit(qh[0], qh[1], 4, false);
      swap_bit(ql[2], ql[3], 4, false);
      swap_bit(qh[2], qh[3], 4, false);
      swap_bit(ql[0], ql[2], 5, false);
      swap_bit(qh[0], qh[2], 5, false);
      swap_bit(ql[1], ql[3], 5, false);
      swap_bit(qh[1], qh[3], 5, false);
      // now q = (p4, p5); lane bits 0-3 = p0..p3, 4 = p6, 5 = p7
      fb(0, 2, T[1]);  // stage 5
      fb(1, 3, T[1]);
      tab_at(tabs, L(5), T[1]);
      fb(0, 1, T[0]);  // stage 4
      tab_at(tabs, L(6), T[0]);
      fb(2, 3, T[1]);
      tab_at(tabs, L(7), T[1]);
      // q (p4, p5) <-> lane bits 2, 3 (p2, p3)
      const bool l2 = (lane >> 2) & 1, l3 = (lane >> 3) & 1;
      swap_bit(ql[0], ql[1], 2, l2);
      swap_bit(qh[0], qh[1], 2, l2);
      swap_bit(ql[2], ql[3], 2, l2);
      swap_bit(qh[2], qh[3], 2, l2);
      swap_bit(ql[0], ql[2], 3, l3);
      swap_bit(qh[0], qh[2], 3, l3);
      swap_bit(ql[1], ql[3], 3, l3);
      swap_bit(qh[1], qh[3], 3, l3);
      // now q = (p2, p3); lane bits 0,1 = p0,p1; 2,3 = p4,p5; 4,5 = p6,p7
      fb(0, 2, T[0]);  // stage 3
      fb(1, 3, T[0]);
      tab_at(tabs, L(8), T[0]);
      fb(0, 1, T[1]);  // stage 2
      tab_at(tabs, L(9), T[1]);
      fb(2, 3, T[0]);
      tab_at(tabs, L(10), T[0]);
      // q (p2, p3) <-> lane bits 0, 1 (p0, p1)
      const bool l0 = lane & 1, l1 = (lane >> 1) & 1;
      swap_bit(ql[0], ql[1], 0, l0);
      swap_bit(qh[0], qh[1], 0, l0);
      swap_bit(ql[2], ql[3], 0, l0);
      swap_bit(qh[2], qh[3], 0, l0);
      swap_bit(ql[0], ql[2], 1, l1);
      swap_bit(qh[0], qh[2], 1, l1);
      swap_bit(ql[1], ql[3], 1, l1);
      swap_bit(qh[1], qh[3], 1, l1);
      // now q = (p0, p1); lane = (p2 .. p7): y = 4 * lane + q
      fb(0, 2, T[1]);  // stage 1
      fb(1, 3, T[1]);
      tab_at(tabs, L(11), T[1]);
      fb(0, 1, T[0]);  // stage 0
      fb(2, 3, T[1]);
    }
    // the output at equal priority (round 4: 11.00-11.03 against 11.05 ms with
    // w leading, which round 3 measured as the better one, 11.26 -> 11.19)
    __builtin_amdgcn_s_setprio(0);

    // ---- phase 5: y = 4*lane + q; columns col0 + 4*wave + c (decode_main:185-188,
    // reconstructSub:138-149).  No workgroup barrier: the operands were
    // requested before the transform.
    {
      uint32_t ra[4], rc[4];  // rows 4 lane .. + 3, group `wave`, as received
      {
        uint32_t ol2 = lane;
        asm volatile("" : "+v"(ol2));
        const uint32_t sa = lds_addr(stage) + stage_addr(4 * ol2, wave);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint2 d = lds_ld2(sa + 8 * q);
          ra[q] = d.x;
          rc[q] = d.y;
        }
      }
      uint32_t ol[4], oh[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t m = (meta[2 + (q >> 1)] >> (16 * (q & 1))) & 0xFFFFu;
        ol[q] = oh[q] = 0;
        if (m != 0xFFFFu) {
          mul_acc(ql[q], qh[q], T5[q], ol[q], oh[q]);
        } else {
          oh[q] = vperm(rc[q], ra[q], 0x06040200u);
          ol[q] = vperm(rc[q], ra[q], 0x07050301u);
        }
      }
      // column c of the group: 4 consecutive y -> 8 bytes BE
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
#pragma unroll
    for (int i = 0; i < 4; ++i) meta[i] = meta_next[i];
    __builtin_amdgcn_s_setprio(0);  // the next tile's gather: equal
  }
}

bool n1024_applicable(const CodeParams &p) { return p.n == 1024 && p.k == 256; }

// packed tiles: fewer columns per payload than a tile, or a shard pitch / base
// the 16-B row loads cannot take (any even pitch and base then)
bool n1024_packed(size_t slen, uintptr_t sh, size_t sstride) {
  return slen / 2 < size_t(COLS) || sh % 16 != 0 || sstride % 16 != 0;
}

hipError_t launch_reconstruct_n1024(const CodeParams &p, const DevTables &t,
                                    const uint8_t *d_shards, size_t slen, size_t sstride,
                                    const uint8_t *d_present, const uint16_t *d_err_log,
                                    const uint32_t *d_pattern,
                                    size_t batch, uint8_t *d_out, size_t ostride, void *scratch,
                                    hipStream_t s) {
  int cus = 0;
  // ECCR_AMD_RECON_PACKED=1 (experiments, scripts/ab_*): packed at every size
  static const bool force_packed = [] {
    const char *e = std::getenv("ECCR_AMD_RECON_PACKED");
    return e && e[0] == '1';
  }();
  const bool packed = force_packed || n1024_packed(slen, reinterpret_cast<uintptr_t>(d_shards), sstride);
  const size_t ncols4 = (slen / 2 + 3) / 4 * 4;
  if (packed && (reinterpret_cast<uintptr_t>(d_shards) % 2 != 0 || sstride % 2 != 0 ||
                 ncols4 * batch + COLS >= (size_t(1) << 32)))
    return hipErrorInvalidValue;
  const void *fn = packed ? reinterpret_cast<const void *>(&reconstruct_n1024<true>)
                          : reinterpret_cast<const void *>(&reconstruct_n1024<false>);
  if (const hipError_t e = prepare_kernel(fn, LDS_BYTES, &cus); e != hipSuccess) return e;
  uint32_t *order = nullptr;
  if (!packed) {  // the packed gather reads rows in natural order
    if (!scratch) return hipErrorInvalidValue;
    order = static_cast<uint32_t *>(scratch);  // gather_order_bytes(p, batch)
    if (const hipError_t e = launch_gather_order(p, d_present, d_err_log, d_pattern, batch, order, s);
        e != hipSuccess)
      return e;
  }
  const size_t tiles = packed ? ncols4 / 4 * batch : (slen / 2 + COLS - 1) / COLS * batch;  // packed: groups
  const unsigned grid = unsigned(tiles < size_t(cus) ? tiles : size_t(cus));
  if (packed)
    hipLaunchKernelGGL(reconstruct_n1024<true>, dim3(grid), dim3(THREADS), LDS_BYTES, s, d_shards,
                       uint64_t(slen), uint64_t(sstride), d_present, d_err_log, d_pattern, order,
                       d_out, uint64_t(ostride), int(p.nv), uint32_t(batch), uint32_t(ncols4), t);
  else
    hipLaunchKernelGGL(reconstruct_n1024<false>, dim3(grid), dim3(THREADS), LDS_BYTES, s, d_shards,
                       uint64_t(slen), uint64_t(sstride), d_present, d_err_log, d_pattern, order,
                       d_out, uint64_t(ostride), int(p.nv), uint32_t(batch), uint32_t(ncols4), t);
  return hipGetLastError();
}


}  // namespace ecamd
