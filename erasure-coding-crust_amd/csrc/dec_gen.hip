// dec_gen.hip — register-blocked reconstruct for n = 2^L, L = 6..10 (n = 64 ..
// 1024), any k with 16 <= k < n: the n_validators the n = 1024 / k = 256
// kernel does not cover (e.g. 512..765 validators: n = 1024, k = 128).
//
// A wave's 1024 positions (tf1024.hpp: 64 lanes x 16
// registers, 4 codewords per byte-planar register) are read as 1024 / n
// independent n-point codewords: position = (instance << L) | local.  Per
// codeword (decode_main, poly_encoder.hpp:164-189):
//   gather + scale the present received symbols by the locator E[v] into the
//   waves' regions (a workgroup tile is 32 * 1024 / n shard columns = 64 KB of
//   received rows), IFFT_n (passes A / B / C over the local stages), the
//   formal derivative in closed form c'[j] = c[j] ^ XOR_{b < L: j_b = 0}
//   c[j | 2^b] in whatever layout the IFFT ended in, the FFT_n restricted to
//   y < k (tf1024.hpp fft_restricted), and y < k out: erased y scaled by E[y]
//   (tables in LDS), present y copied from the shard.
// Stage arithmetic only sees the local bits, exactly as the reference's
// n-point transforms (additive_fft.hpp:99-141, skews at index 0).
#include <hip/hip_runtime.h>

#include "ec_kernels.hpp"
#include "tf1024.hpp"

namespace ecamd {
namespace {

using namespace tf;
constexpr int WAVES = 8;
constexpr int THREADS = 64 * WAVES;
using OutTabs = LdsTabs<128>;  // E[y], y < k <= 128, own area: filled once per payload
constexpr int LDS_BYTES = Tabs::kBytes + WAVES * REG_BYTES + OutTabs::kBytes;
static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");

__device__ __forceinline__ uint32_t mul_index(uint32_t c) { return c == 65535u ? 0u : c; }

// inverse pass over register bits 0..NS-1 (position bits B0..) of
// the local index pos & (n - 1); lb = tlin of the (masked) lane part
// When the pass holds the top local bit (B0 + NS == L), the lane part of a
// skew index has no bits above the stage, so a register block whose bits above
// the stage are 0 (blk < 2d) has skew skews[d - 1] = 0xFFFF: b ^= a only.
// Tower image 0: stages >= SM multiply with subfield tables.
constexpr int SM = tower_sub_min(0);
template <int B0, int NS, int L>
__device__ __forceinline__ void ipassg(S16 &s, const uint8_t *tabs, uint32_t lb) {
  constexpr uint32_t NM = (1u << L) - 1;
  constexpr bool TOP = B0 + NS == L;
  Tab T[2];
  SubTab U[2];
  const auto fetch = [&](int t, int blk, int slot) __attribute__((always_inline)) {
    const uint32_t a = lb ^ tlin(skew_idx((uint32_t(blk) << B0) & NM, B0 + t));
    if (B0 + t >= SM) tab_at(tabs, a, U[slot]);
    else tab_at(tabs, a, T[slot]);
  };
  fetch(0, 0, 0);
  int k = 0;
#pragma unroll
  for (int t = 0; t < NS; ++t) {
    const int d = 1 << t;
#pragma unroll
    for (int blk = 0; blk < 16; blk += 2 * d, ++k) {
      const int nt = blk + 2 * d < 16 ? t : t + 1, nblk = blk + 2 * d < 16 ? blk + 2 * d : 0;
      if (nt < NS) fetch(nt, nblk, (k + 1) & 1);
#pragma unroll
      for (int i = 0; i < d; ++i) {
        if (TOP && ((blk << B0) & NM) >> (B0 + t + 1) == 0) bx(s, blk + i, blk + i + d);
        else if (B0 + t >= SM) ib(s, blk + i, blk + i + d, U[k & 1]);
        else ib(s, blk + i, blk + i + d, T[k & 1]);
      }
    }
  }
}

// layout C, L = 9 or 10: stage 8 (pairs r bit 0, skew by p9 when local) and
// stage 9 (L = 10).  The transform is at index 0, so a stage's block at j = d
// has skew skews[d - 1] = 0xFFFF (no multiply): stage 9, and stage 8's block
// with p9 = 0 (for L = 9 p9 is an instance bit: all of stage 8), are b ^= a.
template <int L>
__device__ __forceinline__ void ipassCg(S16 &s, const uint8_t *tabs) {
#pragma unroll
  for (int hi = 0; hi < 4; ++hi) bx(s, 4 * hi, 4 * hi + 1);
  if constexpr (L == 10) {
    SubTab Tb;  // stage 8 >= SM
    tab_at(tabs, tlin(skew_idx(1u << 9, 8)), Tb);
#pragma unroll
    for (int hi = 0; hi < 4; ++hi) ib(s, 4 * hi + 2, 4 * hi + 3, Tb);
#pragma unroll
    for (int hi = 0; hi < 4; ++hi) {
      bx(s, 4 * hi, 4 * hi + 2);
      bx(s, 4 * hi + 1, 4 * hi + 3);
    }
  } else {
#pragma unroll
    for (int hi = 0; hi < 4; ++hi) bx(s, 4 * hi + 2, 4 * hi + 3);
  }
}


template <int L, int KB>
__global__ void __launch_bounds__(THREADS) reconstruct_gen(
    const uint8_t *__restrict__ shards, uint64_t slen, uint64_t sstride,
    const uint8_t *__restrict__ present, const uint16_t *__restrict__ elog,
    const uint32_t *__restrict__ pattern, const uint32_t *__restrict__ order,
    uint8_t *__restrict__ out, uint64_t ostride, int nv, int k, uint32_t batch, DevTables t) {
  constexpr int N = 1 << L;
  constexpr uint32_t NM = N - 1;
  constexpr int INST = 1024 >> L;          // codewords (x 4 columns) per wave
  constexpr int TC = WAVES * 4 * INST;     // shard columns per tile
  constexpr int CPR = TC * 2 / 16;         // 16-B chunks per received row
  constexpr int CPT = N * CPR / THREADS;   // chunks per thread (8)
  static_assert(N * CPR % THREADS == 0 && CPT == 8, "gather split");
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  uint8_t *tabs = lds;
  uint8_t *regions = lds + Tabs::kBytes;
  uint8_t *outtabs = regions + WAVES * REG_BYTES;
  const uint32_t tid0 = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid0 >> 6);
  uint8_t *my = regions + wave * REG_BYTES;

  Tabs::copy_image<THREADS>(tabs, t.timg_t, tid0);  // skews 0..1022 (index 0), tower image
  __syncthreads();

  // a contiguous range of tiles per workgroup, so consecutive tiles share a
  // payload and its locator state: the gather's per-row tables (registers)
  // and the output tables E[y] (LDS) are loaded once per payload, not per tile
  constexpr int RPT = CPR >= CPT ? 1 : CPT / CPR;  // received rows per thread (2 for n = 1024)
  constexpr int JPR = CPT / RPT;                   // chunks per row and thread
  const uint64_t ncols = slen / 2;
  const uint32_t tiles_pp = uint32_t((ncols + TC - 1) / TC);
  const uint64_t total = uint64_t(tiles_pp) * batch;
  const uint64_t per = (total + gridDim.x - 1) / gridDim.x;
  const uint64_t tile_end = per * (blockIdx.x + 1) < total ? per * (blockIdx.x + 1) : total;
  uint64_t cur_b = ~0ull;
  // this thread's received rows: slot rr * THREADS + tid (RPT = 2) or
  // tid * CPT / CPR (several threads per row) of the payload's gather order
  // (gather_order: present rows first, wave-major), so a wave whose rows are
  // all absent skips the gather's multiplies
  Tab RT[RPT];  // E[v] tables of this thread's received rows
  bool rhave[RPT];
  uint32_t rv[RPT];
  // the next tile's received rows are requested at the end of each gather and
  // land during the transform (same payload and a whole tile only)
  uint4 pre[CPT];
  bool pre_ok = false;
  for (uint64_t tile = per * blockIdx.x; tile < tile_end; ++tile) {
    uint32_t tid = tid0;
    asm volatile("" : "+v"(tid));
    const uint32_t lane = tid & 63;
    const uint64_t b = tile / tiles_pp;
    const uint64_t col0 = (tile % tiles_pp) * TC;
    const uint8_t *SH = shards + b * uint64_t(nv) * sstride;
    const uint64_t pt = pattern ? pattern[b] : b;  // erasure pattern of payload b
    const uint8_t *pr = present + pt * N;
    const uint16_t *E = elog + pt * N;
    uint8_t *O = out + b * ostride;

    __syncthreads();  // previous tile's readers of the regions / output tables are done
    if (b != cur_b) {  // new payload (uniform): its row tables and output tables
      cur_b = b;
#pragma unroll
      for (int rr = 0; rr < RPT; ++rr) {
        const uint32_t slot = RPT == 2 ? rr * THREADS + tid : tid * CPT / CPR;
        const uint32_t e = order[b * N + slot];
        rv[rr] = e >> 16;
        rhave[rr] = (e & 0xffffu) != 0xffffu;
        load_tab(t.mtab_tin, rhave[rr] ? (e & 0xffffu) : 0u, RT[rr]);  // scaled into tower coordinates
      }
#pragma unroll
      for (int it = 0; it < (128 * 5 + THREADS - 1) / THREADS; ++it) {  // k * 5 <= 640 chunks
        const uint32_t i = tid + it * THREADS;
        if (i < uint32_t(k) * 5)
          *reinterpret_cast<uint4 *>(outtabs + OutTabs::addr(i / 5, i % 5)) =
              reinterpret_cast<const uint4 *>(t.mtab_tout + mul_index(E[i / 5]))[i % 5];  // tower in
      }
    }

    // ---- gather + scale (decode_main:174-177): thread -> 8 consecutive
    // 16-B chunks (8 columns = 2 groups each) of the tile's received rows
    {
      const uint64_t avail = slen - 2 * col0;  // bytes of a row inside the tile
#pragma unroll
      for (int rr = 0; rr < RPT; ++rr) {
        const uint32_t cr = RPT == 2 ? 0u : (tid * CPT) % CPR;  // first chunk of the row
        const uint32_t v = rv[rr];
        const bool have = rhave[rr];
        const Tab &T = RT[rr];
#pragma unroll
        for (int j = 0; j < JPR; ++j) {
          const uint32_t c16 = cr + j;
          uint32_t w[4] = {0, 0, 0, 0};
          if (have && pre_ok) {
            const uint4 d = pre[rr * JPR + j];
            w[0] = d.x; w[1] = d.y; w[2] = d.z; w[3] = d.w;
          } else if (have) {
            const uint8_t *src = SH + uint64_t(v) * sstride + 2 * col0 + 16 * c16;
            if (16 * (c16 + 1) <= avail) {
              const uint4 d = *reinterpret_cast<const uint4 *>(src);
              w[0] = d.x; w[1] = d.y; w[2] = d.z; w[3] = d.w;
            } else {
              for (uint64_t e = 0; 16 * c16 + e < avail && e < 16; ++e)
                w[e >> 2] |= uint32_t(src[e]) << (8 * (e & 3));
            }
          }
#pragma unroll
          for (int h2 = 0; h2 < 2; ++h2) {  // columns 8 c16 + 4 h2 .. + 3 = group 2 c16 + h2
            const uint32_t g = 2 * c16 + h2, gw = g / INST, gi = g % INST;
            uint32_t l = 0, h = 0;
            if (have) {  // a wave with no present row skips (exec mask empty)
              const uint32_t a = w[2 * h2], c = w[2 * h2 + 1];
              mul_acc(vperm(c, a, 0x07050301u), vperm(c, a, 0x06040200u), T, l, h);
            }
            *reinterpret_cast<uint2 *>(regions + gw * REG_BYTES + raddr((gi << L) | v)) =
                make_uint2(l, h);
          }
        }
      }
      // prefetch the next tile's rows (uniform condition)
      const uint64_t nt = tile + 1, ncol0 = (nt % tiles_pp) * TC;
      pre_ok = nt < tile_end && nt / tiles_pp == b && 2 * (ncol0 + TC) <= slen;
      if (pre_ok) {
#pragma unroll
        for (int rr = 0; rr < RPT; ++rr) {
          const uint32_t cr = RPT == 2 ? 0u : (tid * CPT) % CPR;
          if (!rhave[rr]) continue;
#pragma unroll
          for (int j = 0; j < JPR; ++j)
            pre[rr * JPR + j] = *reinterpret_cast<const uint4 *>(
                SH + uint64_t(rv[rr]) * sstride + 2 * ncol0 + 16 * (cr + j));
        }
      }
    }
    __syncthreads();

    // ---- IFFT_n, derivative, FFT_n (back to layout A)
    S16 s;
    {
      const uint32_t la = region_lane<LA>(my, lane);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const uint2 x = lds_ld2(region_at<LA>(la, r));
        s.l[r] = x.x;
        s.h[r] = x.y;
      }
    }
    // table addresses are recomputed from an opaque lane for every pass: the
    // compiler would otherwise keep each pass's ~40 addresses live (spilled)
    // from the IFFT to the mirrored FFT pass
    auto lbA = [&] {
      uint32_t l = lane;
      asm volatile("" : "+v"(l));
      return tlin((16 * l) & NM);
    };
    auto lbB = [&] {  // p8, p9 when local
      uint32_t l = lane;
      asm volatile("" : "+v"(l));
      return tlin(((l >> 4) << 8) & NM);
    };
    // the two waves of a SIMD (w, w + 4) take turns at the higher issue
    // priority (pass A: w + 4, then w), as in reconstruct_n1024
    if (wave & 4) __builtin_amdgcn_s_setprio(2);
    else __builtin_amdgcn_s_setprio(0);
    ipassg<0, 4, L>(s, tabs, lbA());
    __builtin_amdgcn_sched_barrier(0);
    if (wave & 4) __builtin_amdgcn_s_setprio(0);
    else __builtin_amdgcn_s_setprio(2);
    exchange<LA, LB>(s, my, lane);
    if constexpr (L <= 8) {
      ipassg<4, L - 4, L>(s, tabs, lbB());
      __builtin_amdgcn_sched_barrier(0);
      derivative<LB, L, KB>(s, lane);
      __builtin_amdgcn_sched_barrier(0);
      fft_restricted<LB, L, KB, SM>(s, tabs, lane);
    } else {
      ipassg<4, 4, L>(s, tabs, lbB());
      __builtin_amdgcn_sched_barrier(0);
      exchange<LB, LC>(s, my, lane);
      ipassCg<L>(s, tabs);
      __builtin_amdgcn_sched_barrier(0);
      derivative<LC, L, KB>(s, lane);
      __builtin_amdgcn_sched_barrier(0);
      fft_restricted<LC, L, KB, SM>(s, tabs, lane);
    }
    __builtin_amdgcn_s_setprio(0);
#pragma unroll
    for (int r = 0; r < 16; ++r) asm volatile("" : "+v"(s.l[r]), "+v"(s.h[r]));  // finished here, not sunk into the output

    // ---- output (decode_main:185-188, reconstructSub:138-149): every live
    // register pair (r: p0 = 0, r | SB: p0 = 1) holds y0, y0 + 1 of one codeword
    // (position = p0 | lane bits 0.. -> p1.. | other register bits | in layout B
    // lane bits 4, 5 -> p8, p9); 4 bytes per column
    {
      constexpr Layout X = L <= 8 ? LB : LC;
      constexpr int SB = swap_rbit<X>(), NL = lane_stages<X>();
      uint32_t olane = lane;
      asm volatile("" : "+v"(olane));  // output addresses / shard re-reads not hoisted over the transform
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (((r >> SB) & 1) || !live_above<X, L, KB>(r & ~(1 << SB), KB - 1)) continue;
        uint32_t pos = ((olane & ((1u << NL) - 1)) << 1);
#pragma unroll
        for (int bb = 0; bb < 4; ++bb)
          if (bb != SB && ((r >> bb) & 1)) pos |= 1u << reg_pbit<X>(bb);
        if constexpr (X == LB) pos |= ((olane >> 4) & 3) << 8;
        const uint32_t gi = pos >> L, y0 = pos & NM;
        if (y0 >= uint32_t(k)) continue;
        const uint64_t cbase = col0 + 4 * (uint64_t(wave) * INST + gi);
        const bool full = cbase + 4 <= ncols;  // else the tile's last, partial group
        uint32_t ol[2], oh[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int rq = q ? (r | (1 << SB)) : r;
          const uint32_t y = y0 + q;
          const bool have = int(y) < nv && pr[y];
          Tab T;
          OutTabs::load(outtabs, y, T);
          uint32_t ml = 0, mh = 0;
          mul_acc(s.l[rq], s.h[rq], T, ml, mh);
          uint32_t a = 0, c = 0;
          const uint8_t *row = SH + uint64_t(have ? y : 0u) * sstride + 2 * cbase;
          if (full) {
            const uint2 d = *reinterpret_cast<const uint2 *>(row);
            a = d.x;
            c = d.y;
          } else if (have && cbase < ncols) {
            for (uint64_t e = 0; e < 2 * (ncols - cbase); ++e) {
              if (e < 4) a |= uint32_t(row[e]) << (8 * e);
              else c |= uint32_t(row[e]) << (8 * (e - 4));
            }
          }
          oh[q] = have ? vperm(c, a, 0x06040200u) : mh;
          ol[q] = have ? vperm(c, a, 0x07050301u) : ml;
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) {  // column c: y0, y0 + 1 -> 4 bytes BE
          const uint64_t col = cbase + c;
          if (col >= ncols) break;
          *reinterpret_cast<uint32_t *>(O + (col * uint64_t(k) + y0) * 2) =
              vperm(ol[0], oh[0], 0x0c0c0400u + 0x0101u * c) |
              (vperm(ol[1], oh[1], 0x0c0c0400u + 0x0101u * c) << 16);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
}

template <int L, int KB>
hipError_t launch_l(const CodeParams &p, const DevTables &t, const uint8_t *d_shards, size_t slen,
                    size_t sstride, const uint8_t *d_present, const uint16_t *d_err_log,
                                    const uint32_t *d_pattern,
                    size_t batch, uint8_t *d_out, size_t ostride, const uint32_t *order, hipStream_t s) {
  int cus = 0;
  if (const hipError_t e = prepare_kernel(reinterpret_cast<const void *>(&reconstruct_gen<L, KB>),
                                          LDS_BYTES, &cus);
      e != hipSuccess)
    return e;
  constexpr int TC = WAVES * 4 * (1024 >> L);
  const size_t tiles = (slen / 2 + TC - 1) / TC * batch;
  const unsigned grid = unsigned(tiles < size_t(cus) ? tiles : size_t(cus));
  hipLaunchKernelGGL((reconstruct_gen<L, KB>), dim3(grid), dim3(THREADS), LDS_BYTES, s, d_shards,
                     uint64_t(slen), uint64_t(sstride), d_present, d_err_log, d_pattern, order, d_out,
                     uint64_t(ostride), int(p.nv), int(p.k), uint32_t(batch), t);
  return hipGetLastError();
}

}  // namespace

bool decgen_applicable(const CodeParams &p) {  // the (n, k) instantiated below
  return (p.n == 64 && p.k == 16) || (p.n == 128 && (p.k == 16 || p.k == 32)) ||
         (p.n == 256 && (p.k == 32 || p.k == 64)) || (p.n == 512 && (p.k == 64 || p.k == 128)) ||
         (p.n == 1024 && p.k == 128);
}

hipError_t launch_reconstruct_gen(const CodeParams &p, const DevTables &t,
                                  const uint8_t *d_shards, size_t slen, size_t sstride,
                                  const uint8_t *d_present, const uint16_t *d_err_log,
                                  const uint32_t *d_pattern,
                                  size_t batch, uint8_t *d_out, size_t ostride, void *scratch,
                                  hipStream_t s) {
  if (!scratch) return hipErrorInvalidValue;
  uint32_t *order = static_cast<uint32_t *>(scratch);  // gather_order_bytes(p, batch)
  if (const hipError_t e = launch_gather_order(p, d_present, d_err_log, d_pattern, batch, order, s);
      e != hipSuccess)
    return e;
#define ECAMD_DG(Lv, KBv)                                                                   \
  if (p.n == (1u << Lv) && p.k == (1u << KBv))                                             \
    return launch_l<Lv, KBv>(p, t, d_shards, slen, sstride, d_present, d_err_log, d_pattern, batch, d_out, \
                             ostride, order, s);
  // every (n, k) of 46 <= n_validators <= 765 (decgen_applicable)
  ECAMD_DG(6, 4)
  ECAMD_DG(7, 4)
  ECAMD_DG(7, 5)
  ECAMD_DG(8, 5)
  ECAMD_DG(8, 6)
  ECAMD_DG(9, 6)
  ECAMD_DG(9, 7)
  ECAMD_DG(10, 7)
#undef ECAMD_DG
  return hipErrorInvalidValue;
}

}  // namespace ecamd
