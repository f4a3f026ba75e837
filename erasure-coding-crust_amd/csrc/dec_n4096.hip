// dec_n4096.hip — reconstruct specialised for n = 4096, k = 1024
// (n_validators 3070..4096; BASELINE config 4), instantiated as well for
// n = 2048 (two halves, stage 10 only across them) and for k = 256 / 512 (only
// the outputs y < k of the final FFT_1024 are written): n_validators 1025..4096.
//
// decode_main (poly_encoder.hpp:164-189) at n = 4096 per codeword (shard
// column): IFFT_4096 of the locator-scaled received word, formal derivative,
// FFT_4096 of which the k = 1024 outputs y < k are read.  Structure used:
//  * IFFT_4096 stages 0..9 act inside each quarter q (positions 1024q ..
//    1024q + 1023) with skew indices 1024q + (0..1022): four IFFT_1024 (tf1024.hpp)
//    with per-quarter tables;
//  * IFFT stages 10 / 11 across the quarters, the quarter bits of the formal
//    derivative and FFT stages 11 / 10 on the side that reaches y < 1024 are
//    folded into two accumulators (constants from the host, n4096_lin), each
//    quarter added in as soon as it is transformed; the within-quarter
//    derivative in closed form c'[j] = c[j] ^ XOR_{b < 10: j_b = 0} c[j | 2^b]
//    (poly_encoder.hpp:195-215);
//  * one FFT_1024 (index 0): whole for k = 1024, restricted to y < k otherwise.
// A wave owns one byte-planar group (4 columns) for the whole tile, in layout
// C.  The workgroup (8 waves, 32 columns) shares one
// 80 KB multiply-table set in LDS, reloaded per quarter (3, 2, 1, then 0, which
// stays for the FFT) and finally replaced by the output tables E[y], y < k.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "ec_kernels.hpp"
#include "tf1024.hpp"

namespace ecamd {
namespace {

using namespace tf;
constexpr int WAVES = 8;
constexpr int THREADS = 64 * WAVES;
constexpr int COLS = 4 * WAVES;
constexpr uint32_t SLOT = Tabs::kBytes + WAVES * REG_BYTES;  // the next tile's index
constexpr int LDS_BYTES = int(SLOT + 16);
static_assert(LDS_BYTES <= 160 * 1024 && Tabs::kBytes == kTabImageBytes, "LDS budget");

__device__ __forceinline__ uint32_t mul_index(uint32_t c) { return c == 65535u ? 0u : c; }

// multiplier logs (65535 = multiply by zero) of the linearised cross-quarter part
// The data runs in tower coordinates; every p_q / k_q is a
// subfield element (skews 1023 / 2047 / 3071 are 0, 0 and 2: p, k in {0, 1, 2, 3}),
// multiplied with its subfield table ps / ks.
struct Lin {
  uint32_t p[4], k[4];
  uint32_t ps[4][5], ks[4][5];
};

// Fold IFFT stages 10 (skews 1023 / 3071) and 11 (2047), the quarter bits of
// the formal derivative and FFT stages 11 / 10 (a-side only) into
// y = D(sum p_q u_q) + sum k_q u_q, by pushing u_q = 1 through them with the
// reference's butterflies (additive_fft.hpp:99-141; skews[] == 0xFFFF: no
// multiply).  Derivative quarter terms (poly_encoder.hpp:195-215):
// c'0 = Dc0 + c1 + c2, c'1 = Dc1 + c3, c'2 = Dc2 + c3, c'3 = Dc3.
Lin n4096_lin(int nq) {
  const Field &f = field();
  const auto mul = [&](uint16_t x, uint16_t c) -> uint16_t { return c == 0xFFFF ? 0 : f.mul(x, c); };
  const uint16_t sa = f.skews[1023], sb = f.skews[3071], sc = f.skews[2047];
  Lin lin{};
  for (int q = 0; q < 4; ++q) {
    uint16_t u[4] = {0, 0, 0, 0}, P = 0, Q = 0;
    if (q < nq) u[q] = f.exp[0];  // the multiplicative identity
    if (nq == 4) {
      const uint16_t u1 = u[1] ^ u[0], u0 = u[0] ^ mul(u1, sa);
      const uint16_t u3 = u[3] ^ u[2], u2 = u[2] ^ mul(u3, sb);
      const uint16_t c2 = u2 ^ u0, c0 = u0 ^ mul(c2, sc);
      const uint16_t c3 = u3 ^ u1, c1 = u1 ^ mul(c3, sc);
      // y = c'0 + sc c'2 + sa (c'1 + sc c'3) = D(c0 + sa c1 + sc c2 + sa sc c3) + c1 + c2 + (sa + sc) c3
      P = c0 ^ mul(c1, sa) ^ mul(c2, sc) ^ mul(mul(c3, sc), sa);
      Q = c1 ^ c2 ^ mul(c3, sc) ^ mul(c3, sa);
    } else {
      const uint16_t c1 = u[1] ^ u[0], c0 = u[0] ^ mul(c1, sa);
      // y = c'0 + sa c'1 = D(c0 + sa c1) + c1
      P = c0 ^ mul(c1, sa);
      Q = c1;
    }
    lin.p[q] = P ? f.log[P] : 65535u;
    lin.k[q] = Q ? f.log[Q] : 65535u;
    // subfield elements (tests/cpp/tower_check.cpp checks the skews' elements)
    const MulTabSub sp = f.sub_tab(P < 256 ? lin.p[q] : 65535u), sk = f.sub_tab(Q < 256 ? lin.k[q] : 65535u);
    for (int i = 0; i < 5; ++i) {
      lin.ps[q][i] = sp.w[i];
      lin.ks[q][i] = sk.w[i];
    }
    if (P >= 256 || Q >= 256) lin.p[0] = 0xDEAD;  // never: launch refuses (n4096_lin_ok)
  }
  return lin;
}

// Per payload, the LDS image (LdsTabs<1024> layout, as DevTables::timg) of
// its output tables E[y], y < 1024 (decode_main:185-188): the k = 1024
// reconstruct fills its output tables with one linear LDS-DMA per tile
// instead of a per-tile gather of 1024 indexed 80-byte tables (two dependent
// global latencies).  Chunk i of the image is plane i / 1024, slot i % 1024 of
// entry y = (slot & ~15) | f with LdsTabs::addr's swizzle f inverted.  After
// the image, the payload's present mask of y < 1024 (bit y of dword y / 32: row
// y is received), read by the reconstruct at its tile start so that the output
// phase's received-row loads can be issued before the final FFT.
constexpr size_t kOutImageBytes = kTabImageBytes + 1024 / 8;
__global__ void __launch_bounds__(256)
    n4096_out_image(const uint16_t *__restrict__ elog, const uint8_t *__restrict__ present,
                    const uint32_t *__restrict__ pattern, int n, int nv,
                    const MulTab *__restrict__ mtab, uint8_t *__restrict__ img) {
  const uint64_t b = blockIdx.x, pt = pattern ? pattern[b] : b;
  const uint16_t *E = elog + pt * uint64_t(n);
  uint4 *dst = reinterpret_cast<uint4 *>(img + b * kOutImageBytes);
  for (uint32_t i = threadIdx.x; i < 5 * 1024; i += 256) {
    const uint32_t q = i >> 10, sl = i & 1023;
    const uint32_t y = (sl & ~15u) | ((sl ^ (sl >> 4) ^ (sl >> 8)) & 15u);
    dst[i] = reinterpret_cast<const uint4 *>(mtab + mul_index(E[y]))[q];
  }
  if (threadIdx.x < 32) {
    const uint8_t *pr = present + pt * uint64_t(n);
    uint32_t m = 0;
    for (uint32_t j = 0; j < 32; ++j) {
      const uint32_t y = 32 * threadIdx.x + j;
      m |= uint32_t(int(y) < nv && pr[y]) << j;
    }
    reinterpret_cast<uint32_t *>(img + b * kOutImageBytes + kTabImageBytes)[threadIdx.x] = m;
  }
}

}  // namespace

// layout C after the restricted FFT: y0 = (lane << 1) | reg_pos(r, swap bit),
// the register part only in y bits 7.. (the output's mask dword md[R >> 7])
constexpr bool regbits_above_lane() {
  for (int r = 0; r < 16; ++r)
    if (reg_pos<LC, 10>(r, swap_rbit<LC>()) & 127u) return false;
  return true;
}

// NQ = n / 1024 quarters (2 or 4); K = k = 2^KB (256, 512 or 1024)
template <int NQ, int KB>
__global__ void __launch_bounds__(THREADS)
reconstruct_n4096(
    const uint8_t *__restrict__ shards, uint64_t slen, uint64_t sstride,
    const uint8_t *__restrict__ present, const uint16_t *__restrict__ elog,
    const uint32_t *__restrict__ pattern, const uint32_t *__restrict__ order,
    uint8_t *__restrict__ out, uint64_t ostride, int nv, uint32_t K, uint32_t batch,
    DevTables t, Lin lin, const uint8_t *__restrict__ oimg, uint32_t *__restrict__ tick) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  uint8_t *tabs = lds;
  uint8_t *regions = lds + Tabs::kBytes;
  const uint32_t tid0 = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid0 >> 6);
  uint8_t *my = regions + wave * REG_BYTES;

  const uint64_t ncols = slen / 2;
  const uint32_t tiles_pp = uint32_t((ncols + COLS - 1) / COLS);
  const uint64_t total = uint64_t(tiles_pp) * batch;
  // n = 4096: dynamic XCD-affine schedule (TileQueue; config 4 reconstruct
  // 7.64 -> 7.37 ms at B = 2048): thread 0 takes the tile after this one at
  // the tile start and publishes it before the output phase's first barrier;
  // every wave reads it right after that barrier; the slot is rewritten only
  // in the next tile, after several barriers.  n = 2048: the static XCD spans
  // (its shorter tiles ran 2-3% slower dynamically at n_validators 1500)
  constexpr bool DYN = NQ == 4;
  const TileQueue tq(uint32_t(total), tick);  // total < 2^32 (launch)
  const TileSpan span = xcd_span(total);
  auto *slot = reinterpret_cast<__attribute__((address_space(3))) volatile uint32_t *>(uintptr_t(SLOT));
  uint64_t tile = span.first, end = span.end;
  if constexpr (DYN) {
    if (tid0 == 0) *slot = tq.take();
    __syncthreads();
    tile = __builtin_amdgcn_readfirstlane(*slot);
    end = tq.hi;
  }
  while (tile < end) {
    uint64_t nxt = tile + span.step;  // (static)
    uint32_t taken = 0;
    if constexpr (DYN)
      if (tid0 == 0) taken = tq.take();
    uint32_t tid = tid0;
    asm volatile("" : "+v"(tid));
    const uint32_t lane = tid & 63;
    const uint64_t b = tile / tiles_pp;
    const uint64_t col0 = (tile % tiles_pp) * COLS;
    const uint8_t *SH = shards + b * uint64_t(nv) * sstride;
    uint8_t *O = out + b * ostride;
    // n4096_out_image's mask of the received rows y < k: bit i of pw[j] = row
    // (k / 8) wave + 32 j + i (wave-uniform, for the staging DMA); k = 1024: bit r
    // of pm = row 16 lane + r (the output rows of the lane)
    const uint32_t *mask = reinterpret_cast<const uint32_t *>(oimg + b * kOutImageBytes + kTabImageBytes);
    constexpr int MPW = (1 << KB) / 256;  // mask dwords per wave
    uint32_t pw[MPW];
#pragma unroll
    for (int j = 0; j < MPW; ++j) pw[j] = mask[MPW * wave + j];
    uint32_t pm = 0;
    if constexpr (KB == 10) pm = mask[lane >> 1] >> (16 * (lane & 1));
    S16 P, Qa;  // the two accumulators of the linearised cross-quarter stages
    // a wave whose 4 columns lie past the payload's last one (its last, partial
    // tile: 1 MB at k = 1024 is 489 columns, the 16th tile has 9) gathers with
    // the others but skips its transforms and output (uniform)
    const bool idle = col0 + 4 * wave >= ncols;
    // this thread's two gather slots of a quarter (gather_order, dec_n1024.hip:
    // present rows first, dealt wave-major): (row in quarter << 16) |
    // mul_index(E[row]), low half 0xFFFF = absent.  The next quarter's are
    // loaded right after a quarter's gather, so its gather waits on one global
    // latency (the table and the row) instead of two.
    uint32_t mq[1024 / THREADS];
    const auto load_meta = [&](const int q, const uint32_t tq) __attribute__((always_inline)) {
#pragma unroll
      for (int half = 0; half < 1024 / THREADS; ++half)
        mq[half] = order[(b * NQ + q) * 1024 + half * THREADS + tq];
    };
    const auto has = [&](int half) { return (mq[half] & 0xffffu) != 0xffffu; };

    // ---- IFFT quarters 3, 2, 1, 0 (quarter 0's tables stay for the FFT), each
    // folded into P and Qa as soon as it is transformed.  A quarter's table
    // image is requested (LDS-DMA) as soon as every wave is done with the
    // previous quarter's IFFT, so it lands behind that quarter's accumulation
    // and this quarter's row gather; the first gather row and its E[v] table
    // are requested before that barrier (registers only).
    uint32_t w0[16];  // this thread's first gather slot of the next quarter
    Tab RT0;
    const uint64_t avail = slen - 2 * col0;
    const auto load_row = [&](const int q, const int half, uint32_t (&w)[16], Tab &RT) __attribute__((always_inline)) {
      const uint8_t *row = SH + uint64_t(1024 * q + (mq[half] >> 16)) * sstride + 2 * col0;
      if (avail >= 64) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint4 d = reinterpret_cast<const uint4 *>(row)[j];
          w[4 * j] = d.x;
          w[4 * j + 1] = d.y;
          w[4 * j + 2] = d.z;
          w[4 * j + 3] = d.w;
        }
      } else {
        load_row_tail64(row, avail, w);
      }
      load_tab(t.mtab_tin, mq[half] & 0xffffu, RT);  // scaled into tower coordinates
    };
    // qc: std::integral_constant quarter (its tower image's subfield stages)
    const auto quarter = [&](auto qc, const int qnext) __attribute__((always_inline)) {
      constexpr int q = decltype(qc)::value;
      S16 Qq;
      __builtin_amdgcn_sched_barrier(0);
      uint32_t tq = tid;
      asm volatile("" : "+v"(tq));  // this quarter's addresses and loads are not hoisted above here
      const uint32_t lq = tq & 63;
      // gather + scale the quarter's present rows (decode_main:174-177) into
      // the 8 groups' regions: thread -> rows 1024q + tid, + 512
#pragma unroll
      for (int half = 0; half < 1024 / THREADS; ++half) {
        const uint32_t vl = mq[half] >> 16;
        uint32_t l[8], h[8];
#pragma unroll
        for (int g = 0; g < 8; ++g) l[g] = h[g] = 0;
        if (has(half)) {
          uint32_t w1[16];
          Tab RT1;
          if (half > 0) load_row(q, half, w1, RT1);
          const uint32_t *w = half > 0 ? w1 : w0;
          const Tab &RT = half > 0 ? RT1 : RT0;
#pragma unroll
          for (int g = 0; g < 8; ++g) {
            const uint32_t a = w[2 * g], c = w[2 * g + 1];
            const uint32_t xh = vperm(c, a, 0x06040200u), xl = vperm(c, a, 0x07050301u);
            mul_acc(xl, xh, RT, l[g], h[g]);
          }
        }
#pragma unroll
        for (int g = 0; g < 8; ++g)
          *reinterpret_cast<uint2 *>(regions + g * REG_BYTES + raddr(vl)) = make_uint2(l[g], h[g]);
      }
      if (qnext >= 0) load_meta(qnext, tq);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // table image landed
      lds_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (!idle) {
        const uint32_t la = region_lane<LA>(my, lq);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const uint2 x = lds_ld2(region_at<LA>(la, r));
          Qq.l[r] = x.x;
          Qq.h[r] = x.y;
        }
        // n = 2048: the two waves of a SIMD (w, w + 4) alternate the higher
        // issue priority from half to half (as reconstruct_n1024's passes);
        // n = 4096: equal priority (alternating: config 4 reconstruct 7.81
        // against 7.65 ms; n = 2048 without: 2.92-2.98 against 2.88-2.89)
        if (NQ == 2 && (((wave >> 2) ^ uint32_t(q)) & 1)) __builtin_amdgcn_s_setprio(2);
        else __builtin_amdgcn_s_setprio(0);
        // -> layout C; quarter 0 is at index 0
        ifft1024<q == 0, tower_sub_min(q)>(Qq, tabs, my, lq);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (qnext >= 0) {  // the next quarter's first row and tables
        if (has(0)) load_row(qnext, 0, w0, RT0);
        lds_barrier();  // every wave is done with this quarter's tables and its region
        Tabs::dma_image<THREADS>(tabs, t.timg_t + qnext * kTabImageBytes, tq);
        __builtin_amdgcn_sched_barrier(0);
      }
      // P += p_q u_q, Qa += k_q u_q.  The constants are mostly 0 or 1 (the
      // skews at 1023 and 2047 are 0xFFFF: n = 4096 gives p = (1, 0, 0, 0),
      // k = (0, 1, 1 + s, s); n = 2048 p = (1, 0), k = (1, 1)), so each is a
      // uniform branch: skip (log 65535 = zero), XOR (log 0 = one) or multiply.
      // Qa is read at the registers reaching y < k only; P also at their
      // single-bit partners (the derivative): everywhere but r & 3 == 3
      // (p8 = p9 = 1) when k = 256.
      if (idle) return;
      uint32_t ip = lin.p[q], ik = lin.k[q];
      asm volatile("" : "+s"(ip), "+s"(ik));  // loaded here, not hoisted (and kept live) from the top
      if (ip == 0) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          P.l[r] ^= Qq.l[r];
          P.h[r] ^= Qq.h[r];
        }
      } else if (ip != 65535u) {
        SubTab TP;
#pragma unroll
        for (int i = 0; i < 5; ++i) TP.t[i] = lin.ps[q][i];
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (KB >= 9 || (r & 3) != 3) mul_acc_sub(Qq.l[r], Qq.h[r], TP, P.l[r], P.h[r]);
      }
      if (ik == 0) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (live_above<LC, 10, KB>(r, KB - 1)) {
            Qa.l[r] ^= Qq.l[r];
            Qa.h[r] ^= Qq.h[r];
          }
      } else if (ik != 65535u) {
        SubTab TK;
#pragma unroll
        for (int i = 0; i < 5; ++i) TK.t[i] = lin.ks[q][i];
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (live_above<LC, 10, KB>(r, KB - 1)) mul_acc_sub(Qq.l[r], Qq.h[r], TK, Qa.l[r], Qa.h[r]);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r)  // accumulated here, not sunk into the next quarter's gather
        asm volatile("" : "+v"(P.l[r]), "+v"(P.h[r]), "+v"(Qa.l[r]), "+v"(Qa.h[r]));
      __builtin_amdgcn_sched_barrier(0);
    };
#pragma unroll
    for (int r = 0; r < 16; ++r) P.l[r] = P.h[r] = Qa.l[r] = Qa.h[r] = 0;
    // a quarter wholly at or above n_validators holds no received symbol: its
    // IFFT is zero and adds nothing (n = 4096 with n_validators <= 3072)
    const int qfirst = NQ == 4 && 3 * 1024 < nv ? 3 : NQ == 4 ? 2 : 1;
    load_meta(qfirst, tid);
    if (has(0)) load_row(qfirst, 0, w0, RT0);
    lds_barrier();  // every wave is done with the last tile's output tables and its region
    Tabs::dma_image<THREADS>(tabs, t.timg_t + qfirst * kTabImageBytes, tid);
    if constexpr (NQ == 4) {
      if (3 * 1024 < nv) quarter(std::integral_constant<int, 3>(), 2);
      quarter(std::integral_constant<int, 2>(), 1);
    }
    quarter(std::integral_constant<int, 1>(), 0);
    quarter(std::integral_constant<int, 0>(), -1);

    // ---- cross-quarter IFFT stages (10, 11), the quarter bits of the formal
    // derivative and FFT stages 11 / 10 on the side that reaches y < 1024 are
    // all GF-linear with constant multipliers, so the FFT_1024 input is
    //   y = D(P) + Qa,  P = sum_q p_q u_q,  Qa = sum_q k_q u_q
    // (u_q = IFFT_1024 of quarter q, D = the within-quarter derivative, p_q /
    // k_q folded on the host from skews 1023 / 2047 / 3071: n4096_lin()).
    // D in closed form (poly_encoder.hpp:195-215) over bits 0..9, in place:
    // lane = p0..p5, r = (p8, p9, p6, p7).
    __builtin_amdgcn_s_setprio(0);
    S16 Y;
    const uint64_t cbase = col0 + 4 * wave;
    const bool full = cbase + 4 <= ncols;
    if (!idle) {
      derivative<LC, 10, KB>(P, lane);  // at the registers reaching y < k only
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        Y.l[r] = P.l[r] ^ Qa.l[r];
        Y.h[r] = P.h[r] ^ Qa.h[r];
      }

      // ---- FFT_1024, index 0 (quarter 0's tables still resident): whole for
      // k = 1024 (-> layout A: y = 16 lane + r), else restricted to y < k
      // (tf1024.hpp fft_restricted: live register pairs hold y0, y0 + 1)
      if constexpr (KB == 10) fft1024<true, tower_sub_min(0)>(Y, tabs, my, lane);
      else fft_restricted<LC, 10, KB, tower_sub_min(0)>(Y, tabs, lane);
#pragma unroll
      for (int r = 0; r < 16; ++r) asm volatile("" : "+v"(Y.l[r]), "+v"(Y.h[r]));  // not sunk past the table gather
    }

    // ---- output (decode_main:185-188, reconstructSub:138-149): erased y < k
    // scaled by E[y] (tables now in LDS), present y copied from the shard
    if constexpr (DYN)
      if (tid0 == 0) *slot = taken;  // (issued at the tile start: long returned)
    lds_barrier();  // every wave is done with the FFT tables
    if constexpr (DYN) nxt = __builtin_amdgcn_readfirstlane(*slot);
    // the output tables E[y] from this payload's prebuilt image (n4096_out_image)
    __builtin_amdgcn_sched_barrier(0);
    Tabs::dma_image<THREADS>(tabs, oimg + b * kOutImageBytes, tid);
    const bool staged = col0 + COLS <= ncols;  // the received rows y < k go through the regions
    if (staged) {
      // their 64-B tile segments -> the regions, by LDS-DMA in the same latency:
      // 1 KB window w = rows 16 w .. 16 w + 15, 16-B slot (4 (y & 15) + chunk) ^
      // (w & 15) (swizzled so that the reads below, one row per lane, spread
      // over the banks); each wave fills k / 128 windows
#pragma unroll
      for (int j = 0; j < 2 * MPW; ++j) {
        const uint32_t W = 2 * MPW * wave + j, l = lane ^ (W & 15);
        const uint32_t yy = l >> 2;
        if ((pw[j >> 1] >> (16 * (j & 1) + yy)) & 1)
          lds_dma16(lds_addr(regions) + 1024 * W, SH + uint64_t(16 * W + yy) * sstride + 2 * col0 + 16 * (l & 3));
      }
    }
    // k < 1024: mask dwords (lane >> 4) + 4 m (rows y0 = 2 lane + 128 m + (0, 1))
    uint32_t md[KB < 10 ? (1 << KB) / 128 : 1];
    if constexpr (KB < 10) {
#pragma unroll
      for (int m = 0; m < (1 << KB) / 128; ++m) md[m] = mask[(lane >> 4) + 4 * m];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    lds_barrier();
    if (idle) {
      tile = nxt;
      continue;
    }
    if constexpr (KB < 10) {
      constexpr int SB = swap_rbit<LC>();
      static_assert(regbits_above_lane(), "the output rows' register bits are y bits 7..");
      uint32_t olane = lane;
      asm volatile("" : "+v"(olane));
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (((r >> SB) & 1) || !live_above<LC, 10, KB>(r & ~(1 << SB), KB - 1)) continue;
        const uint32_t R = reg_pos<LC, 10>(r, SB);  // y bits 7.. (regbits_above_lane)
        const uint32_t y0 = (olane << 1) | R;
        uint32_t ol[2], oh[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int rq = q ? (r | (1 << SB)) : r;
          const uint32_t y = y0 + q;
          const bool have = (md[R >> 7] >> ((y0 & 31) + q)) & 1;  // int(y) < nv && pr[y]
          Tab T;
          Tabs::load(tabs, y, T);
          uint32_t ml = 0, mh = 0;
          mul_acc(Y.l[rq], Y.h[rq], T, ml, mh);
          uint32_t a = 0, c = 0;
          const uint8_t *row = SH + uint64_t(have ? y : 0u) * sstride + 2 * cbase;
          if (staged) {
            if (have) {
              const uint2 d = lds_ld2(lds_addr(regions) + 1024 * (y >> 4) +
                                      16 * ((4 * (y & 15) + (wave >> 1)) ^ ((y >> 4) & 15)) + 8 * (wave & 1));
              a = d.x;
              c = d.y;
            }
          } else if (full) {
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
          *reinterpret_cast<uint32_t *>(O + (col * uint64_t(K) + y0) * 2) =
              vperm(ol[0], oh[0], 0x0c0c0400u + 0x0101u * c) |
              (vperm(ol[1], oh[1], 0x0c0c0400u + 0x0101u * c) << 16);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
      uint32_t ol[16], oh[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const uint32_t y = 16 * lane + r;
        ol[r] = oh[r] = 0;
        if ((pm >> r) & 1) {  // int(y) < nv && pr[y]
          const uint8_t *row = SH + uint64_t(y) * sstride + 2 * cbase;
          uint32_t a = 0, c = 0;
          if (staged) {
            const uint2 d = lds_ld2(lds_addr(regions) + 1024 * lane + 16 * ((4 * r + (wave >> 1)) ^ (lane & 15)) +
                                    8 * (wave & 1));
            a = d.x;
            c = d.y;
          } else if (full) {
            const uint2 d = *reinterpret_cast<const uint2 *>(row);
            a = d.x;
            c = d.y;
          } else {
            for (uint64_t e = 0; e < 2 * (ncols > cbase ? ncols - cbase : 0); ++e) {
              if (e < 4) a |= uint32_t(row[e]) << (8 * e);
              else c |= uint32_t(row[e]) << (8 * (e - 4));
            }
          }
          oh[r] = vperm(c, a, 0x06040200u);
          ol[r] = vperm(c, a, 0x07050301u);
        } else {
          Tab T;
          Tabs::load(tabs, y, T);
          mul_acc(Y.l[r], Y.h[r], T, ol[r], oh[r]);
        }
      }
      // column c: y = 16 lane .. 16 lane + 15 -> 32 contiguous bytes (BE symbols)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const uint64_t col = cbase + c;
        if (col >= ncols) break;
        uint32_t wd[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
          wd[j] = vperm(ol[2 * j], oh[2 * j], 0x0c0c0400u + 0x0101u * c) |
                  (vperm(ol[2 * j + 1], oh[2 * j + 1], 0x0c0c0400u + 0x0101u * c) << 16);
        uint8_t *dst = O + (col * K + 16 * lane) * 2;
        reinterpret_cast<uint4 *>(dst)[0] = make_uint4(wd[0], wd[1], wd[2], wd[3]);
        reinterpret_cast<uint4 *>(dst)[1] = make_uint4(wd[4], wd[5], wd[6], wd[7]);
      }
    }
    tile = nxt;
  }
}

size_t n4096_scratch_bytes(const CodeParams &p, size_t batch) {
  return gather_order_bytes(p, batch) + batch * kOutImageBytes + kTileQueueBytes;
}

bool n4096_applicable(const CodeParams &p) {  // the (n, k) instantiated below
  return (p.n == 4096 && (p.k == 1024 || p.k == 512)) || (p.n == 2048 && (p.k == 512 || p.k == 256));
}

hipError_t launch_reconstruct_n4096(const CodeParams &p, const DevTables &t,
                                    const uint8_t *d_shards, size_t slen, size_t sstride,
                                    const uint8_t *d_present, const uint16_t *d_err_log,
                                    const uint32_t *d_pattern,
                                    size_t batch, uint8_t *d_out, size_t ostride, void *scratch,
                                    hipStream_t s) {
  int cus = 0;
  const void *fn = nullptr;
  if (p.n == 4096) fn = p.k == 1024 ? reinterpret_cast<const void *>(&reconstruct_n4096<4, 10>)
                                    : reinterpret_cast<const void *>(&reconstruct_n4096<4, 9>);
  else fn = p.k == 512 ? reinterpret_cast<const void *>(&reconstruct_n4096<2, 9>)
                       : reinterpret_cast<const void *>(&reconstruct_n4096<2, 8>);
  if (const hipError_t e = prepare_kernel(fn, LDS_BYTES, &cus); e != hipSuccess) return e;
  if (!scratch) return hipErrorInvalidValue;
  uint32_t *order = static_cast<uint32_t *>(scratch);  // n4096_scratch_bytes(p, batch)
  if (const hipError_t e = launch_gather_order(p, d_present, d_err_log, d_pattern, batch, order, s);
      e != hipSuccess)
    return e;
  uint8_t *oimg = static_cast<uint8_t *>(scratch) + gather_order_bytes(p, batch);
  hipLaunchKernelGGL(n4096_out_image, dim3(unsigned(batch)), dim3(256), 0, s, d_err_log, d_present, d_pattern,
                       int(p.n), int(p.nv), t.mtab_tout, oimg);  // tower in, symbols out
  const size_t tiles = (slen / 2 + COLS - 1) / COLS * batch;
  if (tiles >= (size_t(1) << 32) - size_t(2) * cus) return hipErrorInvalidValue;
  uint32_t *tick = reinterpret_cast<uint32_t *>(oimg + batch * kOutImageBytes);  // the TileQueue counters
  if (const hipError_t e = launch_zero_counters(tick, kTileQueueBytes, s); e != hipSuccess) return e;
  const unsigned grid = unsigned(tiles < size_t(cus) ? tiles : size_t(cus));
  static const Lin lin4 = n4096_lin(4), lin2 = n4096_lin(2);
  if (lin4.p[0] == 0xDEAD || lin2.p[0] == 0xDEAD) return hipErrorInvalidValue;  // not subfield (never)
#define ECAMD_D4(NQv, KBv)                                                                    \
  if (p.n == 1024u * NQv && p.k == (1u << KBv))                                                  \
    hipLaunchKernelGGL((reconstruct_n4096<NQv, KBv>), dim3(grid), dim3(THREADS), LDS_BYTES, s,   \
                       d_shards, uint64_t(slen), uint64_t(sstride), d_present, d_err_log, d_pattern, order, d_out, \
                       uint64_t(ostride), int(p.nv), uint32_t(p.k), uint32_t(batch), t,         \
                       NQv == 4 ? lin4 : lin2, oimg, tick);
  ECAMD_D4(4, 10)
  else ECAMD_D4(4, 9)
  else ECAMD_D4(2, 9)
  else ECAMD_D4(2, 8)
  else return hipErrorInvalidValue;
#undef ECAMD_D4
  return hipGetLastError();
}

}  // namespace ecamd
