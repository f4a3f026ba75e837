// enc_gen.hip — register-blocked encode for k = 2^M, M = 4..9 (k = 16 .. 512)
// and n <= 4096: n_validators 46..3069 outside the k = 256 / n = 1024 and
// k = 1024 / n = 4096 kernels; this includes today's Polkadot validator counts
// (k = 128, n = 1024 for 512..765 validators) and n = 2048 / 4096 with k = 256 / 512.
//
// The 1024 positions a wave holds (tf1024.hpp: 64 lanes x 16 registers, 4
// pieces per byte-planar register) are read as 1024 / k independent k-point
// transforms: position = (instance << M) | local, so a wave encodes
// 4 * 1024 / k pieces at once.  encodeLow (poly_encoder.hpp:217-240):
//   IFFT_k  = pass A (stages 0-3, register bits = position bits 0-3) and, after
//             the A -> B exchange, pass B (stages 4..M-1): ends in layout B;
//   FFT_k at each coset s = k, 2k, .. < n: pass B (stages M-1..4), B -> A
//             exchange, pass A (stages 3..0): ends in layout A = shard rows.
// Stage index arithmetic only sees the local bits (pos & (k-1)); instance bits
// ride along as extra register / lane bits.  k = 512 adds stage 8, done in
// layout C (IFFT: A -> B -> C, coset FFT: C -> B -> A).  Skews 1024q .. 1024q +
// 1023 are LDS table image q; a coset s uses image s / 1024 at offset s % 1024,
// folded into the linear table address (tlin): n <= 1024 needs image 0 only,
// n = 2048 / 4096 reload the image when s crosses a multiple of 1024 (and
// image 0 again for the next tile's IFFT).
//
// Shard rows: per coset, k rows x 32 * 1024 / k pieces (64 KB) are staged in the
// waves' own regions (row v of wave w: 8 * 1024 / k bytes) and stored as 16-B
// lane chunks of contiguous row segments (64 * 1024 / k bytes).
#include <hip/hip_runtime.h>

#include <type_traits>

#include "ec_kernels.hpp"
#include "tf1024.hpp"

namespace ecamd {
namespace {

using namespace tf;
constexpr int WAVES = 8;
constexpr int THREADS = 64 * WAVES;
constexpr int SLOT = Tabs::kBytes + WAVES * REG_BYTES;  // the next tile's index (dynamic schedule)
constexpr int LDS_BYTES = SLOT + 16;
static_assert(LDS_BYTES <= 160 * 1024 && Tabs::kBytes == kTabImageBytes, "LDS budget");

template <int M>
struct Geo {
  static constexpr uint32_t K = 1u << M;
  static constexpr int INST = 1024 >> M;  // transforms per wave
  static constexpr int WP = 4 * INST;     // pieces per wave
  static constexpr int TP = WAVES * WP;   // pieces per tile
  static constexpr int ROWB = 2 * WP;     // bytes of one shard row per wave and tile
};

// inverse pass over register bits 0..NS-1 = position bits B0..B0+NS-1
// SM: the tower image's first subfield stage
template <int B0, int NS, int M, int SM>
__device__ __forceinline__ void ipassg(S16 &s, const uint8_t *tabs, uint32_t lb) {
  constexpr uint32_t KM = Geo<M>::K - 1;
  Tab T[2];
  SubTab U[2];
  const auto fetch = [&](int t, int blk, int slot) __attribute__((always_inline)) {
    const uint32_t a = lb ^ tlin(skew_idx((uint32_t(blk) << B0) & KM, B0 + t));
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
        if (B0 + t >= SM) ib(s, blk + i, blk + i + d, U[k & 1]);
        else ib(s, blk + i, blk + i + d, T[k & 1]);
      }
    }
  }
}

template <int B0, int NS, int M, int SM>
__device__ __forceinline__ void fpassg(S16 &s, const uint8_t *tabs, uint32_t lb) {
  constexpr uint32_t KM = Geo<M>::K - 1;
  Tab T[2];
  SubTab U[2];
  const auto fetch = [&](int t, int blk, int slot) __attribute__((always_inline)) {
    const uint32_t a = lb ^ tlin(skew_idx((uint32_t(blk) << B0) & KM, B0 + t));
    if (B0 + t >= SM) tab_at(tabs, a, U[slot]);
    else tab_at(tabs, a, T[slot]);
  };
  fetch(NS - 1, 0, 0);
  int k = 0;
#pragma unroll
  for (int t = NS - 1; t >= 0; --t) {
    const int d = 1 << t;
#pragma unroll
    for (int blk = 0; blk < 16; blk += 2 * d, ++k) {
      const int nt = blk + 2 * d < 16 ? t : t - 1, nblk = blk + 2 * d < 16 ? blk + 2 * d : 0;
      if (nt >= 0) fetch(nt, nblk, (k + 1) & 1);
#pragma unroll
      for (int i = 0; i < d; ++i) {
        if (B0 + t >= SM) fb(s, blk + i, blk + i + d, U[k & 1]);
        else fb(s, blk + i, blk + i + d, T[k & 1]);
      }
    }
  }
}

// k = 512: pass B's lane part is p8 (lane bit 4); p9 is an instance bit
__device__ __forceinline__ uint32_t lbB(uint32_t lane) {
  asm volatile("" : "+v"(lane));
  return tlin(((lane >> 4) & 1) << 8);
}

// k = 512, layout C: stage 8 (register bit 0); its skew index 255 (+ offset)
// is uniform since p9 is an instance bit
__device__ __forceinline__ void ipassC9(S16 &s, const uint8_t *tabs, uint32_t lo) {
  SubTab T;  // stage 8: subfield in every tower image
  tab_at(tabs, lo ^ tlin(skew_idx(0, 8)), T);
#pragma unroll
  for (int r = 0; r < 16; r += 2) ib(s, r, r + 1, T);
}

__device__ __forceinline__ void fpassC9(S16 &s, const uint8_t *tabs, uint32_t lo) {
  SubTab T;
  tab_at(tabs, lo ^ tlin(skew_idx(0, 8)), T);
#pragma unroll
  for (int r = 0; r < 16; r += 2) fb(s, r, r + 1, T);
}

// layout A rows of the wave -> own region: row local, instance i -> 8 B at
// row * ROWB + 8 i
template <int M>
__device__ __forceinline__ void stage(const S16 &s, uint8_t *my, uint32_t lane) {
  using Gm = Geo<M>;
  const uint32_t inst = (16 * lane) >> M, local0 = (16 * lane) & (Gm::K - 1);
#pragma unroll
  for (int r = 0; r < 16; ++r)
    *reinterpret_cast<uint2 *>(my + (local0 + r) * Gm::ROWB + 8 * inst) = to_be(s.l[r], s.h[r]);
}

// all waves: rows s0 + v, v < k, from the 8 regions -> shards
template <int M>
__device__ __forceinline__ void store_rows(const uint8_t *regions, uint8_t *SH, uint64_t sstride,
                                           uint32_t s0, int nv, uint64_t piece0, uint64_t npieces,
                                           uint32_t tid) {
  using Gm = Geo<M>;
  constexpr int CPW = Gm::ROWB / 16;      // 16-B chunks per row per wave
  constexpr int CPR = CPW * WAVES;        // chunks per row
  constexpr int ITER = Gm::K * CPR / THREADS;
  static_assert(Gm::K * CPR % THREADS == 0, "whole iterations");
  const bool wide = ((sstride | reinterpret_cast<uintptr_t>(SH)) & 15) == 0;  // 16-B aligned rows
#pragma unroll 4
  for (int it = 0; it < ITER; ++it) {
    const uint32_t ch = uint32_t(it) * THREADS + tid;
    const uint32_t v = ch / CPR, c16 = ch % CPR;
    const uint32_t w = c16 / CPW, o = (c16 % CPW) * 16;
    const uint4 val = *reinterpret_cast<const uint4 *>(regions + w * REG_BYTES + v * Gm::ROWB + o);
    const uint32_t shard = s0 + v;
    const uint64_t p = piece0 + 8 * c16;  // first of the chunk's 8 pieces
    if (int(shard) >= nv || p >= npieces) continue;
    uint8_t *dst = SH + uint64_t(shard) * sstride + 2 * p;
    if (p + 8 <= npieces) {
      if (wide) {
        *reinterpret_cast<uint4 *>(dst) = val;
      } else {
        reinterpret_cast<uint2 *>(dst)[0] = make_uint2(val.x, val.y);
        reinterpret_cast<uint2 *>(dst)[1] = make_uint2(val.z, val.w);
      }
    } else {
      const uint32_t wd[4] = {val.x, val.y, val.z, val.w};
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (p + e < npieces)
          *reinterpret_cast<uint16_t *>(dst + 2 * e) = uint16_t(wd[e >> 1] >> (16 * (e & 1)));
    }
  }
}

template <int M>
__global__ void __launch_bounds__(THREADS)
    encode_gen(const uint8_t *__restrict__ payloads, uint64_t plen, uint64_t pstride,
               uint8_t *__restrict__ shards, uint64_t slen, uint64_t sstride, int nv, int n,
               uint32_t batch, uint32_t *tick, DevTables t) {
  using Gm = Geo<M>;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  uint8_t *tabs = lds;
  uint8_t *regions = lds + Tabs::kBytes;
  const uint32_t tid0 = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid0 >> 6);
  uint8_t *my = regions + wave * REG_BYTES;

  int img = 0;  // table image in LDS (or requested): skews 1024 img .. + 1022
  // n = 2048 / 4096: the next coset's (or the next tile's index-0) image is
  // requested by LDS-DMA as soon as every wave is past the current coset's
  // FFT, so it lands behind that coset's row stores; `pending` until retired
  bool pending = false;
  const auto retire = [&]() __attribute__((always_inline)) {
    if (pending) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lds_barrier();
      pending = false;
    }
  };
  // tower images: the transforms run in tower coordinates
  // Tiles (round 5): a workgroup's first is blockIdx.x, every later one
  // gridDim.x + a ticket from *tick (zeroed by the launcher), taken by thread
  // 0 during a tile and published in the LDS word SLOT at its end (read after
  // the next tile's first barrier).  The static stride gave the workgroups
  // blockIdx = -1 mod tiles-per-payload every partial last tile (15.27 tiles
  // per payload at k = 512: ~5% of the launch idle).  tick == nullptr: static.
  volatile uint32_t *slot = reinterpret_cast<volatile uint32_t *>(lds + SLOT);
  uint32_t taken = 0;
  if (tick && tid0 == 0) taken = gridDim.x + atomicAdd(tick, 1u);
  Tabs::copy_image<THREADS>(tabs, t.timg_t, tid0);  // skews 0..1022: every coset of n <= 1024
  __syncthreads();
  if (tid0 == 0) *slot = taken;

  const uint64_t npieces = slen / 2;
  const uint32_t tiles_pp = uint32_t((npieces + Gm::TP - 1) / Gm::TP);
  const uint64_t total = uint64_t(tiles_pp) * batch;
  uint64_t nxt = 0;
  for (uint64_t tile = blockIdx.x; tile < total; tile = nxt) {
    uint32_t tid = tid0;
    asm volatile("" : "+v"(tid));
    const uint32_t lane = tid & 63;
    const uint64_t b = tile / tiles_pp;
    const uint64_t piece0 = (tile % tiles_pp) * Gm::TP;
    const uint8_t *P = payloads + b * pstride;
    uint8_t *SH = shards + b * uint64_t(nv) * sstride;

    // ---- load: lane -> positions 16 lane .. + 15 = instance i, locals l0 .. l0 + 15
    S16 s;
    {
      const uint32_t inst = (16 * lane) >> M, local0 = (16 * lane) & (Gm::K - 1);
      uint32_t D[4][8];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint64_t piece = piece0 + uint64_t(Gm::WP) * wave + 4 * inst + u;
        const uint64_t off = piece * 2 * Gm::K + 2 * local0;
        if (off + 32 <= plen) {
          const uint4 a = *reinterpret_cast<const uint4 *>(P + off);
          const uint4 c = *reinterpret_cast<const uint4 *>(P + off + 16);
          D[u][0] = a.x; D[u][1] = a.y; D[u][2] = a.z; D[u][3] = a.w;
          D[u][4] = c.x; D[u][5] = c.y; D[u][6] = c.z; D[u][7] = c.w;
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) D[u][j] = 0;
#pragma unroll
          for (int e = 0; e < 32; ++e)  // constant trip count: D stays in registers
            if (off + e < plen) D[u][e >> 2] |= uint32_t(P[off + e]) << (8 * (e & 3));
        }
      }
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

    // ---- systematic shards 0..k-1 = the data symbols (poly_encoder.hpp:239).
    // Barriers are lazy: a wave's region is next written by its first exchange
    // (or staging), so the barrier that waits for the other waves' reads of
    // the regions (store_rows) sits right before that write, and the stores
    // overlap the register-only first pass that precedes it.
    lds_barrier();  // the other waves are done reading the regions (last tile)
    nxt = tick ? uint64_t(__builtin_amdgcn_readfirstlane(*slot)) : tile + gridDim.x;
    if (tick && tid0 == 0) taken = gridDim.x + atomicAdd(tick, 1u);  // the tile after nxt
    stage<M>(s, my, lane);
    lds_barrier();
    store_rows<M>(regions, SH, sstride, 0, nv, piece0, npieces, tid);
    {  // into tower coordinates
      const TowerK tk = tower_k();
#pragma unroll
      for (int r = 0; r < 16; ++r) s.l[r] = tower_lo(s.l[r], s.h[r], tk);
    }

    // ---- IFFT_k (index 0): pass A, exchange, pass B -> layout B
    retire();  // the index-0 image requested by the previous tile's last coset
    const uint32_t lbA = tlin((16 * lane) & (Gm::K - 1));
    constexpr int S0 = tower_sub_min(0);
    ipassg<0, (M < 4 ? M : 4), M, S0>(s, tabs, lbA);
    if constexpr (M == 4) {
      // k = 16: the whole IFFT is pass A; coefficients stay in layout A
    } else if constexpr (M <= 8) {
      lds_barrier();  // systematic rows read out of the regions
      exchange<LA, LB>(s, my, lane);
      ipassg<4, M - 4, M, S0>(s, tabs, 0);
    } else {
      lds_barrier();  // systematic rows read out of the regions
      exchange<LA, LB>(s, my, lane);
      ipassg<4, 4, M, S0>(s, tabs, lbB(lane));
      exchange<LB, LC>(s, my, lane);
      ipassC9(s, tabs, 0);
    }
    const S16 coef = s;

    // ---- FFT_k at each coset shift (encodeLow, poly_encoder.hpp:229-237)
    // coset FFT with tower image img's first subfield stage SMv (integral_constant)
    const auto coset_fft = [&](auto smv, const uint32_t lo) __attribute__((always_inline)) {
      constexpr int SMc = decltype(smv)::value;
      if constexpr (M == 4) {
        lds_barrier();  // previous rows read out of the regions
      } else if constexpr (M <= 8) {
        fpassg<4, M - 4, M, SMc>(s, tabs, lo);
        lds_barrier();  // previous rows read out of the regions
        exchange<LB, LA>(s, my, lane);
      } else {
        fpassC9(s, tabs, lo);
        lds_barrier();  // previous rows read out of the regions
        exchange<LC, LB>(s, my, lane);
        fpassg<4, 4, M, SMc>(s, tabs, lbB(lane) ^ lo);
        exchange<LB, LA>(s, my, lane);
      }
      fpassg<0, (M < 4 ? M : 4), M, SMc>(s, tabs, tlin((16 * lane) & (Gm::K - 1)) ^ lo);
    };
    for (int sh = int(Gm::K); sh < n && sh < nv; sh += int(Gm::K)) {
      retire();  // this coset's image
      s = coef;
#pragma unroll
      for (int r = 0; r < 16; ++r) asm volatile("" : "+v"(s.l[r]), "+v"(s.h[r]));
      const uint32_t lo = tlin(uint32_t(sh) & 1023u);  // tables at offset sh (disjoint bits)
      if (img == 0) coset_fft(std::integral_constant<int, tower_sub_min(0)>(), lo);
      else if (img == 1) coset_fft(std::integral_constant<int, tower_sub_min(1)>(), lo);
      else coset_fft(std::integral_constant<int, tower_sub_min(2)>(), lo);  // images 2, 3
      {  // back to symbol coordinates
        const TowerK tk = tower_k();
#pragma unroll
        for (int r = 0; r < 16; ++r) s.l[r] = tower_lo(s.l[r], s.h[r], tk);
      }
      stage<M>(s, my, lane);  // own region: no other wave touches it since the barrier above
      lds_barrier();  // (every wave is past this coset's FFT: its tables are free)
      {
        const int nsh = sh + int(Gm::K);
        const int next = nsh < n && nsh < nv ? nsh >> 10 : 0;
        if (next != img) {
          Tabs::dma_image<THREADS>(tabs, t.timg_t + next * kTabImageBytes, tid);
          img = next;
          pending = true;
        }
      }
      store_rows<M>(regions, SH, sstride, uint32_t(sh), nv, piece0, npieces, tid);
    }
    // (every wave read SLOT before this tile's second barrier)
    if (tid0 == 0) *slot = taken;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA outlives the workgroup
}

template <int M>
hipError_t launch_m(const CodeParams &p, const DevTables &t, const uint8_t *d_payloads,
                    size_t plen, size_t pstride, size_t batch, uint8_t *d_shards, size_t sstride,
                    void *scratch, hipStream_t s) {
  int cus = 0;
  if (const hipError_t e = prepare_kernel(reinterpret_cast<const void *>(&encode_gen<M>), LDS_BYTES, &cus);
      e != hipSuccess)
    return e;
  const size_t sl = shard_len(p.k, plen);
  const size_t tiles = (sl / 2 + Geo<M>::TP - 1) / Geo<M>::TP * batch;
  const unsigned grid = unsigned(tiles < size_t(cus) ? tiles : size_t(cus));
  // dynamic tiles when the caller gave the counter's scratch (encgen_scratch_bytes)
  uint32_t *tick = tiles + 2 * size_t(cus) < (size_t(1) << 32) ? static_cast<uint32_t *>(scratch) : nullptr;
  if (tick)
    if (const hipError_t e = launch_zero_counters(tick, sizeof(uint32_t), s); e != hipSuccess) return e;
  hipLaunchKernelGGL(encode_gen<M>, dim3(grid), dim3(THREADS), LDS_BYTES, s, d_payloads,
                     uint64_t(plen), uint64_t(pstride), d_shards, uint64_t(sl), uint64_t(sstride),
                     int(p.nv), int(p.n), uint32_t(batch), tick, t);
  return hipGetLastError();
}

}  // namespace

bool encgen_applicable(const CodeParams &p) {
  return p.k >= 16 && p.k <= 512 && (p.k & (p.k - 1)) == 0 && p.n <= 4096 && p.n >= 2 * p.k;
}

size_t encgen_scratch_bytes(const CodeParams &p) { return encgen_applicable(p) ? 256 : 0; }

hipError_t launch_encode_gen(const CodeParams &p, const DevTables &t, const uint8_t *d_payloads,
                             size_t plen, size_t pstride, size_t batch, uint8_t *d_shards,
                             size_t sstride, void *scratch, hipStream_t s) {
  switch (p.k) {
    case 16: return launch_m<4>(p, t, d_payloads, plen, pstride, batch, d_shards, sstride, scratch, s);
    case 32: return launch_m<5>(p, t, d_payloads, plen, pstride, batch, d_shards, sstride, scratch, s);
    case 64: return launch_m<6>(p, t, d_payloads, plen, pstride, batch, d_shards, sstride, scratch, s);
    case 128: return launch_m<7>(p, t, d_payloads, plen, pstride, batch, d_shards, sstride, scratch, s);
    case 256: return launch_m<8>(p, t, d_payloads, plen, pstride, batch, d_shards, sstride, scratch, s);
    default: return launch_m<9>(p, t, d_payloads, plen, pstride, batch, d_shards, sstride, scratch, s);
  }
}

}  // namespace ecamd
