// enc_k1024.hip — encode specialised for k = 1024, n = 4096 (n_validators
// 3070..4096; BASELINE config 4).
//
// encodeLow (poly_encoder.hpp:217-240) for k = 1024 is one IFFT_1024 and up to
// three FFT_1024 at coset shifts 1024 / 2048 / 3072, each with its own 1023
// skews (80 KB of multiply tables).  All 4095 tables do not fit LDS next to the
// exchange regions, so the encode runs as one launch per transform, each with
// its transform's tables resident for the whole (persistent) launch:
//   launch 0: payload -> systematic shards 0..1023, IFFT -> coefficients,
//             written to a device scratch in the kernel's register order;
//   launch s (s = 1024, 2048, 3072 < nv): coefficients -> FFT -> shards
//             [s, s + 1024).
// The scratch round trip adds 4 x payload bytes of HBM traffic to a VALU-bound
// kernel.
//
// Tile = 64 consecutive pieces (piece = 2048 payload bytes = 1024 symbols);
// wave w owns pieces [8w, 8w + 8) as two byte-planar groups of 4, each run
// through tf1024.hpp's register passes.  Shard rows (128 B per row per tile)
// are staged in two halves of 512 rows through the waves' own regions and
// stored as 16 B per lane, 128-B row segments.
#include <hip/hip_runtime.h>

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
constexpr size_t SCRATCH_PER_TILE = size_t(WAVES) * 2 * 16 * 64 * sizeof(uint2);

// own-region staging slot of row v (0..511) of wave w: the 8 lanes reading one
// row from the 8 regions hit 8 distinct 16-B slots
__device__ __forceinline__ uint32_t soff(uint32_t v, uint32_t w) {
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

__device__ __forceinline__ uint2 *coef_at(uint2 *scratch, uint64_t tile, uint32_t wave, int g) {
  return scratch + ((tile * WAVES + wave) * 2 + uint64_t(g)) * (16 * 64);
}

// MODE 0: IFFT launch (shift 0); MODE 1: FFT launch at coset `shift`
template <int MODE>
__global__ void __launch_bounds__(THREADS)
    encode_k1024(const uint8_t *__restrict__ payloads, uint64_t plen, uint64_t pstride,
                 uint8_t *__restrict__ shards, uint64_t slen, uint64_t sstride, int nv,
                 uint32_t batch, uint32_t shift, uint2 *__restrict__ coef, DevTables t) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  uint8_t *tabs = lds;
  uint8_t *regions = lds + Tabs::kBytes;
  const uint32_t tid0 = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid0 >> 6);
  uint8_t *my = regions + wave * REG_BYTES;

  // this transform's 1023 skews (additive_fft.hpp:108,126: skews[j - 1 + index])
  Tabs::copy_image<THREADS>(tabs, t.timg + (shift / K) * kTabImageBytes, tid0);
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
    S16 g0, g1;
    if constexpr (MODE == 0) {
      const uint8_t *P = payloads + b * pstride;
      load_group(g0, P, plen, piece0 + 8 * wave, lane);
      load_group(g1, P, plen, piece0 + 8 * wave + 4, lane);
      // systematic shards 0..1023 = the data symbols (poly_encoder.hpp:239)
#pragma unroll
      for (uint32_t hf = 0; hf < 2; ++hf) {
        lds_barrier();  // the other waves are done reading the regions
        stage_half(g0, g1, my, lane, wave, hf);
        lds_barrier();
        store_half(regions, SH, sstride, 512 * hf, nv, piece0, npieces, wave, lane);
      }
      lds_barrier();
      ifft1024<true>(g0, tabs, my, lane);  // index 0 (zero skews at the top stages)
      ifft1024<true>(g1, tabs, my, lane);
      uint2 *c0 = coef_at(coef, tile, wave, 0), *c1 = coef_at(coef, tile, wave, 1);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        c0[r * 64 + lane] = make_uint2(g0.l[r], g0.h[r]);
        c1[r * 64 + lane] = make_uint2(g1.l[r], g1.h[r]);
      }
    } else {
      const uint2 *c0 = coef_at(coef, tile, wave, 0), *c1 = coef_at(coef, tile, wave, 1);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const uint2 a = c0[r * 64 + lane], bb = c1[r * 64 + lane];
        g0.l[r] = a.x;
        g0.h[r] = a.y;
        g1.l[r] = bb.x;
        g1.h[r] = bb.y;
      }
      lds_barrier();  // the other waves are done reading this region (last tile)
      fft1024(g0, tabs, my, lane);
      fft1024(g1, tabs, my, lane);
#pragma unroll
      for (uint32_t hf = 0; hf < 2; ++hf) {
        if (hf) lds_barrier();
        stage_half(g0, g1, my, lane, wave, hf);
        lds_barrier();
        store_half(regions, SH, sstride, shift + 512 * hf, nv, piece0, npieces, wave, lane);
      }
    }
  }
}

}  // namespace

bool k1024_applicable(const CodeParams &p) { return p.k == 1024 && p.n == 4096; }

size_t k1024_scratch_bytes(size_t plen, size_t batch) {
  const size_t pieces = shard_len(K, plen) / 2;
  return (pieces + TILE - 1) / TILE * batch * SCRATCH_PER_TILE;
}

hipError_t launch_encode_k1024(const CodeParams &p, const DevTables &t, const uint8_t *d_payloads,
                               size_t plen, size_t pstride, size_t batch, uint8_t *d_shards,
                               size_t sstride, void *scratch, hipStream_t s) {
  int cus = 0;
  for (const void *f : {reinterpret_cast<const void *>(&encode_k1024<0>),
                        reinterpret_cast<const void *>(&encode_k1024<1>)})
    if (const hipError_t e = prepare_kernel(f, LDS_BYTES, &cus); e != hipSuccess) return e;
  if (!scratch) return hipErrorInvalidValue;
  const size_t sl = shard_len(p.k, plen);
  const size_t tiles = (sl / 2 + TILE - 1) / TILE * batch;
  const unsigned grid = unsigned(tiles < size_t(cus) ? tiles : size_t(cus));
  uint2 *coef = static_cast<uint2 *>(scratch);
  hipLaunchKernelGGL(encode_k1024<0>, dim3(grid), dim3(THREADS), LDS_BYTES, s, d_payloads,
                     uint64_t(plen), uint64_t(pstride), d_shards, uint64_t(sl), uint64_t(sstride),
                     int(p.nv), uint32_t(batch), 0u, coef, t);
  for (uint32_t sh = K; sh < p.n && sh < p.nv; sh += K)
    hipLaunchKernelGGL(encode_k1024<1>, dim3(grid), dim3(THREADS), LDS_BYTES, s, d_payloads,
                       uint64_t(plen), uint64_t(pstride), d_shards, uint64_t(sl), uint64_t(sstride),
                       int(p.nv), uint32_t(batch), sh, coef, t);
  return hipGetLastError();
}

}  // namespace ecamd
