// ec_device.hpp — CDNA4 device arithmetic for the NPB codec.
//
// Byte-planar symbols: one uint2 {l, h} holds 4 GF(2^16) symbols (4 pieces or
// 4 shard positions); l has their low bytes, h their high bytes.  A multiply
// by a log-domain constant c is a GF(2)-linear map, so
//     x * c = XOR_g T_g[group_g(x)]
// over 3-bit (and 2-bit) bit groups of x.  Each T_g lookup of 4 symbols at
// once is one v_perm_b32 (8-entry byte table held in two registers, selector
// bytes = the 4 group values), i.e. 12 v_perm + 6 selector masks + 6 v_bitop3
// per 4 multiply-accumulates.  No LOG/EXP gathers.  v_perm issues at half the
// rate of v_and/v_bitop3 on gfx950 (scripts/micro/oprate.hip), so the perms are
// ~60% of a multiply's issue slots and set the arithmetic ceiling.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "gf_field.hpp"

namespace ecamd {

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

__device__ __forceinline__ uint32_t vperm(uint32_t hi, uint32_t lo, uint32_t sel) {
  return __builtin_amdgcn_perm(hi, lo, sel);
}

// Workgroup barrier that orders LDS only: waits for this wave's LDS operations
// (lgkmcnt) but NOT for outstanding global stores/loads, unlike __syncthreads()
// whose fence drains vmcnt and would serialize the HBM write stream with the
// next tile's compute.  The asm "memory" clobbers stop compiler reordering of
// LDS accesses across the barrier.
// bytes [0, avail) (avail < 64) of a 4-B aligned row slice into w[16], zero
// beyond: dword loads for whole dwords, bytes for the last partial one (nothing
// past the row's end is read).  Constant indices only, so w stays in registers
// and at most 16 loads are in flight.
__device__ __forceinline__ void load_row_tail64(const uint8_t *row, uint64_t avail, uint32_t (&w)[16]) {
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    w[j] = 0;
    if (uint64_t(4 * j + 4) <= avail) {
      w[j] = reinterpret_cast<const uint32_t *>(row)[j];
    } else if (uint64_t(4 * j) < avail) {
      for (uint32_t e = 0; 4 * j + e < avail; ++e) w[j] |= uint32_t(row[4 * j + e]) << (8 * e);
    }
  }
}

// 32-bit LDS address of an LDS pointer, and 8-byte accesses at such an
// address.  For GF(2)-linear swizzles: an access at (per-lane part) XOR
// (compile-time part) is then one v_xor (the compiler does not see the
// linearity through pointer arithmetic and emits ~4 VALU per access).
typedef __attribute__((address_space(3))) uint8_t lds_u8;
__device__ __forceinline__ uint32_t lds_addr(const uint8_t *p) {
  return uint32_t(uintptr_t((const lds_u8 *)p));
}
__device__ __forceinline__ uint2 lds_ld2(uint32_t a) {
  const uint64_t v = *(const __attribute__((address_space(3))) uint64_t *)(uintptr_t(a));
  return make_uint2(uint32_t(v), uint32_t(v >> 32));
}
__device__ __forceinline__ void lds_st2(uint32_t a, uint2 v) {
  *(__attribute__((address_space(3))) uint64_t *)(uintptr_t(a)) = (uint64_t(v.y) << 32) | v.x;
}

// One LDS-DMA wave-instruction: 16 B per lane from `src` (per lane) to the
// wave's 1 KB of LDS at `dst` (wave-uniform: M0) + 16 lane.  Inline asm
// instead of __builtin_amdgcn_global_load_lds: the compiler treats a pending
// LDS-DMA as a write to every LDS address and waits for it with vmcnt(0)
// before the next LDS access it cannot prove disjoint, which also waits for
// every shard store issued after the DMA (enc_k1024: before each coset's first
// table read, right after the previous coset's row stores).  Hidden from the
// compiler, the DMA is retired only by the kernels' own s_waitcnt vmcnt(N)
// before the barrier that precedes the first read of its bytes; the
// compiler's own vmcnt waits stay correct (the counter retires in issue
// order, so an op it does not know of only makes its waits stricter).
__device__ __forceinline__ void lds_dma16(uint32_t dst, const void *src) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off"
               :
               : "s"(__builtin_amdgcn_readfirstlane(dst)), "v"(src)
               : "memory");  // (M0 is reserved: the compiler sets it before each of its own uses)
}

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// (payload, tile in payload) of a grid-stride tile walk, tile = b * per + i,
// advanced by `step` tiles with an add and a compare instead of a 64-bit
// division per tile (wave-uniform: SGPRs)
struct TileWalk {
  uint64_t b = 0, i = 0, qs = 0, rs = 0, per = 1;
  __device__ TileWalk(uint64_t first, uint64_t step, uint64_t per_) : per(per_ ? per_ : 1) {
    b = first / per;
    i = first % per;
    qs = step / per;
    rs = step % per;
  }
  __device__ __forceinline__ void next_of(uint64_t &nb, uint64_t &ni) const {
    ni = i + rs;
    nb = b + qs;
    if (ni >= per) {
      ni -= per;
      ++nb;
    }
  }
  __device__ __forceinline__ void advance() { next_of(b, i); }
};

// XCD-affine split of a persistent grid's tiles (blocks b and b + 8 share an
// XCD and its L2; the placement is a speed hint only, any placement is
// correct): tiles [0, total) are cut into 8 contiguous spans, span b % 8 walked
// grid-stride by that group's blocks, so a payload's tiles, and its per-payload
// tables, masks and gather lists, stay in one L2.  Grids not a multiple of 8
// (small batches) walk the whole range.
struct TileSpan {
  uint64_t first, step, end;
};
__device__ __forceinline__ TileSpan xcd_span(uint64_t total) {
  const uint32_t g = gridDim.x;
  if (g % 8 != 0 || total < 8ull * g) return {blockIdx.x, g, total};
  const uint64_t chunk = (total + 7) / 8, lo = (blockIdx.x % 8) * chunk;
  return {lo + blockIdx.x / 8, g / 8, lo + chunk < total ? lo + chunk : total};
}

// Dynamic, XCD-affine tile schedule of a persistent grid: the tiles [0, total)
// are cut into 8 contiguous spans as xcd_span does, span b % 8 served to its
// group's workgroups from its own counter (zeroed before the launch, 64 B
// apart), so a payload's tiles stay in one L2 and the workgroups of a group
// finish together whatever their issue rates.  Grids not a multiple of 8 or
// small batches: one counter over the whole range.  take() is one atomic; a
// value >= hi means the span is done.
constexpr size_t kTileQueueBytes = 8 * 64;
struct TileQueue {
  uint32_t lo, hi;
  uint32_t *ctr;
  __device__ TileQueue(uint32_t total, uint32_t *ctrs) {
    const uint32_t g = gridDim.x;
    if (g % 8 != 0 || total < 8u * g) {
      lo = 0;
      hi = total;
      ctr = ctrs;
    } else {
      const uint32_t chunk = (total + 7) / 8, x = blockIdx.x % 8;
      lo = x * chunk;
      hi = lo + chunk < total ? lo + chunk : total;
      ctr = ctrs + 16 * x;
    }
  }
  __device__ __forceinline__ uint32_t take() const { return lo + atomicAdd(ctr, 1u); }
};

struct Tab {
  uint32_t t[20];
};

// One 80-byte multiply table from LDS at absolute LDS address `a` (plane 0;
// planes `plane` bytes apart), planes loaded last-used first so the first
// multiply waits once.  The big-LDS kernels have no static LDS (checked by
// prepare_kernel), so their dynamic LDS starts at address 0 and a table
// address is a per-lane base XOR a compile-time value: no add of the LDS base
// per table (the base is a link-time symbol the compiler cannot fold).
template <int PLANE>
__device__ __forceinline__ void lds_tab_abs(uint32_t a, Tab &T) {
#pragma unroll
  for (int q = 4; q >= 0; --q) {
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const v4u v = *(const __attribute__((address_space(3))) v4u *)(uintptr_t(a + q * PLANE));
    T.t[4 * q] = v.x;
    T.t[4 * q + 1] = v.y;
    T.t[4 * q + 2] = v.z;
    T.t[4 * q + 3] = v.w;
  }
}

__device__ __forceinline__ void load_tab(const MulTab *__restrict__ mt, uint32_t c, Tab &T) {
  const uint4 *p = reinterpret_cast<const uint4 *>(mt + c);
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    const uint4 v = p[q];
    T.t[4 * q + 0] = v.x;
    T.t[4 * q + 1] = v.y;
    T.t[4 * q + 2] = v.z;
    T.t[4 * q + 3] = v.w;
  }
}

// {hi:lo} >> S as one v_lshrrev_b64: both byte planes' selector groups from one
// (full-rate) instruction; the compiler narrows a C++ 64-bit shift back into
// two 32-bit shifts, hence the asm (non-volatile: still scheduled and CSE'd).
template <int S>
__device__ __forceinline__ uint64_t shr64(uint64_t x) {
  uint64_t r;
  asm("v_lshrrev_b64 %0, %1, %2" : "=v"(r) : "i"(S), "v"(x));
  return r;
}

// (yl, yh) ^= (xl, xh) * c, four symbols at once: 12 v_perm (half rate on
// gfx950), 6 v_and, 2 v_lshrrev_b64, 6 v_bitop3 = 38 issue slots.
__device__ __forceinline__ void mul_acc(uint32_t xl, uint32_t xh, const Tab &T, uint32_t &yl,
                                        uint32_t &yh) {
  const uint64_t x = (uint64_t(xh) << 32) | xl;
  const uint64_t t3 = shr64<3>(x), t6 = shr64<6>(x);
  const uint32_t s0 = xl & 0x07070707u;
  const uint32_t s1 = uint32_t(t3) & 0x07070707u;
  const uint32_t s2 = uint32_t(t6) & 0x03030303u;
  const uint32_t s3 = xh & 0x07070707u;
  const uint32_t s4 = uint32_t(t3 >> 32) & 0x07070707u;
  const uint32_t s5 = uint32_t(t6 >> 32) & 0x03030303u;
  uint32_t l = xor3(yl, vperm(T.t[1], T.t[0], s0), vperm(T.t[5], T.t[4], s1));
  l = xor3(l, vperm(T.t[9], T.t[8], s3), vperm(T.t[13], T.t[12], s4));
  l = xor3(l, vperm(T.t[16], T.t[16], s2), vperm(T.t[18], T.t[18], s5));
  uint32_t h = xor3(yh, vperm(T.t[3], T.t[2], s0), vperm(T.t[7], T.t[6], s1));
  h = xor3(h, vperm(T.t[11], T.t[10], s3), vperm(T.t[15], T.t[14], s4));
  h = xor3(h, vperm(T.t[17], T.t[17], s2), vperm(T.t[19], T.t[19], s5));
  yl = l;
  yh = h;
}

// ---- subfield multiplies in tower coordinates -------------
// Symbols < 256 are the subfield GF(2^8).  In tower coordinates
// (gf_field.hpp: x -> x ^ L(x >> 8), an involution) a multiply by a subfield
// constant c acts on each byte alone, as GF(2^8) multiplication by c, so one
// 8-bit table (3 + 3 + 2 bit groups: 5 dwords) serves both byte planes:
// 6 v_perm + 6 v_and + 2 v_lshrrev_b64 + 4 XOR = 24 issue slots per 4
// multiply-accumulates (mul_acc: 38).  SubTab words: t[0..1] group [0:3),
// t[2..3] group [3:6), t[4] group [6:8) (MulTabSub, gf_field.hpp).
struct SubTab {
  uint32_t t[5];
};

__device__ __forceinline__ void mul_acc_sub(uint32_t xl, uint32_t xh, const SubTab &T, uint32_t &yl,
                                            uint32_t &yh) {
  const uint64_t x = (uint64_t(xh) << 32) | xl;
  const uint64_t t3 = shr64<3>(x), t6 = shr64<6>(x);
  const uint32_t s0 = xl & 0x07070707u;
  const uint32_t s1 = uint32_t(t3) & 0x07070707u;
  const uint32_t s2 = uint32_t(t6) & 0x03030303u;
  const uint32_t s3 = xh & 0x07070707u;
  const uint32_t s4 = uint32_t(t3 >> 32) & 0x07070707u;
  const uint32_t s5 = uint32_t(t6 >> 32) & 0x03030303u;
  yl = xor3(yl, vperm(T.t[1], T.t[0], s0), vperm(T.t[3], T.t[2], s1)) ^ vperm(T.t[4], T.t[4], s2);
  yh = xor3(yh, vperm(T.t[1], T.t[0], s3), vperm(T.t[3], T.t[2], s4)) ^ vperm(T.t[4], T.t[4], s5);
}

// ---- F9 multiplies: a constant c0 + c1 w with c1 in {0, 1}
// (tower coordinates, w^2 = alpha w + beta) as three subfield tables and a mask:
//   low  ^= c0 x0 ^ (c1 beta) x1,   high ^= (c0 + c1 alpha) x1 ^ (x0 & m)
// 9 v_perm + 6 v_and + 2 v_lshrrev_b64 + 5 XOR + 1 v_and = 32 issue slots per
// 4 multiply-accumulates (mul_acc: 38).  F9Tab = MulTabF9 (gf_field.hpp).
struct F9Tab {
  uint32_t t[16];
};

__device__ __forceinline__ void mul_acc_f9(uint32_t xl, uint32_t xh, const F9Tab &T, uint32_t &yl,
                                           uint32_t &yh) {
  const uint64_t x = (uint64_t(xh) << 32) | xl;
  const uint64_t t3 = shr64<3>(x), t6 = shr64<6>(x);
  const uint32_t s0 = xl & 0x07070707u;
  const uint32_t s1 = uint32_t(t3) & 0x07070707u;
  const uint32_t s2 = uint32_t(t6) & 0x03030303u;
  const uint32_t s3 = xh & 0x07070707u;
  const uint32_t s4 = uint32_t(t3 >> 32) & 0x07070707u;
  const uint32_t s5 = uint32_t(t6 >> 32) & 0x03030303u;
  uint32_t l = xor3(yl, vperm(T.t[1], T.t[0], s0), vperm(T.t[3], T.t[2], s1));
  l = xor3(l, vperm(T.t[4], T.t[4], s2), vperm(T.t[6], T.t[5], s3));
  yl = xor3(l, vperm(T.t[8], T.t[7], s4), vperm(T.t[9], T.t[9], s5));
  const uint32_t h = xor3(yh, vperm(T.t[11], T.t[10], s3), vperm(T.t[13], T.t[12], s4));
  yh = xor3(h, vperm(T.t[14], T.t[14], s5), xl & T.t[15]);
}

// An F9 table in an F9 image slot at absolute LDS address `a` (plane 0;
// planes PLANE bytes apart): planes 0..3
template <int PLANE>
__device__ __forceinline__ void lds_f9tab_abs(uint32_t a, F9Tab &T) {
#pragma unroll
  for (int q = 3; q >= 0; --q) {
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const v4u v = *(const __attribute__((address_space(3))) v4u *)(uintptr_t(a + q * PLANE));
    T.t[4 * q] = v.x;
    T.t[4 * q + 1] = v.y;
    T.t[4 * q + 2] = v.z;
    T.t[4 * q + 3] = v.w;
  }
}

// symbol <-> tower coordinates of a byte-planar group (the map is its own
// inverse): l ^= L(h) bytewise, L = kTowerL, as compile-time v_perm tables
__host__ __device__ constexpr uint8_t tower_l8(uint32_t h) {
  uint8_t r = 0;
  for (int i = 0; i < 8; ++i)
    if ((h >> i) & 1) r ^= kTowerL[i];
  return r;
}
__host__ __device__ constexpr uint32_t tower_word(uint32_t pos, uint32_t first) {
  uint32_t w = 0;
  for (uint32_t e = 0; e < 4; ++e) w |= uint32_t(tower_l8((first + e) << pos)) << (8 * e);
  return w;
}
struct TowerK {  // the five table words in VGPRs
  uint32_t w[5];
};
// materialised where the conversion runs (opaque: not hoisted out of a loop
// and kept live across it)
__device__ __forceinline__ TowerK tower_k() {
  TowerK k = {{tower_word(0, 0), tower_word(0, 4), tower_word(3, 0), tower_word(3, 4), tower_word(6, 0)}};
#pragma unroll
  for (int i = 0; i < 5; ++i) asm volatile("" : "+v"(k.w[i]));
  return k;
}
__device__ __forceinline__ uint32_t tower_lo(uint32_t l, uint32_t h, const TowerK &k) {
  const uint32_t s0 = h & 0x07070707u, s1 = (h >> 3) & 0x07070707u, s2 = (h >> 6) & 0x03030303u;
  return xor3(l, vperm(k.w[1], k.w[0], s0), vperm(k.w[3], k.w[2], s1)) ^ vperm(k.w[4], k.w[4], s2);
}

// A subfield table in a tower LDS image (same slots as the general tables:
// plane 0 holds t[0..3], the first dword of plane 1 holds t[4]) at absolute
// LDS address `a` (plane 0).
template <int PLANE>
__device__ __forceinline__ void lds_subtab_abs(uint32_t a, SubTab &T) {
  T.t[4] = *(const __attribute__((address_space(3))) uint32_t *)(uintptr_t(a + PLANE));
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  const v4u v = *(const __attribute__((address_space(3))) v4u *)(uintptr_t(a));
  T.t[0] = v.x;
  T.t[1] = v.y;
  T.t[2] = v.z;
  T.t[3] = v.w;
}

// LDS-resident multiply tables: plane-major (5 planes of 16-byte chunks), the
// 16-byte slot of entry idx XOR-swizzled by f(idx) = (idx ^ idx>>4 ^ idx>>8) & 15.
// f is injective on every set of entries one ds_read_b128 lane group touches in
// the kernels (index strides 1..16 over the group's lanes, or 64 / 256 over <=4
// distinct entries), so per-lane table loads are bank-conflict free.
template <int ENTRIES>
struct LdsTabs {
  static constexpr int kPlane = ENTRIES * 16;
  static constexpr int kBytes = 5 * kPlane;
  __device__ static __forceinline__ uint32_t addr(uint32_t idx, uint32_t plane) {
    const uint32_t f = (idx ^ (idx >> 4) ^ (idx >> 8)) & 15;
    return plane * kPlane + ((idx >> 4) << 8) + (f << 4);
  }
  __device__ static __forceinline__ void load(const uint8_t *base, uint32_t idx, Tab &T) {
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      const uint4 v = *reinterpret_cast<const uint4 *>(base + addr(idx, q));
      T.t[4 * q] = v.x;
      T.t[4 * q + 1] = v.y;
      T.t[4 * q + 2] = v.z;
      T.t[4 * q + 3] = v.w;
    }
  }
  // cooperative copy of a prebuilt image (DevTables::timg) of ENTRIES entries:
  // every load issued before the first store
  template <int THREADS>
  __device__ static __forceinline__ void copy_image(uint8_t *base, const uint8_t *img,
                                                    uint32_t tid) {
    constexpr int kChunks = kBytes / 16;
    static_assert(kChunks % THREADS == 0, "whole chunks per thread");
    uint32_t v[kChunks / THREADS][4];  // scalars, not uint4: an aggregate copy would stay in scratch
#pragma unroll
    for (int k = 0; k < kChunks / THREADS; ++k) {
      const uint4 x = reinterpret_cast<const uint4 *>(img)[tid + k * THREADS];
      v[k][0] = x.x;
      v[k][1] = x.y;
      v[k][2] = x.z;
      v[k][3] = x.w;
    }
#pragma unroll
    for (int k = 0; k < kChunks / THREADS; ++k)
      reinterpret_cast<uint4 *>(base)[tid + k * THREADS] = make_uint4(v[k][0], v[k][1], v[k][2], v[k][3]);
  }
  // the same copy by LDS-DMA (global_load_lds_dwordx4): no VGPRs, completes in
  // the background; the caller retires it (s_waitcnt vmcnt) before the
  // barrier that precedes the first table read.  A wave-instruction writes 1 KB
  // of LDS linearly, which is exactly the image layout.  Issued by lds_dma16
  // (inline asm), so the compiler's wait model does not see it: see there.
  // HIDDEN = false: the compiler's builtin (and its conservative waits)
  template <int THREADS, bool HIDDEN = true>
  __device__ static __forceinline__ void dma_image(uint8_t *base, const uint8_t *img,
                                                   uint32_t tid) {
    constexpr int kChunks = kBytes / 16;
    static_assert(kChunks % THREADS == 0 && THREADS % 64 == 0, "whole chunks per thread");
    // wave-uniform source / destination (SGPRs) + one per-lane byte offset:
    // no per-chunk address registers for the compiler to keep live between calls
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t loff = (tid & 63) * 16;
#pragma unroll
    for (int k = 0; k < kChunks / THREADS; ++k) {
      const uint32_t off = (uint32_t(k) * THREADS + wave * 64) * 16;  // this wave's 1 KB slice
      if constexpr (HIDDEN)
        lds_dma16(lds_addr(base) + off, img + off + loff);
      else
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(img + off + loff),
                                         (__attribute__((address_space(3))) void *)(base + off), 16, 0, 0);
    }
  }
  // cooperative gather of ENTRIES tables, entry i <- mtab[src(i)], all index
  // loads then all table loads in flight at once
  template <int THREADS, typename F>
  __device__ static __forceinline__ void gather(uint8_t *base, const MulTab *mtab, F src,
                                                uint32_t tid) {
    constexpr int kChunks = ENTRIES * 5;
    constexpr int kPer = (kChunks + THREADS - 1) / THREADS;
    constexpr bool kExact = kChunks % THREADS == 0;  // no bounds test (keeps v[] in registers)
    uint32_t c[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const uint32_t i = tid + k * THREADS;
      c[k] = (kExact || i < uint32_t(kChunks)) ? src(i / 5) : 0u;
    }
    uint4 v[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const uint32_t i = tid + k * THREADS;
      v[k] = make_uint4(0, 0, 0, 0);
      if (kExact || i < uint32_t(kChunks)) v[k] = reinterpret_cast<const uint4 *>(mtab + c[k])[i % 5];
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const uint32_t i = tid + k * THREADS;
      if (kExact || i < uint32_t(kChunks)) *reinterpret_cast<uint4 *>(base + addr(i / 5, i % 5)) = v[k];
    }
  }
  // gather() restricted to the entries with keep(i) (cheap: no memory reads)
  // and need(i) (may read memory: evaluated beside src(i), so it adds no
  // dependent latency); the others are neither loaded nor written (their LDS
  // bytes stay stale and must not be read)
  template <int THREADS, typename F, typename K, typename N>
  __device__ static __forceinline__ void gather_if(uint8_t *base, const MulTab *mtab, F src, K keep,
                                                   N need, uint32_t tid) {
    constexpr int kChunks = ENTRIES * 5;
    constexpr int kPer = (kChunks + THREADS - 1) / THREADS;
    constexpr bool kExact = kChunks % THREADS == 0;
    uint32_t c[kPer];
    bool on[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const uint32_t i = tid + k * THREADS;
      on[k] = (kExact || i < uint32_t(kChunks)) && keep(i / 5);
      c[k] = on[k] ? src(i / 5) : 0u;
      on[k] = on[k] && need(i / 5);
    }
    uint4 v[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const uint32_t i = tid + k * THREADS;
      v[k] = make_uint4(0, 0, 0, 0);
      if (on[k]) v[k] = reinterpret_cast<const uint4 *>(mtab + c[k])[i % 5];
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const uint32_t i = tid + k * THREADS;
      if (on[k]) *reinterpret_cast<uint4 *>(base + addr(i / 5, i % 5)) = v[k];
    }
  }
  // cooperative fill: entry i <- mtab[src(i)]
  template <typename F>
  __device__ static __forceinline__ void fill(uint8_t *base, const MulTab *mtab, int count,
                                              F src, uint32_t tid, uint32_t nthreads) {
    for (uint32_t i = tid; i < uint32_t(count) * 5; i += nthreads) {
      const uint32_t e = i / 5, q = i % 5;
      *reinterpret_cast<uint4 *>(base + addr(e, q)) =
          reinterpret_cast<const uint4 *>(mtab + src(e))[q];
    }
  }
};

}  // namespace ecamd
