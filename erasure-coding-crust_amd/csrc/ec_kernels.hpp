// ec_kernels.hpp — launch interface of the HIP kernels (internal, C++).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "gf_field.hpp"

namespace ecamd {

// LDS images of the multiply tables of one 1023-skew set, in the swizzled
// LdsTabs<1024> layout: set q = skews[1024 q + i], i < 1023 (q = 0..3), i.e.
// the tables of an FFT / IFFT of size <= 1024 at index 1024 q.  A kernel loads
// a set with one coalesced 80 KB copy instead of a 1023-entry gather.
constexpr size_t kTabImageBytes = 5 * 1024 * 16;
constexpr int kTabImages = 4;

// Tower images: the same slots in tower coordinates.  Entry
// i of set q is a subfield table (MulTabSub: plane 0 = w[0..3], dword 0 of
// plane 1 = w[4]) when its stage ctz(1024 q + i + 1) >= tower_sub_min(q) --
// every such skew is < 256 -- and a general tower table (Field::tower_tab)
// below; a kernel reading set q uses mul_acc_sub at exactly those stages.
constexpr int tower_sub_min(int q) { return q == 0 ? 2 : q == 1 ? 3 : 4; }

// F9 variants of tower image 0: entry i holds a MulTabF9
// (plane q = w[4q .. 4q + 3]) where f9_slot(kind, i), the tower image's table
// elsewhere.  Kind 0 (reconstruct_n1024): the stage-1 entries (i = 1 mod 4,
// elements 0..510); kind 1 (encode_k256): also the stage-0 entries
// 256..510 (elements 256..510, its coset-256 FFT).  Their elements' high
// tower coordinate is 0 or 1 (tests/cpp/tower_check.cpp).
constexpr int kF9Images = 2;
constexpr bool f9_slot(int kind, uint32_t i) {
  return i % 4 == 1 || (kind == 1 && i % 2 == 0 && i >= 256 && i < 512);
}

// Element-indexed compact image (the n = 1024 encode).  The
// skew of a stage-m butterfly at position pos of an FFT / IFFT at index `off`
// (additive_fft.hpp:99-141) is the element 2 x, x = (pos + off) >> (m + 1)
// (skews[i] = log(((i + 1) >> ctz(i + 1)) - 1); checked against the oracle),
// so a table set can be indexed by x instead of by skew slot.  For the
// k = 256 / n = 1024 encode x < 512, and the element's tower coordinates put
// it in one of three kinds: x < 128 subfield (MulTabSub), 128 <= x < 256 F9
// (MulTabF9), 256 <= x < 512 general (Field::tower_tab).  Plane q of entry x
// sits at base(kind, q) | cimg_lin(x ^ kind_bit), cimg_lin GF(2)-linear (the
// LdsTabs swizzle applied to x), so every table address is a per-lane base XOR
// a wave-uniform value; 32 KB instead of the 80 KB skew-slot image.
constexpr uint32_t kCImgGen = 0, kCImgGenPlane = 4096;      // 5 planes x 256 entries
constexpr uint32_t kCImgF9 = 20480, kCImgF9Plane = 2048;    // 4 planes x 128 entries
constexpr uint32_t kCImgSub0 = 28672, kCImgSub1 = 30720;    // plane 0 / dword 0 of plane 1, 128 entries
constexpr uint32_t kCImgBytes = 32768;
__host__ __device__ constexpr uint32_t cimg_lin(uint32_t x) {
  return ((x >> 4) << 8) | (((x ^ (x >> 4) ^ (x >> 8)) & 15) << 4);
}

// Per-coset extension images of the k = 512 encode (enc_k512w.hip; n = 2048 /
// 4096): the general tables its FFT_512 at coset j (index 512 j, j = 1..7)
// needs beyond the compact image's subfield and F9 entries, element-indexed
// like it: stage m (0, 1, 2) entry e = x - (512 j >> (m + 1)), e < 256 >> m,
// plane q at kEImg512Stage[m] + q * (4096 >> m) + cimg_lin(e).  Coset 1 uses
// stage 0's part (20 KB), cosets 2-3 stages 0-1 (30 KB), cosets 4-7 all.
constexpr uint32_t kEImg512Bytes = 35840, kEImg512Cosets = 7;
constexpr uint32_t kEImg512Stage[3] = {0, 20480, 30720};

// The same for the k = 256, n = 2048 encode (enc_kw.hip): stage 0 of cosets
// j = 4..7 (elements 128 j + e, e < 128), plane q at q * 2048 + cimg_lin(e).
constexpr uint32_t kEImg256Bytes = 10240, kEImg256Cosets = 4;

struct DevTables {
  const uint16_t *skews = nullptr;     // 65535
  const MulTab *mtab = nullptr;        // 65536
  const uint8_t *timg = nullptr;       // kTabImages x kTabImageBytes
  const MulTab *mtab_tin = nullptr;    // 65536, symbols in, tower out
  const MulTab *mtab_tout = nullptr;   // 65536, tower in, symbols out
  const uint8_t *timg_t = nullptr;     // kTabImages x kTabImageBytes, tower images
  const uint8_t *timg_f9 = nullptr;    // kF9Images x kTabImageBytes, F9 variants of tower image 0
  const uint8_t *cimg = nullptr;       // kCImgBytes, the element-indexed compact image
  const MulTab *mslot = nullptr;       // 65535, mslot[i] = mtab[skews[i]]: by skew slot, one load
  const uint8_t *eimg512 = nullptr;    // kEImg512Cosets x kEImg512Bytes, the k = 512 encode's coset images
  const uint8_t *eimg256 = nullptr;    // kEImg256Cosets x kEImg256Bytes, the k = 256 / n = 2048 encode's
};

// Completion signal of a per-call C-ABI call fused into its last kernel: when
// the launcher's kernel runs as a single workgroup it stores v to *flag at
// system scope after its own output (fused = true); otherwise the caller
// launches the separate signal kernel (finish_call).
struct HostSig {
  uint32_t *flag = nullptr;
  uint32_t v = 0;
  bool fused = false;
};

// Per (device, kernel), once and thread-safe: raise `fn`'s dynamic-LDS limit
// to `lds_bytes` (if above the 64 KB default) and return the current device's
// CU count in *cus.  The count is handed out only after the attribute call
// succeeded, so no thread launches a kernel whose limit is not set yet; a
// failed call is retried on the next launch (ec_runtime.cpp).
hipError_t prepare_kernel(const void *fn, int lds_bytes, int *cus);

// Scratch (global memory) needed by each launch for FFT sizes whose working
// set does not fit LDS; 0 for the common sizes.
size_t encode_scratch_bytes(const CodeParams &p, size_t payload_len, size_t batch);
bool encode_scratch_optional(const CodeParams &p);  // only a tile counter: static schedule without it
size_t reconstruct_scratch_bytes(const CodeParams &p, size_t shard_len, size_t batch);

hipError_t launch_encode(const CodeParams &p, const DevTables &t, const uint8_t *d_payloads,
                         size_t payload_len, size_t payload_stride, size_t batch, uint8_t *d_shards,
                         size_t shard_stride, void *scratch, hipStream_t s, HostSig *sig = nullptr);

// Erasure locators (poly_encoder.hpp:90-116, folded form), one workgroup per
// row of d_present.  d_pattern (nullable): rows b with d_pattern[b] != b are
// skipped (their pattern's leader row holds the locator).
hipError_t launch_error_locator(const CodeParams &p, const uint8_t *d_present, size_t batch,
                                const uint16_t *d_fold, const uint32_t *d_pattern,
                                uint16_t *d_err_log, hipStream_t s);
// Pattern dedup: d_pattern[b] = a row whose erasure
// pattern equals payload b's and which is its own leader, or b itself (a hash
// collision with a different pattern only costs the sharing; ec_amd.h).
// Needs dedup_scratch_bytes(batch); batch < 2^31.
// true if launch_error_locator runs the wave-per-pattern form (64 <= n <= 4096),
// cheap enough that a batch computes every row instead of deduplicating
bool locator_wave_applicable(uint32_t n);
// one-lane kernel storing v to a pinned host word (system scope, release)
hipError_t launch_signal_host(uint32_t *h_flag, uint32_t v, hipStream_t s);
// zeroes `bytes` (a multiple of 4) of tile counters at p in stream order
hipError_t launch_zero_counters(uint32_t *p, size_t bytes, hipStream_t s);
size_t dedup_scratch_bytes(size_t batch);
hipError_t launch_dedup_patterns(const CodeParams &p, const uint8_t *d_present, size_t batch,
                                 uint32_t *d_pattern, void *scratch, hipStream_t s);
// follower rows of d_err_log <- their leader's row
hipError_t launch_broadcast_locators(const CodeParams &p, const uint32_t *d_pattern, size_t batch,
                                     uint16_t *d_err_log, hipStream_t s);

// d_pattern (nullable): payload b's erasure pattern is row d_pattern[b] of
// d_present / d_err_log (NULL: row b)
hipError_t launch_reconstruct(const CodeParams &p, const DevTables &t, const uint8_t *d_shards,
                              size_t shard_len, size_t shard_stride, const uint8_t *d_present,
                              const uint16_t *d_err_log, const uint32_t *d_pattern, size_t batch,
                              uint8_t *d_out, size_t out_stride, void *scratch, hipStream_t s);

hipError_t launch_systematic(const CodeParams &p, const uint8_t *d_shards, size_t shard_len,
                             size_t shard_stride, size_t batch, uint8_t *d_out, size_t out_stride,
                             hipStream_t s, HostSig *sig = nullptr);

// the per-call encode of tiny codes (enc_tiny.hip): n <= kTinyMaxN, payload
// <= kTinyBytes and the code's tables carried in the kernel arguments, one workgroup, output rows
// (pitch ostride) written where `out` points (pinned host memory), the
// completion flag stored by the kernel (sig->fused)
constexpr int kTinyMaxN = 16;
constexpr size_t kTinyBytes = 2048;
bool tiny_applicable(const CodeParams &p, size_t plen, size_t ostride);
hipError_t launch_encode_tiny(const CodeParams &p, const DevTables &t, const uint8_t *h_payload, size_t plen,
                              uint8_t *out, size_t ostride, hipStream_t s, HostSig *sig);
// the per-call decode from all k systematic shards of a tiny call (k * slen <=
// kTinyBytes, shards at h_shards with pitch sstride, read on the host into the
// kernel arguments): out = the interleaved payload (pinned), flag by the kernel
bool systematic_tiny_applicable(const CodeParams &p, size_t slen);
hipError_t launch_systematic_tiny(const CodeParams &p, const uint8_t *h_shards, size_t slen, size_t sstride,
                                  uint8_t *out, hipStream_t s, HostSig *sig);
hipError_t warm_encode_tiny(hipStream_t s);  // device set-up: the first launches of the tiny kernels

// specialised kernels (enc_k256.hip)
bool k256_applicable(const CodeParams &p);
// reconstruct_n1024 runs packed (flattened columns, any even shard pitch)
bool n1024_packed(size_t slen, uintptr_t sh, size_t sstride);
// the packed (flattened-piece, any-alignment) encode_k256 applies: small
// payloads or pitches the unpacked kernel cannot take; ..._ok: its own limits
bool k256_packed(size_t plen, size_t pstride, size_t batch, uintptr_t pay, uintptr_t sh, size_t sstride);
bool k256_packed_ok(size_t plen, size_t batch, uintptr_t sh, size_t sstride);
// scratch: k256_scratch_bytes (the n = 1024 unpacked form's tile counter)
hipError_t launch_encode_k256(const CodeParams &p, const DevTables &t, const uint8_t *d_payloads,
                              size_t plen, size_t pstride, size_t batch, uint8_t *d_shards,
                              size_t sstride, void *scratch, hipStream_t s);
size_t k256_scratch_bytes(const CodeParams &p);
// the n = 1024, unpacked case of launch_encode_k256: two 8-wave workgroups per
// CU on the compact image, tiles scheduled dynamically from a counter in
// `scratch` (enc_k256w.hip)
hipError_t launch_encode_k256w(const CodeParams &p, const DevTables &t, const uint8_t *d_payloads,
                               size_t plen, size_t pstride, size_t batch, uint8_t *d_shards,
                               size_t sstride, void *scratch, hipStream_t s);

// specialised kernels (enc_k1024.hip): k = 1024, n = 4096, needs a coefficient
// scratch of k1024_scratch_bytes
bool k1024_applicable(const CodeParams &p);
size_t k1024_scratch_bytes(size_t plen, size_t batch);
hipError_t launch_encode_k1024(const CodeParams &p, const DevTables &t, const uint8_t *d_payloads,
                               size_t plen, size_t pstride, size_t batch, uint8_t *d_shards,
                               size_t sstride, void *scratch, hipStream_t s);

// k = 512, n = 2048 / 4096 (enc_k512w.hip): two 8-wave workgroups per CU on
// the compact image and the per-coset extension images; scratch (nullable:
// static tile schedule) the tile counter, k512w_scratch_bytes
bool k512w_applicable(const CodeParams &p);
size_t k512w_scratch_bytes(const CodeParams &p);
hipError_t launch_encode_k512w(const CodeParams &p, const DevTables &t, const uint8_t *d_payloads,
                               size_t plen, size_t pstride, size_t batch, uint8_t *d_shards,
                               size_t sstride, void *scratch, hipStream_t s);

// k = 16 .. 128, n <= 8 k, and k = 256 at n = 2048 (enc_kw.hip): the same
// model on the compact image (+ coset extension tables at k = 256); scratch
// (nullable) the tile counter, kw_scratch_bytes
bool kw_applicable(const CodeParams &p);
size_t kw_scratch_bytes(const CodeParams &p);
hipError_t launch_encode_kw(const CodeParams &p, const DevTables &t, const uint8_t *d_payloads,
                            size_t plen, size_t pstride, size_t batch, uint8_t *d_shards,
                            size_t sstride, void *scratch, hipStream_t s);

// Per-payload gather order of the received rows, present rows first, per
// 1024-row quarter (or the n < 1024 rows; dec_n1024.hip): the scratch of
// reconstruct_n1024, _n4096 and _gen, gather_order_bytes(p, batch)
size_t gather_order_bytes(const CodeParams &p, size_t batch);
hipError_t launch_gather_order(const CodeParams &p, const uint8_t *d_present,
                               const uint16_t *d_err_log, const uint32_t *d_pattern, size_t batch,
                               uint32_t *order, hipStream_t s);

// specialised kernels (dec_n1024.hip); scratch: n1024_scratch_bytes(p, batch)
bool n1024_applicable(const CodeParams &p);
hipError_t launch_reconstruct_n1024(const CodeParams &p, const DevTables &t,
                                    const uint8_t *d_shards, size_t slen, size_t sstride,
                                    const uint8_t *d_present, const uint16_t *d_err_log,
                                    const uint32_t *d_pattern, size_t batch, uint8_t *d_out,
                                    size_t ostride, void *scratch, hipStream_t s);
// the 12-wave form (dec_n1024x.hip) for the unpacked case; both take
// n1024_scratch_bytes (the gather order + the 12-wave form's tile counter)
size_t n1024_scratch_bytes(const CodeParams &p, size_t batch);
size_t n1024_tick_offset(const CodeParams &p, size_t batch);
hipError_t launch_reconstruct_n1024x(const CodeParams &p, const DevTables &t,
                                     const uint8_t *d_shards, size_t slen, size_t sstride,
                                     const uint8_t *d_present, const uint16_t *d_err_log,
                                     const uint32_t *d_pattern, size_t batch, uint8_t *d_out,
                                     size_t ostride, void *scratch, hipStream_t s);

// specialised kernels (dec_n4096.hip); scratch: n4096_scratch_bytes(p, batch)
bool n4096_applicable(const CodeParams &p);
size_t n4096_scratch_bytes(const CodeParams &p, size_t batch);
hipError_t launch_reconstruct_n4096(const CodeParams &p, const DevTables &t,
                                    const uint8_t *d_shards, size_t slen, size_t sstride,
                                    const uint8_t *d_present, const uint16_t *d_err_log,
                                    const uint32_t *d_pattern, size_t batch, uint8_t *d_out,
                                    size_t ostride, void *scratch, hipStream_t s);

// register-blocked reconstruct for 64 <= n <= 1024, 16 <= k <= 512 (dec_gen.hip);
// scratch: gather_order_bytes(p, batch)
bool decgen_applicable(const CodeParams &p);
hipError_t launch_reconstruct_gen(const CodeParams &p, const DevTables &t,
                                  const uint8_t *d_shards, size_t slen, size_t sstride,
                                  const uint8_t *d_present, const uint16_t *d_err_log,
                                  const uint32_t *d_pattern, size_t batch, uint8_t *d_out,
                                  size_t ostride, void *scratch, hipStream_t s);

}  // namespace ecamd
