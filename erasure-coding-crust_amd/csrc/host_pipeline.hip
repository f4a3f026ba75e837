// host_pipeline.hip — host-resident batch encode / reconstruct (SURVEY.md
// §8f row 2): the reference path starts and ends in host memory (block data
// in, shards out), so these entry points stream a host batch through the GPU
// in chunks, with three slots (stream + device buffers each) so that chunk
// i's H2D, chunk i-1's kernels and chunk i-2's D2H overlap on the two copy
// engines and the CUs.  Host buffers should be pinned (ECCR_AMD_host_alloc)
// for full PCIe rate; pageable memory works but is staged by the runtime.
//
// Reconstruct takes only the present shards, compacted per payload
// ([batch][cnt][sstride] + their indices), so PCIe carries exactly the bytes
// the codec needs; `scatter_present` places them into codeword rows on the
// device and builds the present mask for the error locator.
#include <hip/hip_runtime.h>

#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/erasure_coding/ec_amd.h"
#include "ec_kernels.hpp"
#include "ec_runtime.hpp"
#include "gf_field.hpp"

namespace ecamd {
namespace {

constexpr int kSlots = 3;

// block (j, b): compact row j of payload b -> full row idx[b][j]; present[b][v] = 1
__global__ void __launch_bounds__(256) scatter_present(const uint8_t *__restrict__ compact,
                                                       uint64_t cstride, const uint16_t *__restrict__ idx,
                                                       uint32_t cnt, uint64_t slen,
                                                       uint8_t *__restrict__ full, uint64_t fstride,
                                                       uint32_t nv, uint8_t *__restrict__ present,
                                                       uint32_t n, uint32_t batch) {
  const uint32_t j = blockIdx.x;
  for (uint32_t b = blockIdx.y; b < batch; b += gridDim.y) {  // batch may exceed gridDim.y's limit
    const uint32_t v = idx[uint64_t(b) * cnt + j];
    if (v >= nv) continue;  // validated on the host; never index out of the row block
    const uint8_t *src = compact + (uint64_t(b) * cnt + j) * cstride;
    uint8_t *dst = full + (uint64_t(b) * nv + v) * fstride;
    if (present && threadIdx.x == 0) present[uint64_t(b) * n + v] = 1;
    const bool vec = ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0;
    const uint64_t nvec = vec ? slen / 16 : 0;
    for (uint64_t e = threadIdx.x; e < nvec; e += blockDim.x)
      reinterpret_cast<uint4 *>(dst)[e] = reinterpret_cast<const uint4 *>(src)[e];
    for (uint64_t e = nvec * 16 + threadIdx.x; e < slen; e += blockDim.x) dst[e] = src[e];
  }
}

struct Slot {
  hipStream_t stream = nullptr;
  uint8_t *d_a = nullptr, *d_b = nullptr, *d_c = nullptr;
  uint16_t *d_elog = nullptr;
  // a chunk's pattern index ([cb] u32), its shards' indices ([cb][cnt]
  // u16) and its distinct present rows ([npat][n]) in one device buffer,
  // uploaded by ONE copy from the pinned h_meta (until round 6: three copies,
  // two of them from pageable vectors, beside the shards' copy)
  uint8_t *d_meta = nullptr, *h_meta = nullptr;
  size_t cap_meta = 0, cap_h_meta = 0;
  // the slot's own kernel scratch (k = 1024 encode coefficients, reconstruct
  // gather orders): stream-ordered by the slot, so the three slots overlap; a
  // shared per-device lease would order them behind each other
  uint8_t *d_scr = nullptr;
  size_t cap_a = 0, cap_b = 0, cap_c = 0, cap_elog = 0, cap_scr = 0;
  // host staging of a chunk's distinct erasure patterns (h_rows, then copied
  // into h_meta); `staged` is recorded after h_meta's upload so the next chunk
  // on this slot does not overwrite it early
  std::vector<uint8_t> h_rows;
  hipEvent_t staged = nullptr;
};

struct Pipeline {
  Slot slot[kSlots];
  int device = -1;
  ~Pipeline() { release(); }
  // synchronise and free every slot's stream and buffers, on their own device
  void release() {
    if (device < 0) return;
    int cur = -1;
    const bool switched = hipGetDevice(&cur) == hipSuccess && cur != device &&
                          hipSetDevice(device) == hipSuccess;
    for (Slot &s : slot) {
      if (s.stream) {
        (void)hipStreamSynchronize(s.stream);
        (void)hipStreamDestroy(s.stream);
      }
      if (s.staged) (void)hipEventDestroy(s.staged);
      for (void *p : {static_cast<void *>(s.d_a), static_cast<void *>(s.d_b), static_cast<void *>(s.d_c),
                      static_cast<void *>(s.d_meta), static_cast<void *>(s.d_elog),
                      static_cast<void *>(s.d_scr)})
        if (p) (void)hipFree(p);
      if (s.h_meta) (void)hipHostFree(s.h_meta);
      s = Slot{};
    }
    if (switched) (void)hipSetDevice(cur);
    device = -1;
  }
};

// chunk = 0: payloads per pipeline step such that a step moves ~32 MB over
// the link (small payloads: few large copies instead of many latency-bound
// ones; large payloads: still >= 3 steps in flight when the batch allows)
unsigned long auto_chunk(size_t bytes_per_payload, unsigned long batch) {
  const size_t target = size_t(32) << 20;
  size_t c = bytes_per_payload ? target / bytes_per_payload : batch;
  if (c < 1) c = 1;
  if (batch >= 3 && c > (batch + 2) / 3 && bytes_per_payload * ((batch + 2) / 3) >= (size_t(4) << 20))
    c = (batch + 2) / 3;  // keep the three slots busy on big batches
  return c > batch ? batch : c;
}

Pipeline *pipeline() {  // one per host thread (reentrant like the reference)
  thread_local Pipeline pl;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  if (pl.device != dev) {
    pl.release();  // the previous device's slots
    pl.device = dev;
    for (Slot &s : pl.slot)
      if (hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking) != hipSuccess ||
          hipEventCreateWithFlags(&s.staged, hipEventDisableTiming) != hipSuccess) {
        pl.release();
        return nullptr;
      }
  }
  return &pl;
}

template <typename T>
bool grow(T **p, size_t *cap, size_t bytes) {
  return ensure_dev(reinterpret_cast<void **>(p), cap, bytes);
}

// the slot's scratch for `bytes` (nullptr and true when none is needed)
bool slot_scratch(Slot &s, size_t bytes, void **out) {
  *out = nullptr;
  if (bytes == 0) return true;
  if (!grow(&s.d_scr, &s.cap_scr, bytes)) return false;
  *out = s.d_scr;
  return true;
}

bool ok(hipError_t e, const char *what) {
  if (e == hipSuccess) return true;
  set_error(std::string("erasure_coding_crust(amd): ") + what + ": " + hipGetErrorString(e));
  return false;
}

NPRSResult res(NPRSResult_Tag t) {
  NPRSResult r;
  std::memset(&r, 0, sizeof r);
  r.tag = t;
  return r;
}

size_t round16(size_t x) { return (x + 15) / 16 * 16; }

uint64_t mix64(uint64_t x) {  // splitmix64 finaliser (pattern hash terms)
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

}  // namespace
}  // namespace ecamd

using namespace ecamd;

extern "C" {

void *ECCR_AMD_host_alloc(unsigned long bytes) {
  void *p = nullptr;
  if (hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) return nullptr;
  return p;
}

void ECCR_AMD_host_free(void *p) {
  if (p) (void)hipHostFree(p);
}

NPRSResult ECCR_AMD_encode_host_batch(unsigned long nv, const uint8_t *h_payloads,
                                      unsigned long plen, unsigned long pstride,
                                      unsigned long batch, uint8_t *h_shards,
                                      unsigned long sstride, unsigned long chunk) {
  CodeParams p;
  if (code_params(nv, &p) != ParamError::kOk) return res(NPRS_RESULT_UNKNOWN_CODE_PARAM);
  if (plen == 0 || !h_payloads || !h_shards) return res(NPRS_RESULT_BAD_PAYLOAD);
  const size_t sl = shard_len(p.k, plen);
  if (pstride < plen || sstride < sl) return res(NPRS_RESULT_BAD_PAYLOAD);
  DeviceState *d = device_state();
  Pipeline *pl = d ? pipeline() : nullptr;
  if (!pl) return res(NPRS_RESULT_UNKNOWN_CODE_PARAM);
  if (chunk == 0) chunk = auto_chunk(plen + size_t(nv) * sl, batch);
  // Device rows use the host stride (one linear copy) when it already suits the
  // fast kernels or rows are short: a 2-D copy of many narrow rows is
  // descriptor-bound (2-byte rows ran at ~10 us per row).  Otherwise rows are
  // re-pitched to aligned device strides by a 2-D copy of long rows.
  const bool pay_lin = pstride % 16 == 0 || plen < 256;
  const bool sh_lin = sstride % 8 == 0 || sl < 256;
  const size_t dps = pay_lin ? pstride : round16(plen);
  const size_t dss = sh_lin ? sstride : (sl + 63) / 64 * 64;
  for (unsigned long c0 = 0, i = 0; c0 < batch; c0 += chunk, ++i) {
    Slot &s = pl->slot[i % kSlots];
    const size_t cb = batch - c0 < chunk ? batch - c0 : chunk;
    if (!grow(&s.d_a, &s.cap_a, chunk * dps) || !grow(&s.d_b, &s.cap_b, chunk * nv * dss))
      return res(NPRS_RESULT_UNKNOWN_CODE_PARAM);
    void *scratch = nullptr;
    if (!slot_scratch(s, encode_scratch_bytes(p, plen, cb), &scratch))
      return res(NPRS_RESULT_UNKNOWN_CODE_PARAM);
    const uint8_t *hp = h_payloads + c0 * pstride;
    uint8_t *hs = h_shards + c0 * nv * sstride;
    const hipError_t up =
        pay_lin ? hipMemcpyAsync(s.d_a, hp, (cb - 1) * pstride + plen, hipMemcpyHostToDevice, s.stream)
                : hipMemcpy2DAsync(s.d_a, dps, hp, pstride, plen, cb, hipMemcpyHostToDevice, s.stream);
    if (!ok(up, "H2D payloads") ||
        !ok(launch_encode(p, device_tables(d), s.d_a, plen, dps, cb, s.d_b, dss, scratch, s.stream),
            "encode launch"))
      return res(NPRS_RESULT_UNKNOWN_CODE_PARAM);
    const hipError_t down =
        sh_lin ? hipMemcpyAsync(hs, s.d_b, (cb * nv - 1) * sstride + sl, hipMemcpyDeviceToHost,
                                s.stream)
               : hipMemcpy2DAsync(hs, sstride, s.d_b, dss, sl, cb * nv, hipMemcpyDeviceToHost,
                                  s.stream);
    if (!ok(down, "D2H shards"))
      return res(NPRS_RESULT_UNKNOWN_CODE_PARAM);
  }
  for (Slot &s : pl->slot)
    if (!ok(hipStreamSynchronize(s.stream), "encode_host_batch"))
      return res(NPRS_RESULT_UNKNOWN_CODE_PARAM);
  return res(NPRS_RESULT_OK);
}

NPRSResult ECCR_AMD_reconstruct_host_batch(unsigned long nv, const uint8_t *h_shards,
                                           unsigned long slen, unsigned long sstride,
                                           const uint16_t *h_index, unsigned long cnt,
                                           unsigned long batch, uint8_t *h_out,
                                           unsigned long ostride, unsigned long chunk) {
  CodeParams p;
  if (code_params(nv, &p) != ParamError::kOk) return res(NPRS_RESULT_UNKNOWN_CODE_PARAM);
  if (!h_shards || !h_index || !h_out) return res(NPRS_RESULT_BAD_PAYLOAD);
  if (slen % 2 != 0) return res(NPRS_RESULT_UNEVEN_LENGTH);
  if (sstride < slen || ostride < slen * p.k) return res(NPRS_RESULT_NON_UNIFORM_CHUNKS);
  if (cnt < p.k) return res(NPRS_RESULT_NOT_ENOUGH_CHUNKS);  // reed-solomon.hpp:99-100
  // src/erasure_coding.rs:370-375 (index bounds) and reed-solomon.hpp:99-100
  // (enough distinct shards; a repeated index counts once, its rows must agree)
  // per payload: its erasure pattern's hash (sum of mix64 over the distinct
  // present indices) and size, for the per-chunk pattern dedup below
  std::vector<uint32_t> seen(nv, 0);
  std::vector<uint64_t> phash(batch);
  std::vector<uint32_t> pcount(batch);
  std::vector<uint64_t> term(nv);  // mix64 of each index, once per call
  for (unsigned long v = 0; v < nv; ++v) term[v] = mix64(v);
  for (unsigned long b = 0; b < batch; ++b) {
    unsigned long distinct = 0;
    uint64_t h = 0;
    for (unsigned long j = 0; j < cnt; ++j) {
      const uint16_t v = h_index[b * cnt + j];
      if (v >= nv) {
        NPRSResult r = res(NPRS_RESULT_CHUNK_INDEX_OUT_OF_BOUNDS);
        r.chunk_index_out_of_bounds.chunk_index = v;
        r.chunk_index_out_of_bounds.n_validators = nv;
        return r;
      }
      if (seen[v] != b + 1) {
        seen[v] = uint32_t(b + 1);
        ++distinct;
        h += term[v];
      }
    }
    if (distinct < p.k) return res(NPRS_RESULT_NOT_ENOUGH_CHUNKS);
    phash[b] = h;
    pcount[b] = uint32_t(distinct);
  }
  DeviceState *d = device_state();
  const uint16_t *fold = d ? device_fold(d, p.n) : nullptr;
  Pipeline *pl = fold ? pipeline() : nullptr;
  if (!pl) return res(NPRS_RESULT_UNKNOWN_RECONSTRUCTION);
  if (chunk == 0) chunk = auto_chunk(size_t(cnt) * sstride + size_t(slen) * p.k, batch);
  const size_t dss = (slen + 63) / 64 * 64, ob = slen * p.k;
  const bool out_lin = ostride % 8 == 0 || ob < 256;  // as in encode: linear copy if it suits
  const size_t dos = out_lin ? ostride : ob;
  for (unsigned long c0 = 0, i = 0; c0 < batch; c0 += chunk, ++i) {
    Slot &s = pl->slot[i % kSlots];
    const size_t cb = batch - c0 < chunk ? batch - c0 : chunk;
    // h_meta / d_meta: [pattern index | shard indices | present rows], each part 256-B aligned
    const size_t pat_bytes = (chunk * 4 + 255) / 256 * 256, idx_bytes = (chunk * cnt * 2 + 255) / 256 * 256;
    const size_t rows_at = pat_bytes + idx_bytes;
    if (!grow(&s.d_a, &s.cap_a, chunk * cnt * sstride) || !grow(&s.d_b, &s.cap_b, chunk * nv * dss) ||
        !grow(&s.d_c, &s.cap_c, chunk * dos) || !grow(&s.d_meta, &s.cap_meta, rows_at + chunk * p.n) ||
        !grow(&s.d_elog, &s.cap_elog, chunk * p.n * 2))
      return res(NPRS_RESULT_UNKNOWN_RECONSTRUCTION);
    uint32_t *d_pat = reinterpret_cast<uint32_t *>(s.d_meta);
    const uint16_t *d_idx = reinterpret_cast<const uint16_t *>(s.d_meta + pat_bytes);
    uint8_t *d_present = s.d_meta + rows_at;
    // distinct erasure patterns of the chunk: one present
    // row and one locator each; payload b uses row h_pat[b]
    if (!ok(hipEventSynchronize(s.staged), "staging reuse")) return res(NPRS_RESULT_UNKNOWN_RECONSTRUCTION);
    if (!ensure_host(&s.h_meta, &s.cap_h_meta, rows_at + chunk * p.n))
      return res(NPRS_RESULT_UNKNOWN_RECONSTRUCTION);
    std::memcpy(s.h_meta + pat_bytes, h_index + c0 * cnt, cb * cnt * 2);
    uint32_t *h_pat = reinterpret_cast<uint32_t *>(s.h_meta);
    s.h_rows.clear();
    s.h_rows.reserve(cb * p.n);
    // hash -> first pattern with it; further ones chained through next_pat
    std::unordered_map<uint64_t, uint32_t> by_hash;
    by_hash.reserve(cb);
    std::vector<int32_t> next_pat;
    std::vector<uint32_t> pat_count;  // distinct indices per pattern
    uint32_t npat = 0;
    for (size_t j = 0; j < cb; ++j) {
      const size_t b = c0 + j;
      const uint16_t *ix = h_index + b * cnt;
      if (j > 0 && std::memcmp(ix, ix - cnt, cnt * 2) == 0) {  // same list as the previous payload
        h_pat[j] = h_pat[j - 1];
        continue;
      }
      int32_t found = -1;
      const auto head = by_hash.find(phash[b]);
      const int32_t first = head == by_hash.end() ? -1 : int32_t(head->second);
      for (int32_t q = first; q >= 0; q = next_pat[q]) {  // equal sets: same size, every index of b in q's row
        const uint8_t *row = s.h_rows.data() + size_t(q) * p.n;
        bool same = pat_count[q] == pcount[b];
        for (unsigned long t = 0; t < cnt && same; ++t) same = row[ix[t]] != 0;
        if (same) {
          found = q;
          break;
        }
      }
      if (found < 0) {
        found = int32_t(npat++);
        next_pat.push_back(first);  // new head of the hash's chain
        by_hash[phash[b]] = uint32_t(found);
        pat_count.push_back(pcount[b]);
        s.h_rows.resize(size_t(npat) * p.n, 0);
        uint8_t *row = s.h_rows.data() + size_t(found) * p.n;
        for (unsigned long t = 0; t < cnt; ++t) row[ix[t]] = 1;
      }
      h_pat[j] = uint32_t(found);
    }
    std::memcpy(s.h_meta + rows_at, s.h_rows.data(), size_t(npat) * p.n);
    void *scratch = nullptr;
    if (!slot_scratch(s, reconstruct_scratch_bytes(p, slen, cb), &scratch))
      return res(NPRS_RESULT_UNKNOWN_RECONSTRUCTION);
    bool good =
        ok(hipMemcpyAsync(s.d_a, h_shards + c0 * cnt * sstride, cb * cnt * sstride,
                          hipMemcpyHostToDevice, s.stream),
           "H2D shards") &&
        ok(hipMemcpyAsync(s.d_meta, s.h_meta, rows_at + size_t(npat) * p.n, hipMemcpyHostToDevice,
                          s.stream),
           "H2D patterns") &&
        ok(hipEventRecord(s.staged, s.stream), "staging event");
    if (good) {
      hipLaunchKernelGGL(scatter_present, dim3(unsigned(cnt), unsigned(cb < 65535 ? cb : 65535)), dim3(256),
                         0, s.stream, s.d_a, uint64_t(sstride), d_idx, uint32_t(cnt), uint64_t(slen),
                         s.d_b, uint64_t(dss), uint32_t(nv), static_cast<uint8_t *>(nullptr),
                         uint32_t(p.n), uint32_t(cb));
      good = ok(hipGetLastError(), "scatter launch") &&
             ok(launch_error_locator(p, d_present, npat, fold, nullptr, s.d_elog, s.stream),
                "error locator launch") &&
             ok(launch_reconstruct(p, device_tables(d), s.d_b, slen, dss, d_present, s.d_elog,
                                   d_pat, cb, s.d_c, dos, scratch, s.stream),
                "reconstruct launch") &&
             ok(out_lin ? hipMemcpyAsync(h_out + c0 * ostride, s.d_c, (cb - 1) * ostride + ob,
                                         hipMemcpyDeviceToHost, s.stream)
                        : hipMemcpy2DAsync(h_out + c0 * ostride, ostride, s.d_c, ob, ob, cb,
                                           hipMemcpyDeviceToHost, s.stream),
                "D2H payloads");
    }
    if (!good) return res(NPRS_RESULT_UNKNOWN_RECONSTRUCTION);
  }
  for (Slot &s : pl->slot)
    if (!ok(hipStreamSynchronize(s.stream), "reconstruct_host_batch"))
      return res(NPRS_RESULT_UNKNOWN_RECONSTRUCTION);
  return res(NPRS_RESULT_OK);
}

}  // extern "C"
