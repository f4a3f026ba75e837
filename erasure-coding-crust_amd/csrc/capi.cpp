// capi.cpp — the erasure_coding.h C ABI (src/erasure_coding.rs of the
// reference) plus the ec_amd.h device-batch extension, on the HIP path.
//
// Validation order and error mapping follow src/erasure_coding.rs; the codec
// results follow ec-cpp (include/ec-cpp/reed-solomon.hpp).  Deliberate
// divergence: where the Rust layer panics (null/empty payload, null out
// pointers) we return NPRS_RESULT_BAD_PAYLOAD / abort with a message.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <optional>
#include <string>
#include <vector>

#include "../../include/erasure_coding/ec_amd.h"
#include "../../include/erasure_coding/erasure_coding.h"
#include "ec_kernels.hpp"
#include "ec_runtime.hpp"
#include "gf_field.hpp"

using namespace ecamd;

namespace {

struct Workspace {  // caller-owned device scratch (the *_ws batch entry points)
  void *ptr;
  size_t bytes;
};

NPRSResult result(NPRSResult_Tag tag) {
  NPRSResult r;
  std::memset(&r, 0, sizeof r);
  r.tag = tag;
  return r;
}

[[noreturn]] void contract_violation(const char *what) {  // Rust assert! == abort
  std::fprintf(stderr, "erasure_coding_crust(amd): contract violation: %s\n", what);
  std::abort();
}

// src/erasure_coding.rs:70-98 (recovery_threshold + code_params)
NPRSResult params_or_error(unsigned long nv, CodeParams *p) {
  switch (code_params(nv, p)) {
    case ParamError::kTooManyValidators: return result(NPRS_RESULT_TOO_MANY_VALIDATORS);
    case ParamError::kNotEnoughValidators: return result(NPRS_RESULT_NOT_ENOUGH_VALIDATORS);
    default: return result(NPRS_RESULT_OK);
  }
}

bool hip_check(hipError_t e, const char *what) {
  if (e == hipSuccess) return true;
  set_error(std::string("erasure_coding_crust(amd): ") + what + ": " + hipGetErrorString(e));
  return false;
}

// device row pitch of the per-call paths: 16-B aligned rows for the fast
// kernels; the host staging buffers use the same pitch, so every host<->device
// copy is one linear transfer (a 2-D copy of narrow rows costs ~10 us per row)
inline size_t dev_pitch(size_t sl) { return (sl + 15) / 16 * 16; }

// Calls whose input and output together stay below this run the kernel on
// the pinned staging buffers themselves (device-mapped host memory, read and
// written over PCIe): no copy commands, so a small call costs one launch and
// one synchronisation instead of three commands.  Kernel launches acquire
// and release at system scope, so the host's staging writes are seen by the
// kernel and its results by the host after the synchronisation.
constexpr size_t kDirectBytes = size_t(64) << 10;

// host -> device -> host encode of one payload into pinned h_out [nv][dev_pitch(sl)]
bool encode_host(const CodeParams &p, const uint8_t *payload, size_t len, HostCtx *c,
                 size_t *sl_out) {
  DeviceState *d = device_state();
  if (!d) return false;
  const size_t sl = shard_len(p.k, len);
  const size_t dstride = dev_pitch(sl);
  const size_t out_bytes = size_t(p.nv) * dstride;
  if (tiny_applicable(p, len, dstride) && out_bytes <= kDirectBytes) {
    // tiny codes and payloads (enc_tiny.hip): the payload rides in the kernel
    // arguments, the rows go straight to the pinned output
    if (!ensure_host(&c->h_out, &c->h_out_cap, out_bytes)) return false;
    HostSig sig = call_signal(c);
    if (!hip_check(launch_encode_tiny(p, device_tables(d), payload, len, c->h_out, dstride, c->stream, &sig),
                   "encode launch") ||
        !finish_call(c, "encode", &sig))
      return false;
    *sl_out = sl;
    return true;
  }
  if (len + out_bytes <= kDirectBytes) {
    if (!ensure_host(&c->h_in, &c->h_in_cap, len) || !ensure_host(&c->h_out, &c->h_out_cap, out_bytes))
      return false;
    ScratchLease lease(d, encode_scratch_bytes(p, len, 1), c->stream);
    if (!lease.ok()) return false;
    std::memcpy(c->h_in, payload, len);
    HostSig sig = call_signal(c);  // stored by the encode kernel itself when it can (HostSig)
    if (!hip_check(launch_encode(p, device_tables(d), c->h_in, len, len, 1, c->h_out, dstride,
                                 lease.ptr(), c->stream, &sig),
                   "encode launch") ||
        !finish_call(c, "encode", &sig))
      return false;
    *sl_out = sl;
    return true;
  }
  if (!ensure_host(&c->h_in, &c->h_in_cap, len) ||
      !ensure_dev(reinterpret_cast<void **>(&c->d_in), &c->d_in_cap, len) ||
      !ensure_host(&c->h_out, &c->h_out_cap, out_bytes) ||
      !ensure_dev(reinterpret_cast<void **>(&c->d_out), &c->d_out_cap, size_t(p.nv) * dstride))
    return false;
  ScratchLease lease(d, encode_scratch_bytes(p, len, 1), c->stream);
  if (!lease.ok()) return false;
  void *scratch = lease.ptr();
  std::memcpy(c->h_in, payload, len);
  if (!hip_check(hipMemcpyAsync(c->d_in, c->h_in, len, hipMemcpyHostToDevice, c->stream), "H2D") ||
      !hip_check(launch_encode(p, device_tables(d), c->d_in, len, len, 1, c->d_out, dstride,
                               scratch, c->stream),
                 "encode launch") ||
      !hip_check(hipMemcpyAsync(c->h_out, c->d_out, out_bytes, hipMemcpyDeviceToHost, c->stream),
                 "D2H") ||
      !hip_check(hipStreamSynchronize(c->stream), "encode"))
    return false;
  *sl_out = sl;
  return true;
}

// reconstruct from shards staged in c->h_in ([nv][dev_pitch(sl)], present[] flags) into c->h_out
bool reconstruct_host(const CodeParams &p, const std::vector<uint8_t> &present, size_t sl,
                      HostCtx *c) {
  DeviceState *d = device_state();
  if (!d) return false;
  const size_t in_bytes = size_t(p.nv) * sl, out_bytes = sl * p.k;
  const size_t dstride = dev_pitch(sl);
  if (!ensure_dev(reinterpret_cast<void **>(&c->d_in), &c->d_in_cap, size_t(p.nv) * dstride) ||
      !ensure_dev(reinterpret_cast<void **>(&c->d_out), &c->d_out_cap, out_bytes) ||
      !ensure_host(&c->h_out, &c->h_out_cap, out_bytes))
    return false;
  bool all_systematic = true;
  for (uint32_t y = 0; y < p.k; ++y) all_systematic &= present[y] != 0;
  (void)in_bytes;
  // small calls: the kernels read the staged shards and write the payload
  // in pinned host memory (kDirectBytes)
  const bool direct = size_t(p.nv) * dstride + out_bytes <= kDirectBytes;
  const uint8_t *src = direct ? c->h_in : c->d_in;
  uint8_t *dst = direct ? c->h_out : c->d_out;
  if (!direct && !hip_check(hipMemcpyAsync(c->d_in, c->h_in, size_t(p.nv) * dstride,
                                           hipMemcpyHostToDevice, c->stream),
                            "H2D"))
    return false;
  HostSig sig = direct ? call_signal(c) : HostSig();
  if (all_systematic && direct && systematic_tiny_applicable(p, sl)) {
    // tiny calls: the k systematic shards ride in the kernel arguments (enc_tiny.hip)
    if (!hip_check(launch_systematic_tiny(p, c->h_in, sl, dstride, dst, c->stream, &sig), "systematic launch"))
      return false;
  } else if (all_systematic) {
    // every systematic shard is present: decode == interleave (exact)
    if (!hip_check(launch_systematic(p, src, sl, dstride, 1, dst, out_bytes, c->stream, &sig),
                   "systematic launch"))
      return false;
  } else {
    // the pattern's locator: computed once per device, then reused (§8f row 3)
    std::shared_ptr<const Locator> loc = cached_locator(d, p, present, c->stream);
    if (!loc) return false;
    // on every path below `loc` is dropped only after the stream finished (the
    // cache recycles entries nobody holds, and uses an entry's event only
    // while it is not done: ec_runtime.hpp)
    const auto release = [&](bool ok) {
      // a failed synchronisation may mean the locator kernel itself faulted:
      // the entry leaves the cache instead of being marked done, so no later
      // hit skips the event wait and reads d_elog that was never written
      if (!ok && hipStreamSynchronize(c->stream) != hipSuccess) locator_drop(d, *loc);
      else locator_done(d, *loc);
      return ok;
    };
    ScratchLease lease(d, reconstruct_scratch_bytes(p, sl, 1), c->stream);
    if (!lease.ok()) return release(false);
    void *scratch = lease.ptr();
    const bool launched = hip_check(launch_reconstruct(p, device_tables(d), src, sl, dstride,
                                                       loc->d_present, loc->d_elog, nullptr, 1,
                                                       dst, out_bytes, scratch, c->stream),
                                    "reconstruct launch");
    const bool copied = launched && (direct || hip_check(hipMemcpyAsync(c->h_out, c->d_out, out_bytes,
                                                                        hipMemcpyDeviceToHost, c->stream),
                                                         "D2H"));
    // Kernels only (direct): the signal-kernel wait; after a D2H copy the
    // copy-to-kernel hand-off makes that slower than waiting on the stream
    // 
    const bool synced = (launched && copied) &&
                        (direct ? finish_call(c, "reconstruct", &sig)
                                : hip_check(hipStreamSynchronize(c->stream), "reconstruct"));
    return release(launched && copied && synced);
  }
  return (direct || hip_check(hipMemcpyAsync(c->h_out, c->d_out, out_bytes, hipMemcpyDeviceToHost,
                                             c->stream),
                              "D2H")) &&
         (direct ? finish_call(c, "reconstruct", &sig)
                 : hip_check(hipStreamSynchronize(c->stream), "reconstruct"));
}

bool take_output(HostCtx *c, size_t bytes, DataBlock *out) {
  uint8_t *buf = static_cast<uint8_t *>(std::malloc(bytes ? bytes : 1));
  if (!buf) return false;
  std::memcpy(buf, c->h_out, bytes);
  out->array = buf;
  out->length = bytes;
  return true;
}

}  // namespace

extern "C" {

NPRSResult ECCR_get_recovery_threshold(unsigned long nv, unsigned long *threshold_out) {
  if (!threshold_out) contract_violation("threshold_out is null");
  CodeParams p;
  NPRSResult r = params_or_error(nv, &p);
  if (r.tag == NPRS_RESULT_OK) *threshold_out = p.threshold;
  return r;
}

void ECCR_deallocate_data_block(DataBlock *data) {
  if (!data || !data->array) contract_violation("deallocate_data_block: null");
  std::free(data->array);
  data->array = nullptr;
  data->length = 0;
}

void ECCR_deallocate_chunk(Chunk *data) {
  if (!data) contract_violation("deallocate_chunk: null");
  ECCR_deallocate_data_block(&data->data);
}

void ECCR_deallocate_chunk_list(ChunksList *list) {
  if (!list || !list->data) contract_violation("deallocate_chunk_list: null");
  for (unsigned long i = 0; i < list->count; ++i) ECCR_deallocate_chunk(&list->data[i]);
  std::free(list->data);
  list->data = nullptr;
  list->count = 0;
}

NPRSResult ECCR_AFFT_Table(uint16_t (*output)[65535]) {
  if (!output) contract_violation("AFFT_Table: null");
  std::memcpy(*output, field().skews.data(), 65535 * sizeof(uint16_t));
  return result(NPRS_RESULT_OK);
}

NPRSResult ECCR_obtain_chunks(unsigned long nv, const DataBlock *message, ChunksList *output) {
  if (!message || !output) contract_violation("obtain_chunks: null argument");
  CodeParams p;
  NPRSResult r = params_or_error(nv, &p);
  if (r.tag != NPRS_RESULT_OK) return r;
  if (!message->array || message->length == 0) return result(NPRS_RESULT_BAD_PAYLOAD);
  HostCtx *c = host_ctx();
  size_t sl = 0;
  if (!c || !encode_host(p, message->array, message->length, c, &sl))
    return result(NPRS_RESULT_UNKNOWN_CODE_PARAM);
  Chunk *chunks = static_cast<Chunk *>(std::malloc(sizeof(Chunk) * nv));
  if (!chunks) return result(NPRS_RESULT_UNKNOWN_CODE_PARAM);
  for (unsigned long v = 0; v < nv; ++v) {
    uint8_t *b = static_cast<uint8_t *>(std::malloc(sl));
    std::memcpy(b, c->h_out + v * dev_pitch(sl), sl);
    chunks[v].data.array = b;
    chunks[v].data.length = sl;
    chunks[v].index = v;
  }
  output->data = chunks;
  output->count = nv;
  return result(NPRS_RESULT_OK);
}

NPRSResult ECCR_reconstruct(unsigned long nv, const ChunksList *input, DataBlock *outdata) {
  if (!outdata || !input || !input->data) contract_violation("reconstruct: null argument");
  CodeParams p;
  NPRSResult r = params_or_error(nv, &p);
  if (r.tag != NPRS_RESULT_OK) return r;
  // src/erasure_coding.rs:363-387: first n_validators entries, positional
  std::vector<const Chunk *> slot(nv, nullptr);
  unsigned long sl = 0;
  bool have_len = false;
  const unsigned long take = input->count < nv ? input->count : nv;
  for (unsigned long i = 0; i < take; ++i) {
    const Chunk &ch = input->data[i];
    if (ch.index >= nv) {
      NPRSResult e = result(NPRS_RESULT_CHUNK_INDEX_OUT_OF_BOUNDS);
      e.chunk_index_out_of_bounds.chunk_index = ch.index;
      e.chunk_index_out_of_bounds.n_validators = nv;
      return e;
    }
    if (!ch.data.array || ch.data.length == 0) continue;
    if (!have_len) {
      sl = ch.data.length;
      have_len = true;
    }
    if (sl % 2 != 0) return result(NPRS_RESULT_UNEVEN_LENGTH);
    if (sl != ch.data.length) return result(NPRS_RESULT_NON_UNIFORM_CHUNKS);
    slot[ch.index] = &ch;
  }
  std::vector<uint8_t> present(p.n, 0);
  uint32_t count = 0;
  for (unsigned long v = 0; v < nv; ++v)
    if (slot[v]) {
      present[v] = 1;
      ++count;
    }
  if (count < p.k) return result(NPRS_RESULT_NOT_ENOUGH_CHUNKS);  // reed-solomon.hpp:99-100
  HostCtx *c = host_ctx();
  if (!c || !ensure_host(&c->h_in, &c->h_in_cap, size_t(nv) * dev_pitch(sl)))
    return result(NPRS_RESULT_UNKNOWN_RECONSTRUCTION);
  for (unsigned long v = 0; v < nv; ++v)
    if (slot[v]) std::memcpy(c->h_in + v * dev_pitch(sl), slot[v]->data.array, sl);
  if (!reconstruct_host(p, present, sl, c) || !take_output(c, sl * p.k, outdata))
    return result(NPRS_RESULT_UNKNOWN_RECONSTRUCTION);
  return result(NPRS_RESULT_OK);
}

NPRSResult ECCR_reconstruct_from_systematic(unsigned long nv, const ChunksList *input,
                                            DataBlock *outdata) {
  if (!outdata || !input || !input->data) contract_violation("systematic: null argument");
  CodeParams p;
  NPRSResult r = params_or_error(nv, &p);
  if (r.tag != NPRS_RESULT_OK) return r;
  // src/erasure_coding.rs:291-312: chunks with index < k, all k required
  std::vector<const Chunk *> slot(p.k, nullptr);
  for (unsigned long i = 0; i < input->count; ++i) {
    const Chunk &ch = input->data[i];
    if (ch.index < p.k) slot[ch.index] = &ch;
  }
  for (uint32_t y = 0; y < p.k; ++y)
    if (!slot[y]) return result(NPRS_RESULT_NOT_ENOUGH_CHUNKS);
  // reed-solomon.hpp:155-165: first shard sets the length; empty -> error
  const unsigned long sl = slot[0]->data.array ? slot[0]->data.length : 0;
  if (sl / 2 == 0) return result(NPRS_RESULT_UNKNOWN_RECONSTRUCTION);  // kEmptyShard
  for (uint32_t y = 0; y < p.k; ++y) {
    const unsigned long l = slot[y]->data.array ? slot[y]->data.length : 0;
    if (l / 2 != sl / 2) return result(NPRS_RESULT_NON_UNIFORM_CHUNKS);
  }
  const size_t used = sl / 2 * 2;
  HostCtx *c = host_ctx();
  DeviceState *d = c ? device_state() : nullptr;
  const size_t in_bytes = size_t(p.k) * used, out_bytes = used * p.k;
  if (!c || !d || !ensure_host(&c->h_in, &c->h_in_cap, in_bytes) ||
      !ensure_host(&c->h_out, &c->h_out_cap, out_bytes) ||
      !ensure_dev(reinterpret_cast<void **>(&c->d_in), &c->d_in_cap, in_bytes) ||
      !ensure_dev(reinterpret_cast<void **>(&c->d_out), &c->d_out_cap, out_bytes))
    return result(NPRS_RESULT_UNKNOWN_RECONSTRUCTION);
  for (uint32_t y = 0; y < p.k; ++y) std::memcpy(c->h_in + y * used, slot[y]->data.array, used);
  CodeParams pk = p;
  pk.nv = p.k;  // staged layout holds only the k systematic shards
  if (!hip_check(hipMemcpyAsync(c->d_in, c->h_in, in_bytes, hipMemcpyHostToDevice, c->stream),
                 "H2D") ||
      !hip_check(launch_systematic(pk, c->d_in, used, used, 1, c->d_out, out_bytes, c->stream),
                 "systematic launch") ||
      !hip_check(hipMemcpyAsync(c->h_out, c->d_out, out_bytes, hipMemcpyDeviceToHost, c->stream),
                 "D2H") ||
      !hip_check(hipStreamSynchronize(c->stream), "systematic") ||
      !take_output(c, out_bytes, outdata))
    return result(NPRS_RESULT_UNKNOWN_RECONSTRUCTION);
  return result(NPRS_RESULT_OK);
}

NPRSResult ECCR_Test_MeasurePerformance(const DataBlock *message, unsigned long nv,
                                        unsigned long *us_enc, unsigned long *us_dec) {
  if (!message) return result(NPRS_RESULT_BAD_PAYLOAD);
  CodeParams p;
  NPRSResult r = params_or_error(nv, &p);
  if (r.tag != NPRS_RESULT_OK) return r;
  if (!message->array || message->length == 0) return result(NPRS_RESULT_BAD_PAYLOAD);
  HostCtx *c = host_ctx();
  if (!c) return result(NPRS_RESULT_UNKNOWN_CODE_PARAM);
  using clk = std::chrono::steady_clock;
  size_t sl = 0;
  {  // this thread's pinned staging and completion word for the call's size,
     // allocated before the clock starts (a first call otherwise timed the
     // hipHostMalloc), as the reference builds its encoders outside its timed
     // regions (src/erasure_coding.rs:190-207)
    const size_t pitch_bytes = size_t(nv) * dev_pitch(shard_len(p.k, message->length));
    if (!ensure_host(&c->h_out, &c->h_out_cap, pitch_bytes) ||
        !ensure_host(&c->h_in, &c->h_in_cap, std::max(pitch_bytes, size_t(message->length))))
      return result(NPRS_RESULT_UNKNOWN_CODE_PARAM);
    (void)call_signal(c);
  }
  const auto t0 = clk::now();
  if (!encode_host(p, message->array, message->length, c, &sl))
    return result(NPRS_RESULT_UNKNOWN_CODE_PARAM);
  const auto t1 = clk::now();
  // reconstruct from all shards (src/erasure_coding.rs:200-211)
  if (!ensure_host(&c->h_in, &c->h_in_cap, size_t(nv) * dev_pitch(sl)))
    return result(NPRS_RESULT_UNKNOWN_RECONSTRUCTION);
  std::memcpy(c->h_in, c->h_out, size_t(nv) * dev_pitch(sl));
  std::vector<uint8_t> present(p.n, 0);
  for (unsigned long v = 0; v < nv; ++v) present[v] = 1;
  const auto t2 = clk::now();
  if (!reconstruct_host(p, present, sl, c)) return result(NPRS_RESULT_UNKNOWN_RECONSTRUCTION);
  const auto t3 = clk::now();
  if (us_enc)
    *us_enc = (unsigned long)std::chrono::duration_cast<std::chrono::microseconds>(t1 - t0).count();
  if (us_dec)
    *us_dec = (unsigned long)std::chrono::duration_cast<std::chrono::microseconds>(t3 - t2).count();
  return result(NPRS_RESULT_OK);
}

// ------------------------------------------------------------- ec_amd.h --

NPRSResult ECCR_AMD_code_params(unsigned long nv, unsigned long *n, unsigned long *k,
                                unsigned long *thr) {
  CodeParams p;
  NPRSResult r = params_or_error(nv, &p);
  if (r.tag != NPRS_RESULT_OK) return r;
  if (n) *n = p.n;
  if (k) *k = p.k;
  if (thr) *thr = p.threshold;
  return r;
}

unsigned long ECCR_AMD_shard_len(unsigned long nv, unsigned long plen) {
  CodeParams p;
  if (code_params(nv, &p) != ParamError::kOk) return 0;
  return shard_len(p.k, plen);
}

int ECCR_AMD_device_count(void) {
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) return 0;
  return c;
}

NPRSResult ECCR_AMD_init_device(void) {
  return device_state() ? result(NPRS_RESULT_OK) : result(NPRS_RESULT_UNKNOWN_CODE_PARAM);
}

}  // extern "C"

namespace {
// Device scratch of one batch call: the caller's workspace (the *_ws entry
// points) or else the scratch private to the call's stream (stream_scratch).
// Either way, once the shape has run once on the stream, the call allocates,
// records and waits on nothing (capturable into a hipGraph), and calls on
// different streams never wait on each other.  `ok` false = too small /
// misaligned workspace or a failed allocation: nothing may be launched.
// Without a workspace the stream's scratch lease is held for the object's
// lifetime, i.e. until the call has enqueued all its kernels (ec_runtime.hpp).
struct BatchScratch {
  void *p = nullptr;
  bool ok = false;
  std::optional<StreamScratch> lease;
  BatchScratch(DeviceState *d, size_t need, hipStream_t s, const Workspace *ws) {
    if (need == 0) {
      ok = true;
    } else if (!ws) {
      lease.emplace(d, s, need);
      p = lease->ptr();
      ok = lease->ok();
    } else if (!ws->ptr || ws->bytes < need || reinterpret_cast<uintptr_t>(ws->ptr) % 256 != 0) {
      set_error("erasure_coding_crust(amd): workspace of " + std::to_string(ws->bytes) +
                " bytes (256-B aligned required) is below the " + std::to_string(need) +
                " bytes this shape needs (ECCR_AMD_*_workspace_bytes)");
    } else {
      ok = true;
      p = ws->ptr;
    }
  }
};

// batch > 1 deduplicates patterns only where a locator is expensive (n > 4096:
// the workgroup form); below, every row is computed by the wave form (ec_kernels)
size_t locator_scratch_bytes(const CodeParams &p, size_t batch) {
  return batch <= 1 || locator_wave_applicable(p.n) ? 0
                                                     : (batch * 4 + 255) / 256 * 256 + dedup_scratch_bytes(batch);
}

NPRSResult encode_batch(unsigned long nv, const uint8_t *d_payloads, unsigned long plen,
                        unsigned long pstride, unsigned long batch, uint8_t *d_shards,
                        unsigned long sstride, hipStream_t s, const Workspace *ws) {
  CodeParams p;
  NPRSResult r = params_or_error(nv, &p);
  if (r.tag != NPRS_RESULT_OK) return r;
  if (plen == 0) return result(NPRS_RESULT_BAD_PAYLOAD);
  if (sstride < shard_len(p.k, plen) || pstride < plen) return result(NPRS_RESULT_BAD_PAYLOAD);
  DeviceState *d = device_state();
  if (!d) return result(NPRS_RESULT_UNKNOWN_CODE_PARAM);
  // a workspace below the queried size (e.g. a size of 0 cached from an older
  // release) runs the shapes whose scratch is only a tile counter on the
  // static schedule: slower, not an error
  const bool optional = ws && (!ws->ptr || ws->bytes < encode_scratch_bytes(p, plen, batch)) &&
                        encode_scratch_optional(p);
  BatchScratch sc(d, optional ? 0 : encode_scratch_bytes(p, plen, batch), s, ws);
  if (!sc.ok) return result(NPRS_RESULT_UNKNOWN_CODE_PARAM);
  if (!hip_check(launch_encode(p, device_tables(d), d_payloads, plen, pstride, batch, d_shards,
                               sstride, sc.p, s),
                 "encode launch"))
    return result(NPRS_RESULT_UNKNOWN_CODE_PARAM);
  return result(NPRS_RESULT_OK);
}

NPRSResult error_locator(unsigned long nv, const uint8_t *d_present, unsigned long batch,
                         uint16_t *d_err_log, hipStream_t s, const Workspace *ws) {
  CodeParams p;
  NPRSResult r = params_or_error(nv, &p);
  if (r.tag != NPRS_RESULT_OK) return r;
  DeviceState *d = device_state();
  const uint16_t *fold = d ? device_fold(d, p.n) : nullptr;
  if (!fold) return result(NPRS_RESULT_UNKNOWN_RECONSTRUCTION);
  if (batch <= 1 || locator_wave_applicable(p.n)) {
    if (!hip_check(launch_error_locator(p, d_present, batch, fold, nullptr, d_err_log, s),
                   "error locator launch"))
      return result(NPRS_RESULT_UNKNOWN_RECONSTRUCTION);
    return result(NPRS_RESULT_OK);
  }
  // one locator per distinct pattern (§8f row 3), then copied to its followers
  if (batch >= (1ul << 31)) return result(NPRS_RESULT_BAD_PAYLOAD);  // uint32 pattern indices
  const size_t pat_bytes = (batch * 4 + 255) / 256 * 256;
  BatchScratch sc(d, locator_scratch_bytes(p, batch), s, ws);
  if (!sc.ok) return result(NPRS_RESULT_UNKNOWN_RECONSTRUCTION);
  uint32_t *pat = static_cast<uint32_t *>(sc.p);
  void *work = static_cast<uint8_t *>(sc.p) + pat_bytes;
  if (!hip_check(launch_dedup_patterns(p, d_present, batch, pat, work, s), "pattern dedup") ||
      !hip_check(launch_error_locator(p, d_present, batch, fold, pat, d_err_log, s),
                 "error locator launch") ||
      !hip_check(launch_broadcast_locators(p, pat, batch, d_err_log, s), "locator broadcast"))
    return result(NPRS_RESULT_UNKNOWN_RECONSTRUCTION);
  return result(NPRS_RESULT_OK);
}

NPRSResult reconstruct_batch(unsigned long nv, const uint8_t *d_shards, unsigned long slen,
                             unsigned long sstride, const uint8_t *d_present,
                             const uint16_t *d_err_log, const uint32_t *d_pattern,
                             unsigned long batch, uint8_t *d_out, unsigned long ostride,
                             hipStream_t s, const Workspace *ws) {
  CodeParams p;
  NPRSResult r = params_or_error(nv, &p);
  if (r.tag != NPRS_RESULT_OK) return r;
  if (slen % 2 != 0) return result(NPRS_RESULT_UNEVEN_LENGTH);
  if (sstride < slen || ostride < slen * p.k) return result(NPRS_RESULT_NON_UNIFORM_CHUNKS);
  DeviceState *d = device_state();
  if (!d) return result(NPRS_RESULT_UNKNOWN_RECONSTRUCTION);
  BatchScratch sc(d, reconstruct_scratch_bytes(p, slen, batch), s, ws);
  if (!sc.ok) return result(NPRS_RESULT_UNKNOWN_RECONSTRUCTION);
  if (!hip_check(launch_reconstruct(p, device_tables(d), d_shards, slen, sstride, d_present,
                                    d_err_log, d_pattern, batch, d_out, ostride, sc.p, s),
                 "reconstruct launch"))
    return result(NPRS_RESULT_UNKNOWN_RECONSTRUCTION);
  return result(NPRS_RESULT_OK);
}
}  // namespace

extern "C" {

NPRSResult ECCR_AMD_encode_batch(unsigned long nv, const uint8_t *d_payloads, unsigned long plen,
                                 unsigned long pstride, unsigned long batch, uint8_t *d_shards,
                                 unsigned long sstride, void *stream) {
  return encode_batch(nv, d_payloads, plen, pstride, batch, d_shards, sstride,
                      static_cast<hipStream_t>(stream), nullptr);
}

unsigned long ECCR_AMD_encode_workspace_bytes(unsigned long nv, unsigned long plen,
                                              unsigned long batch) {
  CodeParams p;
  if (code_params(nv, &p) != ParamError::kOk || plen == 0) return 0;
  return encode_scratch_bytes(p, plen, batch);
}

NPRSResult ECCR_AMD_encode_batch_ws(unsigned long nv, const uint8_t *d_payloads,
                                    unsigned long plen, unsigned long pstride, unsigned long batch,
                                    uint8_t *d_shards, unsigned long sstride, void *d_workspace,
                                    unsigned long workspace_bytes, void *stream) {
  const Workspace ws{d_workspace, workspace_bytes};
  return encode_batch(nv, d_payloads, plen, pstride, batch, d_shards, sstride,
                      static_cast<hipStream_t>(stream), &ws);
}

NPRSResult ECCR_AMD_error_locator(unsigned long nv, const uint8_t *d_present, unsigned long batch,
                                  uint16_t *d_err_log, void *stream) {
  return error_locator(nv, d_present, batch, d_err_log, static_cast<hipStream_t>(stream), nullptr);
}

unsigned long ECCR_AMD_error_locator_workspace_bytes(unsigned long nv, unsigned long batch) {
  CodeParams p;
  if (code_params(nv, &p) != ParamError::kOk) return 0;
  return locator_scratch_bytes(p, batch);
}

NPRSResult ECCR_AMD_error_locator_ws(unsigned long nv, const uint8_t *d_present,
                                     unsigned long batch, uint16_t *d_err_log, void *d_workspace,
                                     unsigned long workspace_bytes, void *stream) {
  const Workspace ws{d_workspace, workspace_bytes};
  return error_locator(nv, d_present, batch, d_err_log, static_cast<hipStream_t>(stream), &ws);
}

NPRSResult ECCR_AMD_dedup_patterns(unsigned long nv, const uint8_t *d_present, unsigned long batch,
                                   uint32_t *d_pattern, void *stream) {
  CodeParams p;
  NPRSResult r = params_or_error(nv, &p);
  if (r.tag != NPRS_RESULT_OK) return r;
  if (batch >= (1ul << 31)) return result(NPRS_RESULT_BAD_PAYLOAD);  // uint32 pattern indices
  DeviceState *d = device_state();
  if (!d) return result(NPRS_RESULT_UNKNOWN_RECONSTRUCTION);
  const hipStream_t s = static_cast<hipStream_t>(stream);
  BatchScratch sc(d, dedup_scratch_bytes(batch), s, nullptr);
  if (!sc.ok || !hip_check(launch_dedup_patterns(p, d_present, batch, d_pattern, sc.p, s), "pattern dedup"))
    return result(NPRS_RESULT_UNKNOWN_RECONSTRUCTION);
  return result(NPRS_RESULT_OK);
}

NPRSResult ECCR_AMD_error_locator_patterns(unsigned long nv, const uint8_t *d_present,
                                           const uint32_t *d_pattern, unsigned long batch,
                                           uint16_t *d_err_log, void *stream) {
  CodeParams p;
  NPRSResult r = params_or_error(nv, &p);
  if (r.tag != NPRS_RESULT_OK) return r;
  DeviceState *d = device_state();
  const uint16_t *fold = d ? device_fold(d, p.n) : nullptr;
  if (!fold) return result(NPRS_RESULT_UNKNOWN_RECONSTRUCTION);
  if (!hip_check(launch_error_locator(p, d_present, batch, fold, d_pattern, d_err_log,
                                      static_cast<hipStream_t>(stream)),
                 "error locator launch"))
    return result(NPRS_RESULT_UNKNOWN_RECONSTRUCTION);
  return result(NPRS_RESULT_OK);
}

NPRSResult ECCR_AMD_reconstruct_batch_patterns(unsigned long nv, const uint8_t *d_shards,
                                               unsigned long slen, unsigned long sstride,
                                               const uint8_t *d_present, const uint16_t *d_err_log,
                                               const uint32_t *d_pattern, unsigned long batch,
                                               uint8_t *d_out, unsigned long ostride, void *stream) {
  return reconstruct_batch(nv, d_shards, slen, sstride, d_present, d_err_log, d_pattern, batch,
                           d_out, ostride, static_cast<hipStream_t>(stream), nullptr);
}

unsigned long ECCR_AMD_reconstruct_workspace_bytes(unsigned long nv, unsigned long slen,
                                                   unsigned long batch) {
  CodeParams p;
  if (code_params(nv, &p) != ParamError::kOk) return 0;
  return reconstruct_scratch_bytes(p, slen, batch);
}

NPRSResult ECCR_AMD_reconstruct_batch_ws(unsigned long nv, const uint8_t *d_shards,
                                         unsigned long slen, unsigned long sstride,
                                         const uint8_t *d_present, const uint16_t *d_err_log,
                                         const uint32_t *d_pattern, unsigned long batch,
                                         uint8_t *d_out, unsigned long ostride, void *d_workspace,
                                         unsigned long workspace_bytes, void *stream) {
  const Workspace ws{d_workspace, workspace_bytes};
  return reconstruct_batch(nv, d_shards, slen, sstride, d_present, d_err_log, d_pattern, batch,
                           d_out, ostride, static_cast<hipStream_t>(stream), &ws);
}

NPRSResult ECCR_AMD_reconstruct_batch(unsigned long nv, const uint8_t *d_shards,
                                      unsigned long slen, unsigned long sstride,
                                      const uint8_t *d_present, const uint16_t *d_err_log,
                                      unsigned long batch, uint8_t *d_out,
                                      unsigned long ostride, void *stream) {
  return ECCR_AMD_reconstruct_batch_patterns(nv, d_shards, slen, sstride, d_present, d_err_log,
                                             nullptr, batch, d_out, ostride, stream);
}

NPRSResult ECCR_AMD_locator_cache_stats(unsigned long *hits, unsigned long *misses) {
  DeviceState *d = device_state();
  if (!d) return result(NPRS_RESULT_UNKNOWN_RECONSTRUCTION);
  locator_cache_stats(d, hits, misses);
  return result(NPRS_RESULT_OK);
}

NPRSResult ECCR_AMD_systematic_batch(unsigned long nv, const uint8_t *d_shards, unsigned long slen,
                                     unsigned long sstride, unsigned long batch, uint8_t *d_out,
                                     unsigned long ostride, void *stream) {
  CodeParams p;
  NPRSResult r = params_or_error(nv, &p);
  if (r.tag != NPRS_RESULT_OK) return r;
  if (sstride < slen || ostride < slen / 2 * 2 * p.k) return result(NPRS_RESULT_NON_UNIFORM_CHUNKS);
  if (!device_state()) return result(NPRS_RESULT_UNKNOWN_RECONSTRUCTION);
  if (!hip_check(launch_systematic(p, d_shards, slen / 2 * 2, sstride, batch, d_out, ostride,
                                   static_cast<hipStream_t>(stream)),
                 "systematic launch"))
    return result(NPRS_RESULT_UNKNOWN_RECONSTRUCTION);
  return result(NPRS_RESULT_OK);
}

void ECCR_AMD_set_scratch_limit(unsigned long bytes) { set_scratch_limit(bytes); }

int ECCR_AMD_release_stream_scratch(void *stream) {
  DeviceState *d = device_state();
  return d && release_stream_scratch(d, static_cast<hipStream_t>(stream)) ? 1 : 0;
}

const char *ECCR_AMD_last_error(void) { return last_error(); }

}  // extern "C"
