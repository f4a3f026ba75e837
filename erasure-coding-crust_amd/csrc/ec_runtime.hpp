// ec_runtime.hpp — per-device table residency and per-thread host contexts.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "ec_kernels.hpp"
#include "gf_field.hpp"

namespace ecamd {

// Device-resident skews + multiply tables for the current HIP device,
// uploaded once per device (6.4 MB).  Returns nullptr (and sets the thread's
// last error) if no usable device exists.
struct DeviceState;
DeviceState *device_state();
DevTables device_tables(DeviceState *d);
const uint16_t *device_fold(DeviceState *d, uint32_t n);  // folded LOG_WALSH for n
// Per-device scratch of the per-call C ABI (gather orders, the k = 1024
// encode's coefficient slots, generic kernels beyond LDS).  A lease is held
// while a call's launches are enqueued: it orders the caller's stream
// after the previous lease's work (an event), so launches from different
// streams or host threads never overlap on the buffer.
// Upper bound on one scratch allocation (0 = none): a larger request fails
// like an out-of-memory hipMalloc (ECCR_AMD_set_scratch_limit).
void set_scratch_limit(size_t bytes);
class ScratchLease {
 public:
  ScratchLease(DeviceState *d, size_t bytes, hipStream_t stream);
  ~ScratchLease();  // records the release event on the stream
  ScratchLease(const ScratchLease &) = delete;
  ScratchLease &operator=(const ScratchLease &) = delete;
  void *ptr() const { return p_; }
  // false if scratch was needed and could not be allocated (the caller must
  // not launch: the kernels would run on a null buffer)
  bool ok() const { return want_ == 0 || p_ != nullptr; }

 private:
  DeviceState *d_ = nullptr;
  hipStream_t s_ = nullptr;
  size_t want_ = 0;
  void *p_ = nullptr;
  bool held_ = false;
};

// Scratch private to one (device, stream), for the batch calls made without a
// caller workspace.  A StreamScratch is a lease: it holds the entry's mutex
// from the moment the buffer is handed out until the caller has enqueued every
// kernel that uses it (the object's lifetime), so two host threads issuing on
// the same stream (e.g. the shared default stream) run their kernel sequences
// one after the other on it, never interleaved on one buffer.  The buffer grows
// on the first call of a larger shape on that stream, after synchronising the
// stream (every earlier holder has finished enqueueing by then).  Otherwise a
// call allocates, records and waits on nothing, so it can be captured into a
// hipGraph, and calls on different streams never wait on each other.  At most
// kStreamScratch streams per device keep a buffer; beyond that the least
// recently used entry is evicted to a deferred list.  A lease's destructor
// never frees or synchronises (it may run inside a graph capture); evicted
// buffers nobody holds are freed after a hipDeviceSynchronize at the start of
// a later lease on a stream that is not being captured, or by
// ECCR_AMD_release_stream_scratch (the stream handle of an evicted entry may
// be dangling, so the whole device is waited for: rare, but it does wait on
// every stream).  ECCR_AMD_release_stream_scratch releases one stream's
// buffer explicitly.
// ok() false (error set) if the allocation failed or exceeds the scratch limit.
constexpr size_t kStreamScratch = 64;
struct StreamScratchEntry;
class StreamScratch {
 public:
  StreamScratch(DeviceState *d, hipStream_t s, size_t bytes);
  ~StreamScratch();
  StreamScratch(const StreamScratch &) = delete;
  StreamScratch &operator=(const StreamScratch &) = delete;
  void *ptr() const { return p_; }
  bool ok() const { return want_ == 0 || p_ != nullptr; }

 private:
  std::shared_ptr<StreamScratchEntry> e_;  // declared first: released after the lock
  bool locked_ = false;
  size_t want_ = 0;
  void *p_ = nullptr;
};
// Frees the scratch kept for stream s on the current device (after
// synchronising s).  False if none was kept.
bool release_stream_scratch(DeviceState *d, hipStream_t s);

// Per-pattern erasure-locator cache of the per-call C ABI (SURVEY.md §8f
// row 3): the locator of a pattern (n_validators + present bitmap) is computed
// once per device and reused while it is among the most recent kLocatorCache
// patterns (the common case: the same validators missing for every block).
constexpr size_t kLocatorCache = 64;
struct Locator {
  uint32_t nv = 0;
  uint32_t cap_n = 0;            // n the device buffers were sized for (recycled on eviction)
  std::vector<uint8_t> present;  // the key: [n] flags
  uint8_t *d_present = nullptr;  // [n] on the device
  uint16_t *d_elog = nullptr;    // [n] log-domain multipliers (ECCR_AMD_error_locator)
  hipEvent_t ready = nullptr;    // recorded after the locator kernel, on the creating call's stream
  mutable bool done = false;     // that kernel is known complete (under the cache lock)
  ~Locator();                    // frees (never under the cache lock)
};
// The pattern's locator, computed on `stream` on a miss; on a hit `stream`
// is ordered after the kernel that computed it.  nullptr on a HIP error.
// Every holder synchronises its stream before dropping the pointer, and the
// creating call then marks the entry done (locator_done), so an entry nobody
// holds is idle: a miss recycles its buffers instead of freeing and
// allocating.  `ready` is used only while the entry is not done, i.e. while
// the creating call (and so its thread's stream) is still alive: an event
// whose recording stream was destroyed with its thread is never synchronised
// on (HIP then read the stale stream: "operation not permitted on an event
// last recorded in a capturing stream", round 5).
std::shared_ptr<const Locator> cached_locator(DeviceState *d, const CodeParams &p,
                                              const std::vector<uint8_t> &present,
                                              hipStream_t stream);
// The creating (or any) call's stream has finished everything issued after
// the entry's locator kernel: later hits need no event wait.
void locator_done(DeviceState *d, const Locator &L);
// The call that holds the entry failed to synchronise its stream (the locator
// kernel may have faulted): the entry leaves the cache; its last holder frees it.
void locator_drop(DeviceState *d, const Locator &L);
void locator_cache_stats(DeviceState *d, unsigned long *hits, unsigned long *misses);

// Growable buffers of one host thread (reentrancy = the reference's
// thread_local scratch, reed-solomon.hpp:198-201).
struct HostCtx {
  HostCtx() = default;
  HostCtx(const HostCtx &) = delete;
  HostCtx &operator=(const HostCtx &) = delete;
  ~HostCtx();  // synchronises and releases the stream and every buffer
  hipStream_t stream = nullptr;
  uint8_t *h_in = nullptr, *h_out = nullptr;  // pinned
  size_t h_in_cap = 0, h_out_cap = 0;
  uint8_t *d_in = nullptr, *d_out = nullptr, *d_present = nullptr;
  uint16_t *d_elog = nullptr;
  size_t d_in_cap = 0, d_out_cap = 0, d_present_cap = 0, d_elog_cap = 0;
  int device = -1;
  uint32_t *h_flag = nullptr;  // pinned completion word (finish_call)
  uint32_t seq = 0;
};
HostCtx *host_ctx();  // nullptr if no device
// Waits until the KERNELS enqueued on c->stream are done (the small direct
// calls, which run on pinned staging and issue no copy): a signal kernel stores a
// sequence number to the context's pinned word and the host spins on it for up
// to kFinishSpinUs, then falls back to hipStreamSynchronize (which also
// reports an asynchronous error).  False (error set) on a HIP error.
// Every kFinishProbeEvery-th spin-completed call also queries the stream, so
// an asynchronous kernel error is reported within that many calls.  (A kernel
// that faults never stores the word, so its call times out of the spin into
// hipStreamSynchronize and reports the error itself; the probe is for the
// rest.  A hipStreamQuery costs ~10 us, so every 16th call, as until round 5,
// put 12-20 us outliers into the per-call times: scripts/micro/mp_calls.cpp,
// encode 844-899 -> 761-804 us per 100 calls at 1024.)
// sig: the completion word and sequence number of the call (call_signal),
// offered to the call's last kernel launch first: if that kernel stored it
// itself (HostSig::fused, a single-workgroup launch), no signal kernel is
// launched.
constexpr double kFinishSpinUs = 200.0;
#ifndef ECCR_PROBE_EVERY
#define ECCR_PROBE_EVERY 1024
#endif
constexpr uint32_t kFinishProbeEvery = ECCR_PROBE_EVERY;
bool finish_call(HostCtx *c, const char *what, const HostSig *sig = nullptr);
// the next completion word / value of this context (flag null if the pinned
// word could not be allocated: finish_call then synchronises the stream)
HostSig call_signal(HostCtx *c);
bool ensure_host(uint8_t **p, size_t *cap, size_t need);
bool ensure_dev(void **p, size_t *cap, size_t need);

void set_error(const std::string &msg);  // also printed to stderr
const char *last_error();

}  // namespace ecamd
