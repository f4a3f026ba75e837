// ec_runtime.hpp — per-device table residency and per-thread host contexts.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <string>

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
// Per-device scratch for the launches that need one (the k = 1024 encode's
// coefficients between its four launches, generic kernels beyond LDS).  A
// lease is held while a launch is enqueued: it orders the caller's stream
// after the previous lease's work (an event), so launches from different
// streams or host threads never overlap on the buffer.
class ScratchLease {
 public:
  ScratchLease(DeviceState *d, size_t bytes, hipStream_t stream);
  ~ScratchLease();  // records the release event on the stream
  ScratchLease(const ScratchLease &) = delete;
  ScratchLease &operator=(const ScratchLease &) = delete;
  void *ptr() const { return p_; }

 private:
  DeviceState *d_ = nullptr;
  hipStream_t s_ = nullptr;
  void *p_ = nullptr;
  bool held_ = false;
};

// Growable buffers of one host thread (reentrancy = the reference's
// thread_local scratch, reed-solomon.hpp:198-201).
struct HostCtx {
  hipStream_t stream = nullptr;
  uint8_t *h_in = nullptr, *h_out = nullptr;  // pinned
  size_t h_in_cap = 0, h_out_cap = 0;
  uint8_t *d_in = nullptr, *d_out = nullptr, *d_present = nullptr;
  uint16_t *d_elog = nullptr;
  size_t d_in_cap = 0, d_out_cap = 0, d_present_cap = 0, d_elog_cap = 0;
  int device = -1;
};
HostCtx *host_ctx();  // nullptr if no device
bool ensure_host(uint8_t **p, size_t *cap, size_t need);
bool ensure_dev(void **p, size_t *cap, size_t need);

void set_error(const std::string &msg);  // also printed to stderr
const char *last_error();

}  // namespace ecamd
