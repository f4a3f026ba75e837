// ec_runtime.cpp — device table residency, scratch, per-thread contexts.
#include "ec_runtime.hpp"

#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

namespace ecamd {

struct DeviceState {
  int id = -1;
  uint16_t *skews = nullptr;
  MulTab *mtab = nullptr;
  uint8_t *timg = nullptr;
  std::mutex mu;
  std::map<uint32_t, uint16_t *> fold;
  std::mutex scratch_mu;  // held by a ScratchLease
  void *scratch = nullptr;
  size_t scratch_cap = 0;
  hipEvent_t scratch_done = nullptr;  // the last lease's work on its stream
  bool scratch_used = false;
};

namespace {
thread_local std::string t_err;
std::mutex g_mu;
std::vector<std::unique_ptr<DeviceState>> g_dev;

bool hip_ok(hipError_t e, const char *what) {
  if (e == hipSuccess) return true;
  set_error(std::string("erasure_coding_crust(amd): ") + what + ": " + hipGetErrorString(e));
  return false;
}
}  // namespace

void set_error(const std::string &msg) {
  t_err = msg;
  std::fprintf(stderr, "%s\n", msg.c_str());
}
const char *last_error() { return t_err.c_str(); }

DeviceState *device_state() {
  int dev = -1, count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
    set_error("erasure_coding_crust(amd): no HIP device available (the HIP path is required; "
              "there is no CPU fallback)");
    return nullptr;
  }
  if (!hip_ok(hipGetDevice(&dev), "hipGetDevice")) return nullptr;
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_dev.size() < size_t(count)) g_dev.resize(count);
  auto &slot = g_dev[dev];
  if (slot) return slot.get();
  const Field &f = field();
  auto st = std::make_unique<DeviceState>();
  st->id = dev;
  if (!hip_ok(hipMalloc(&st->skews, f.skews.size() * 2), "hipMalloc(skews)")) return nullptr;
  if (!hip_ok(hipMalloc(&st->mtab, f.mtab.size() * sizeof(MulTab)), "hipMalloc(mtab)"))
    return nullptr;
  if (!hip_ok(hipMemcpy(st->skews, f.skews.data(), f.skews.size() * 2, hipMemcpyHostToDevice),
              "upload skews") ||
      !hip_ok(hipMemcpy(st->mtab, f.mtab.data(), f.mtab.size() * sizeof(MulTab),
                        hipMemcpyHostToDevice),
              "upload mtab"))
    return nullptr;
  // LDS table images (ec_kernels.hpp kTabImages): LdsTabs<1024>::addr layout
  std::vector<uint8_t> img(kTabImages * kTabImageBytes, 0);
  for (int q = 0; q < kTabImages; ++q)
    for (uint32_t i = 0; i < 1023; ++i) {
      const uint8_t *src = reinterpret_cast<const uint8_t *>(&f.mtab[f.skews[1024 * q + i]]);
      const uint32_t sw = (i ^ (i >> 4) ^ (i >> 8)) & 15;
      for (uint32_t plane = 0; plane < 5; ++plane)
        std::memcpy(&img[q * kTabImageBytes + plane * 16384 + ((i >> 4) << 8) + (sw << 4)],
                    src + 16 * plane, 16);
    }
  if (!hip_ok(hipMalloc(&st->timg, img.size()), "hipMalloc(table images)") ||
      !hip_ok(hipMemcpy(st->timg, img.data(), img.size(), hipMemcpyHostToDevice),
              "upload table images"))
    return nullptr;
  slot = std::move(st);
  return slot.get();
}

DevTables device_tables(DeviceState *d) {
  DevTables t;
  t.skews = d->skews;
  t.mtab = d->mtab;
  t.timg = d->timg;
  return t;
}

const uint16_t *device_fold(DeviceState *d, uint32_t n) {
  std::lock_guard<std::mutex> lk(d->mu);
  auto it = d->fold.find(n);
  if (it != d->fold.end()) return it->second;
  std::vector<uint16_t> F = field().fold_log_walsh(n);
  uint16_t *p = nullptr;
  if (!hip_ok(hipMalloc(&p, n * 2), "hipMalloc(fold)")) return nullptr;
  if (!hip_ok(hipMemcpy(p, F.data(), n * 2, hipMemcpyHostToDevice), "upload fold")) return nullptr;
  d->fold[n] = p;
  return p;
}

ScratchLease::ScratchLease(DeviceState *d, size_t bytes, hipStream_t stream)
    : d_(d), s_(stream) {
  if (!d || bytes == 0) return;
  d->scratch_mu.lock();
  held_ = true;
  if (d->scratch_cap < bytes) {
    if (d->scratch) {
      if (d->scratch_used) (void)hipEventSynchronize(d->scratch_done);
      (void)hipFree(d->scratch);
    }
    d->scratch = nullptr;
    d->scratch_cap = 0;
    if (!hip_ok(hipMalloc(&d->scratch, bytes), "hipMalloc(scratch)")) return;
    d->scratch_cap = bytes;
  } else if (d->scratch_used) {
    (void)hipStreamWaitEvent(stream, d->scratch_done, 0);
  }
  p_ = d->scratch;
}

ScratchLease::~ScratchLease() {
  if (!held_) return;
  if (!d_->scratch_done) (void)hipEventCreateWithFlags(&d_->scratch_done, hipEventDisableTiming);
  d_->scratch_used = d_->scratch_done && hipEventRecord(d_->scratch_done, s_) == hipSuccess;
  d_->scratch_mu.unlock();
}

bool ensure_host(uint8_t **p, size_t *cap, size_t need) {
  if (*cap >= need && *p) return true;
  if (*p) (void)hipHostFree(*p);
  *p = nullptr;
  *cap = 0;
  size_t sz = need < 4096 ? 4096 : need + need / 4;
  if (!hip_ok(hipHostMalloc(reinterpret_cast<void **>(p), sz, hipHostMallocDefault),
              "hipHostMalloc"))
    return false;
  *cap = sz;
  return true;
}

bool ensure_dev(void **p, size_t *cap, size_t need) {
  if (*cap >= need && *p) return true;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  size_t sz = need < 4096 ? 4096 : need + need / 4;
  if (!hip_ok(hipMalloc(p, sz), "hipMalloc")) return false;
  *cap = sz;
  return true;
}

HostCtx *host_ctx() {
  thread_local std::unique_ptr<HostCtx> ctx;
  DeviceState *d = device_state();
  if (!d) return nullptr;
  if (ctx && ctx->device == d->id) return ctx.get();
  ctx = std::make_unique<HostCtx>();
  ctx->device = d->id;
  if (!hip_ok(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking), "hipStreamCreate")) {
    ctx.reset();
    return nullptr;
  }
  return ctx.get();
}

}  // namespace ecamd
