// ec_runtime.cpp — device table residency, scratch, per-thread contexts.
#include "ec_runtime.hpp"

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <list>
#include <map>
#include <memory>
#include <mutex>
#include <utility>
#include <vector>

namespace ecamd {

struct DeviceState {
  int id = -1;
  uint16_t *skews = nullptr;
  MulTab *mtab = nullptr;
  uint8_t *timg = nullptr;
  MulTab *mtab_t = nullptr;  // mtab_tin, then mtab_tout
  uint8_t *timg_t = nullptr;
  uint8_t *timg_f9 = nullptr;
  uint8_t *cimg = nullptr;
  uint8_t *eimg512 = nullptr;
  uint8_t *eimg256 = nullptr;
  MulTab *mslot = nullptr;  // mtab by skew slot (DevTables::mslot)
  std::mutex mu;
  std::map<uint32_t, uint16_t *> fold;
  std::mutex scratch_mu;  // held by a ScratchLease
  void *scratch = nullptr;
  size_t scratch_cap = 0;
  hipEvent_t scratch_done = nullptr;  // the last lease's work on its stream
  hipStream_t scratch_stream = nullptr;  // that stream (a HostCtx's)
  bool scratch_used = false;
  std::mutex loc_mu;
  std::list<std::shared_ptr<Locator>> loc;  // most recent first
  unsigned long loc_hits = 0, loc_misses = 0;
  std::mutex ss_mu;
  std::list<std::shared_ptr<StreamScratchEntry>> ss;  // per-stream scratch, most recent first
  std::list<std::shared_ptr<StreamScratchEntry>> ss_dead;  // evicted, freed by drain_dead()
};

// One stream's scratch buffer.  `mu` is held by a StreamScratch lease while
// its caller enqueues.  An evicted entry is never freed by a lease's
// destructor (that could be inside another thread's graph capture, ADVICE
// r04): it waits in DeviceState::ss_dead for drain_dead() (see ec_runtime.hpp).
struct StreamScratchEntry {
  hipStream_t s = nullptr;
  void *p = nullptr;
  size_t cap = 0;
  std::mutex mu;
};

namespace {
thread_local std::string t_err;
std::mutex g_mu;
// never destroyed: its entries own HIP objects, and HIP calls from static
// destructors at process exit can crash or hang; process teardown reclaims them
std::vector<std::unique_ptr<DeviceState>> &g_dev = *new std::vector<std::unique_ptr<DeviceState>>();

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
  // this thread's last device, if still current: no device count, no lock
  // (the per-call C ABI asks this two or three times per call)
  thread_local DeviceState *t_last = nullptr;
  if (t_last && hipGetDevice(&dev) == hipSuccess && dev == t_last->id) return t_last;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
    set_error("erasure_coding_crust(amd): no HIP device available (the HIP path is required; "
              "there is no CPU fallback)");
    return nullptr;
  }
  if (!hip_ok(hipGetDevice(&dev), "hipGetDevice")) return nullptr;
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_dev.size() < size_t(count)) g_dev.resize(count);
  auto &slot = g_dev[dev];
  if (slot) return t_last = slot.get();
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
  // LDS table images (ec_kernels.hpp kTabImages): LdsTabs<1024>::addr layout;
  // img_t: the tower images (subfield tables at stages >= tower_sub_min(q))
  std::vector<uint8_t> img(kTabImages * kTabImageBytes, 0), img_t(kTabImages * kTabImageBytes, 0);
  for (int q = 0; q < kTabImages; ++q)
    for (uint32_t i = 0; i < 1023; ++i) {
      const uint32_t c = f.skews[1024 * q + i];
      const uint8_t *src = reinterpret_cast<const uint8_t *>(&f.mtab[c]);
      const uint32_t sw = (i ^ (i >> 4) ^ (i >> 8)) & 15;
      const size_t slot = size_t(q) * kTabImageBytes + ((i >> 4) << 8) + (sw << 4);
      for (uint32_t plane = 0; plane < 5; ++plane) std::memcpy(&img[slot + plane * 16384], src + 16 * plane, 16);
      if (__builtin_ctz(1024 * q + i + 1) >= tower_sub_min(q)) {
        const MulTabSub u = f.sub_tab(c);
        std::memcpy(&img_t[slot], &u.w[0], 16);
        std::memcpy(&img_t[slot + 16384], &u.w[4], 4);
      } else {
        const MulTab g = f.tower_tab(c);
        for (uint32_t plane = 0; plane < 5; ++plane)
          std::memcpy(&img_t[slot + plane * 16384], reinterpret_cast<const uint8_t *>(&g) + 16 * plane, 16);
      }
    }
  std::vector<uint8_t> img_f9(kF9Images * kTabImageBytes, 0);
  for (int kind = 0; kind < kF9Images; ++kind) {
    std::memcpy(&img_f9[size_t(kind) * kTabImageBytes], img_t.data(), kTabImageBytes);
    for (uint32_t i = 0; i < 1023; ++i) {
      if (!f9_slot(kind, i)) continue;
      MulTabF9 t9;
      if (!f.f9_tab(f.skews[i], &t9)) return nullptr;  // (tower_check: never)
      const uint32_t sw = (i ^ (i >> 4) ^ (i >> 8)) & 15;
      const size_t slot = size_t(kind) * kTabImageBytes + ((i >> 4) << 8) + (sw << 4);
      for (uint32_t plane = 0; plane < 4; ++plane)
        std::memcpy(&img_f9[slot + plane * 16384], &t9.w[4 * plane], 16);
    }
  }
  // the element-indexed compact image (ec_kernels.hpp): entry x = element 2 x
  std::vector<uint8_t> cimg(kCImgBytes, 0);
  for (uint32_t x = 0; x < 512; ++x) {
    const uint32_t e = 2 * x, c = e == 0 ? kZeroTab : f.log[e];
    if (x < 128) {
      const MulTabSub u = f.sub_tab(c);
      std::memcpy(&cimg[kCImgSub0 | cimg_lin(x)], &u.w[0], 16);
      std::memcpy(&cimg[kCImgSub1 | cimg_lin(x)], &u.w[4], 4);
    } else if (x < 256) {
      MulTabF9 t9;
      if (!f.f9_tab(c, &t9)) return nullptr;  // (tower(e) >> 8 == 1 for 256 <= e < 512)
      for (uint32_t q = 0; q < 4; ++q)
        std::memcpy(&cimg[(kCImgF9 + q * kCImgF9Plane) | cimg_lin(x ^ 128)], &t9.w[4 * q], 16);
    } else {
      const MulTab g = f.tower_tab(c);
      for (uint32_t q = 0; q < 5; ++q)
        std::memcpy(&cimg[(kCImgGen + q * kCImgGenPlane) | cimg_lin(x ^ 256)], &g.w[4 * q], 16);
    }
  }
  if (!hip_ok(hipMalloc(&st->cimg, cimg.size()), "hipMalloc(compact image)") ||
      !hip_ok(hipMemcpy(st->cimg, cimg.data(), cimg.size(), hipMemcpyHostToDevice),
              "upload compact image"))
    return nullptr;
  // the k = 512 encode's per-coset extension images (ec_kernels.hpp kEImg512*):
  // general tower tables of the elements x = (512 j >> (m + 1)) + e
  std::vector<uint8_t> eimg(kEImg512Cosets * kEImg512Bytes, 0);
  for (uint32_t j = 1; j <= kEImg512Cosets; ++j)
    for (uint32_t m = 0; m < 3; ++m)
      for (uint32_t e = 0; e < (256u >> m); ++e) {
        const uint32_t x = ((512 * j) >> (m + 1)) + e;
        const MulTab g = f.tower_tab(f.log[2 * x]);
        for (uint32_t q = 0; q < 5; ++q)
          std::memcpy(&eimg[(j - 1) * kEImg512Bytes + kEImg512Stage[m] + q * (4096 >> m) + cimg_lin(e)],
                      &g.w[4 * q], 16);
      }
  std::vector<uint8_t> eimg256(kEImg256Cosets * kEImg256Bytes, 0);
  for (uint32_t j = 4; j < 4 + kEImg256Cosets; ++j)
    for (uint32_t e = 0; e < 128; ++e) {
      const MulTab g = f.tower_tab(f.log[2 * (128 * j + e)]);
      for (uint32_t q = 0; q < 5; ++q)
        std::memcpy(&eimg256[(j - 4) * kEImg256Bytes + q * 2048 + cimg_lin(e)], &g.w[4 * q], 16);
    }
  if (!hip_ok(hipMalloc(&st->eimg256, eimg256.size()), "hipMalloc(k256 coset images)") ||
      !hip_ok(hipMemcpy(st->eimg256, eimg256.data(), eimg256.size(), hipMemcpyHostToDevice),
              "upload k256 coset images"))
    return nullptr;
  if (!hip_ok(hipMalloc(&st->eimg512, eimg.size()), "hipMalloc(k512 coset images)") ||
      !hip_ok(hipMemcpy(st->eimg512, eimg.data(), eimg.size(), hipMemcpyHostToDevice),
              "upload k512 coset images"))
    return nullptr;
  if (!hip_ok(hipMalloc(&st->timg_f9, img_f9.size()), "hipMalloc(F9 images)") ||
      !hip_ok(hipMemcpy(st->timg_f9, img_f9.data(), img_f9.size(), hipMemcpyHostToDevice),
              "upload F9 images"))
    return nullptr;
  if (!hip_ok(hipMalloc(&st->timg, img.size()), "hipMalloc(table images)") ||
      !hip_ok(hipMemcpy(st->timg, img.data(), img.size(), hipMemcpyHostToDevice),
              "upload table images") ||
      !hip_ok(hipMalloc(&st->timg_t, img_t.size()), "hipMalloc(tower images)") ||
      !hip_ok(hipMemcpy(st->timg_t, img_t.data(), img_t.size(), hipMemcpyHostToDevice),
              "upload tower images"))
    return nullptr;
  {  // the multiply tables by skew slot (the generic kernels: one load per table)
    std::vector<MulTab> ms(f.skews.size());
    for (size_t i = 0; i < ms.size(); ++i) ms[i] = f.mtab[f.skews[i]];
    if (!hip_ok(hipMalloc(&st->mslot, ms.size() * sizeof(MulTab)), "hipMalloc(mslot)") ||
        !hip_ok(hipMemcpy(st->mslot, ms.data(), ms.size() * sizeof(MulTab), hipMemcpyHostToDevice),
                "upload mslot"))
      return nullptr;
  }
  if (!hip_ok(hipMalloc(&st->mtab_t, 2 * f.mtab.size() * sizeof(MulTab)), "hipMalloc(tower mtab)") ||
      !hip_ok(hipMemcpy(st->mtab_t, f.mtab_tin.data(), f.mtab_tin.size() * sizeof(MulTab),
                        hipMemcpyHostToDevice),
              "upload mtab_tin") ||
      !hip_ok(hipMemcpy(st->mtab_t + f.mtab.size(), f.mtab_tout.data(),
                        f.mtab_tout.size() * sizeof(MulTab), hipMemcpyHostToDevice),
              "upload mtab_tout"))
    return nullptr;
  // load the library's code object now (the first kernel launch of a process
  // loads it, ~1 ms): one one-lane launch, so no C-ABI call's timed region
  // (ECCR_Test_MeasurePerformance starts its clock after this) pays it
  uint32_t *warm = nullptr;
  if (hipMalloc(&warm, 64) == hipSuccess) {
    if (launch_signal_host(warm, 1, nullptr) == hipSuccess && warm_encode_tiny(nullptr) == hipSuccess)
      (void)hipDeviceSynchronize();
    (void)hipFree(warm);
  }
  slot = std::move(st);
  return t_last = slot.get();
}

DevTables device_tables(DeviceState *d) {
  DevTables t;
  t.skews = d->skews;
  t.mtab = d->mtab;
  t.timg = d->timg;
  t.mtab_tin = d->mtab_t;
  t.mtab_tout = d->mtab_t + kFieldSize;
  t.timg_t = d->timg_t;
  t.timg_f9 = d->timg_f9;
  t.cimg = d->cimg;
  t.mslot = d->mslot;
  t.eimg512 = d->eimg512;
  t.eimg256 = d->eimg256;
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

hipError_t prepare_kernel(const void *fn, int lds_bytes, int *cus) {
  static std::mutex mu;
  static std::map<std::pair<int, const void *>, bool> prepared;
  static std::map<int, int> cu_count;
  int dev = 0;
  if (const hipError_t e = hipGetDevice(&dev); e != hipSuccess) return e;
  std::lock_guard<std::mutex> lk(mu);
  auto c = cu_count.find(dev);
  if (c == cu_count.end()) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    c = cu_count.emplace(dev, n).first;
  }
  bool &done = prepared[{dev, fn}];
  if (!done && lds_bytes >= 65536) {
    // these kernels address their multiply tables by absolute LDS address,
    // assuming their dynamic LDS starts at 0, i.e. no static LDS (lds_tab_at)
    hipFuncAttributes attr{};
    if (const hipError_t e = hipFuncGetAttributes(&attr, fn); e != hipSuccess) return e;
    if (attr.sharedSizeBytes != 0) return hipErrorInvalidKernelFile;
    if (lds_bytes > 65536) {
      const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes);
      if (e != hipSuccess) return e;
    }
  }
  done = true;
  *cus = c->second;
  return hipSuccess;
}

namespace {
std::atomic<size_t> g_scratch_limit{0};  // 0 = no limit (ECCR_AMD_set_scratch_limit)
}

void set_scratch_limit(size_t bytes) { g_scratch_limit = bytes; }

ScratchLease::ScratchLease(DeviceState *d, size_t bytes, hipStream_t stream)
    : d_(d), s_(stream), want_(bytes) {
  if (!d || bytes == 0) return;
  const size_t limit = g_scratch_limit;
  if (limit && bytes > limit) {  // as if hipMalloc had failed
    set_error("erasure_coding_crust(amd): scratch of " + std::to_string(bytes) +
              " bytes exceeds the limit set by ECCR_AMD_set_scratch_limit");
    return;
  }
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
  d_->scratch_stream = s_;
  d_->scratch_mu.unlock();
}

namespace {
// A HostCtx's stream, synchronised, is about to be destroyed: the scratch
// event recorded on it is complete and must not be waited on any more (HIP
// would consult the destroyed stream).  Locator events need nothing: their
// creating call marks them done before it returns (locator_done).
void forget_stream(int dev, hipStream_t s) {
  DeviceState *d = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (dev >= 0 && size_t(dev) < g_dev.size()) d = g_dev[dev].get();
  }
  if (!d) return;
  std::lock_guard<std::mutex> lk(d->scratch_mu);
  if (d->scratch_stream == s) {
    d->scratch_used = false;
    d->scratch_stream = nullptr;
  }
}
}  // namespace

Locator::~Locator() {
  // idle: every holder synchronised its stream before dropping it
  if (ready) (void)hipEventDestroy(ready);
  if (d_present) (void)hipFree(d_present);
  if (d_elog) (void)hipFree(d_elog);
}

std::shared_ptr<const Locator> cached_locator(DeviceState *d, const CodeParams &p,
                                              const std::vector<uint8_t> &present,
                                              hipStream_t stream) {
  // declared first, so destroyed last: an evicted entry still held elsewhere
  // is freed by its last holder, never here under loc_mu
  std::shared_ptr<Locator> evicted;
  std::shared_ptr<Locator> L;
  {
    std::lock_guard<std::mutex> lk(d->loc_mu);
    for (auto it = d->loc.begin(); it != d->loc.end(); ++it)
      if ((*it)->nv == p.nv && (*it)->present == present) {
        std::shared_ptr<Locator> hit = *it;
        d->loc.erase(it);
        d->loc.push_front(hit);
        ++d->loc_hits;
        // not done: the creating call is still in flight (it marks the entry
        // under this lock before returning), so `ready`'s stream is alive
        if (!hit->done && !hip_ok(hipStreamWaitEvent(stream, hit->ready, 0), "locator wait")) return nullptr;
        return hit;
      }
    ++d->loc_misses;
    if (d->loc.size() >= kLocatorCache) {
      evicted = std::move(d->loc.back());
      d->loc.pop_back();
      // nobody else holds it (no new holder can appear: it left the list under
      // the lock), so only its own locator kernel may still touch the buffers
      if (evicted.use_count() == 1 && evicted->cap_n >= p.n) L = std::move(evicted);
    }
  }
  const uint16_t *fold = device_fold(d, p.n);
  if (!fold) return nullptr;
  if (L) {
    // nobody holds it, so every call that used it has synchronised its stream
    // (its kernel and the H2D of its key are complete); a fresh event, as the
    // old one may belong to a destroyed stream
    (void)hipEventDestroy(L->ready);
    L->ready = nullptr;
    L->done = false;
    if (!hip_ok(hipEventCreateWithFlags(&L->ready, hipEventDisableTiming), "hipEventCreate")) return nullptr;
  } else {
    L = std::make_shared<Locator>();
    L->cap_n = p.n;
    if (!hip_ok(hipMalloc(&L->d_present, p.n), "hipMalloc(locator)") ||
        !hip_ok(hipMalloc(&L->d_elog, size_t(p.n) * 2), "hipMalloc(locator)") ||
        !hip_ok(hipEventCreateWithFlags(&L->ready, hipEventDisableTiming), "hipEventCreate"))
      return nullptr;
  }
  L->nv = p.nv;
  L->present = present;
  if (!hip_ok(hipMemcpyAsync(L->d_present, L->present.data(), p.n, hipMemcpyHostToDevice, stream),
              "H2D present") ||
      !hip_ok(launch_error_locator(p, L->d_present, 1, fold, nullptr, L->d_elog, stream),
              "error locator launch") ||
      !hip_ok(hipEventRecord(L->ready, stream), "hipEventRecord")) {
    (void)hipStreamSynchronize(stream);  // nothing issued above may outlive L
    return nullptr;
  }
  std::lock_guard<std::mutex> lk(d->loc_mu);
  d->loc.push_front(L);
  return L;
}

namespace {
// Frees the evicted entries nobody holds any more, after a device
// synchronisation (their streams may be gone, so the whole device is waited
// for).  Called where waiting is allowed: never while `s` is being captured.
// A device-wide synchronisation (and hipFree) made while ANOTHER thread
// captures a stream in global mode invalidates that capture, so the implicit
// drain at the start of a plain call runs only once kDeadDrain evicted buffers
// have gathered (at most one such drain per kDeadDrain evictions, i.e. only
// when more than 64 streams of a device use the plain calls; ec_amd.h); the
// explicit one (ECCR_AMD_release_stream_scratch) always runs.
constexpr size_t kDeadDrain = 16;
void drain_dead(DeviceState *d, hipStream_t s, bool force) {
  std::list<std::shared_ptr<StreamScratchEntry>> dead;
  {
    std::lock_guard<std::mutex> lk(d->ss_mu);
    if (d->ss_dead.empty() || (!force && d->ss_dead.size() < kDeadDrain)) return;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return;
    for (auto it = d->ss_dead.begin(); it != d->ss_dead.end();)
      if (it->use_count() == 1) {  // no lease holds it
        dead.push_back(std::move(*it));
        it = d->ss_dead.erase(it);
      } else {
        ++it;
      }
  }
  if (dead.empty()) return;
  (void)hipDeviceSynchronize();
  for (auto &e : dead)
    if (e->p) (void)hipFree(e->p);
}
}  // namespace

StreamScratch::StreamScratch(DeviceState *d, hipStream_t s, size_t bytes) : want_(bytes) {
  if (!d || bytes == 0) return;
  drain_dead(d, s, false);
  const size_t limit = g_scratch_limit;
  if (limit && bytes > limit) {  // as if hipMalloc had failed
    set_error("erasure_coding_crust(amd): scratch of " + std::to_string(bytes) +
              " bytes exceeds the limit set by ECCR_AMD_set_scratch_limit");
    return;
  }
  {
    std::lock_guard<std::mutex> lk(d->ss_mu);
    auto it = d->ss.begin();
    while (it != d->ss.end() && (*it)->s != s) ++it;
    if (it != d->ss.end()) {
      d->ss.splice(d->ss.begin(), d->ss, it);  // most recent first
    } else {
      if (d->ss.size() >= kStreamScratch) {
        d->ss_dead.push_back(std::move(d->ss.back()));  // freed by a later drain_dead()
        d->ss.pop_back();
      }
      auto e = std::make_shared<StreamScratchEntry>();
      e->s = s;
      d->ss.push_front(std::move(e));
    }
    e_ = d->ss.front();
  }
  e_->mu.lock();
  locked_ = true;
  if (e_->cap < bytes) {
    // every earlier holder on this stream has finished enqueueing (they held
    // mu), so once the stream drains nothing reads the smaller buffer
    if (e_->p) {
      if (!hip_ok(hipStreamSynchronize(s), "scratch grow sync")) return;
      (void)hipFree(e_->p);
    }
    e_->p = nullptr;
    e_->cap = 0;
    if (!hip_ok(hipMalloc(&e_->p, bytes), "hipMalloc(stream scratch)")) return;
    e_->cap = bytes;
  }
  p_ = e_->p;
}

StreamScratch::~StreamScratch() {
  if (locked_) e_->mu.unlock();
}

bool release_stream_scratch(DeviceState *d, hipStream_t s) {
  std::shared_ptr<StreamScratchEntry> e;
  {
    std::lock_guard<std::mutex> lk(d->ss_mu);
    for (auto it = d->ss.begin(); it != d->ss.end(); ++it)
      if ((*it)->s == s) {
        e = std::move(*it);
        d->ss.erase(it);
        break;
      }
  }
  if (!e) return false;
  {
    std::lock_guard<std::mutex> lk(e->mu);  // no caller is enqueueing on it
    if (e.use_count() == 1 && e->p) {       // nobody else can reach it any more
      (void)hipStreamSynchronize(s);
      (void)hipFree(e->p);
      e->p = nullptr;
      e->cap = 0;
    }
  }
  if (e->p) {  // a lease still holds it: freed by a later drain
    std::lock_guard<std::mutex> lk(d->ss_mu);
    d->ss_dead.push_back(std::move(e));
  }
  drain_dead(d, s, true);
  return true;
}

void locator_done(DeviceState *d, const Locator &L) {
  std::lock_guard<std::mutex> lk(d->loc_mu);
  L.done = true;
}

void locator_drop(DeviceState *d, const Locator &L) {
  std::shared_ptr<Locator> gone;  // released after the lock (~Locator frees)
  std::lock_guard<std::mutex> lk(d->loc_mu);
  for (auto it = d->loc.begin(); it != d->loc.end(); ++it)
    if (it->get() == &L) {
      gone = std::move(*it);
      d->loc.erase(it);
      break;
    }
}

void locator_cache_stats(DeviceState *d, unsigned long *hits, unsigned long *misses) {
  std::lock_guard<std::mutex> lk(d->loc_mu);
  if (hits) *hits = d->loc_hits;
  if (misses) *misses = d->loc_misses;
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

HostCtx::~HostCtx() {
  // the thread's work is finished (every C-ABI call synchronises its stream);
  // release on the context's own device
  int cur = -1;
  const bool switched = hipGetDevice(&cur) == hipSuccess && cur != device && device >= 0 &&
                        hipSetDevice(device) == hipSuccess;
  if (stream) {
    (void)hipStreamSynchronize(stream);
    forget_stream(device, stream);
    (void)hipStreamDestroy(stream);
  }
  for (uint8_t *h : {h_in, h_out})
    if (h) (void)hipHostFree(h);
  if (h_flag) (void)hipHostFree(h_flag);
  for (void *p : {static_cast<void *>(d_in), static_cast<void *>(d_out),
                  static_cast<void *>(d_present), static_cast<void *>(d_elog)})
    if (p) (void)hipFree(p);
  if (switched) (void)hipSetDevice(cur);
}

HostSig call_signal(HostCtx *c) {
  HostSig s;
  if (!c->h_flag) {
    if (hipHostMalloc(reinterpret_cast<void **>(&c->h_flag), 64, hipHostMallocDefault) != hipSuccess) {
      c->h_flag = nullptr;
      return s;
    }
    // a recycled pinned word may hold any stale value: start from a known one
    __atomic_store_n(c->h_flag, 0u, __ATOMIC_RELEASE);
    c->seq = 0;
  }
  uint32_t v = ++c->seq;
  if (v == 0) v = c->seq = 1;  // (wrap) 0 is the initial value
  s.flag = c->h_flag;
  s.v = v;
  return s;
}

bool finish_call(HostCtx *c, const char *what, const HostSig *sig) {
  const auto sync = [&]() { return hip_ok(hipStreamSynchronize(c->stream), what); };
  const HostSig s = sig ? *sig : call_signal(c);
  if (!s.flag) return sync();
  const uint32_t v = s.v;
  if (!s.fused && launch_signal_host(s.flag, v, c->stream) != hipSuccess) return sync();
  // now and then ask the stream for an asynchronous error the spin cannot see
  const bool probe = (v & (kFinishProbeEvery - 1)) == 0;
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  for (;;) {
    for (int i = 0; i < 64; ++i)
      if (__atomic_load_n(c->h_flag, __ATOMIC_ACQUIRE) == v) {
        if (!probe) return true;
        const hipError_t e = hipStreamQuery(c->stream);
        return e == hipSuccess || e == hipErrorNotReady || hip_ok(e, what);
      }
    if (std::chrono::duration<double, std::micro>(clk::now() - t0).count() > kFinishSpinUs)
      return sync();  // long calls block instead of spinning; errors surface here
  }
}

HostCtx *host_ctx() {
  // destroyed (buffers and stream released) at thread exit or when the
  // thread switches devices
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
