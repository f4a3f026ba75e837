// Round trip of a one-wave kernel + host spin on a pinned flag, by where a
// small call's payload comes from (the per-call C ABI at
// 15 B / 300 B, nv = 6).  Every variant writes OUT bytes of "shards" to pinned
// host memory, then __threadfence_system and the flag (the direct path of
// capi.cpp):
//   flag      nothing but the flag (the launch + spin floor)
//   host      the payload read from pinned host memory (capi.cpp today)
//   karg      the payload passed by value in the kernel arguments
//   host+tab  as host, plus one dependent 80-B table load from device memory
//   karg+tab  as karg, plus the table load
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

constexpr int PB = 320;  // payload bytes carried (>= 300)
struct Karg {
  uint32_t w[PB / 4];
};

template <bool KARG, bool TAB>
__global__ void small(const uint32_t *hin, Karg ka, const uint4 *tab, uint32_t *hout, int out_words,
                      volatile uint32_t *flag, uint32_t v) {
  const int l = threadIdx.x;
  uint32_t x = 0;
  if (l < PB / 4) x = KARG ? ka.w[l] : hin[l];
  if (TAB) {
    const uint4 t = tab[x & 7];
    x ^= t.x ^ t.w;
  }
  for (int i = l; i < out_words; i += 64) hout[i] = x + uint32_t(i);
  __threadfence_system();
  __syncthreads();
  if (l == 0) __hip_atomic_store(const_cast<uint32_t *>(flag), v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  uint32_t *hin, *hout, *flag;
  uint4 *tab;
  (void)hipHostMalloc(reinterpret_cast<void **>(&hin), 4096, hipHostMallocDefault);
  (void)hipHostMalloc(reinterpret_cast<void **>(&hout), 65536, hipHostMallocDefault);
  (void)hipHostMalloc(reinterpret_cast<void **>(&flag), 64, hipHostMallocDefault);
  (void)hipMalloc(&tab, 4096);
  (void)hipMemset(tab, 0, 4096);
  std::memset(hin, 1, 4096);
  *flag = 0;
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  Karg ka;
  std::memset(&ka, 2, sizeof(ka));
  const int N = 2000;
  uint32_t v = 0;
  auto run = [&](const char *name, int out_words, auto launch) {
    std::vector<double> t;
    for (int i = 0; i < N + 50; ++i) {
      ++v;
      const double t0 = now_us();
      std::memcpy(hin, &ka, 64);  // the host copy into the pinned staging, as capi.cpp
      launch(out_words, v);
      while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != v) {
      }
      const double t1 = now_us();
      if (i >= 50) t.push_back(t1 - t0);
    }
    std::sort(t.begin(), t.end());
    double m = 0;
    for (double x : t) m += x;
    std::printf("%-10s out %6d B  median %6.2f us  mean %6.2f us  p90 %6.2f us\n", name, 4 * out_words,
                t[t.size() / 2], m / t.size(), t[t.size() * 9 / 10]);
  };
  for (int ow : {8, 96, 1024}) {
    run("flag", 0, [&](int, uint32_t vv) {
      hipLaunchKernelGGL((small<false, false>), dim3(1), dim3(64), 0, s, hin, ka, tab, hout, 0, flag, vv);
    });
    run("host", ow, [&](int o, uint32_t vv) {
      hipLaunchKernelGGL((small<false, false>), dim3(1), dim3(64), 0, s, hin, ka, tab, hout, o, flag, vv);
    });
    run("karg", ow, [&](int o, uint32_t vv) {
      hipLaunchKernelGGL((small<true, false>), dim3(1), dim3(64), 0, s, hin, ka, tab, hout, o, flag, vv);
    });
    run("host+tab", ow, [&](int o, uint32_t vv) {
      hipLaunchKernelGGL((small<false, true>), dim3(1), dim3(64), 0, s, hin, ka, tab, hout, o, flag, vv);
    });
    run("karg+tab", ow, [&](int o, uint32_t vv) {
      hipLaunchKernelGGL((small<true, true>), dim3(1), dim3(64), 0, s, hin, ka, tab, hout, o, flag, vv);
    });
  }
  (void)hipStreamSynchronize(s);
  return 0;
}
