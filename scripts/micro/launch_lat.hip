// Round-trip latency of one small kernel launch + host wait on gfx950, by
// wait method: hipStreamSynchronize,
// spinning on hipStreamQuery, hipEventSynchronize, and a host spin on a
// pinned flag the kernel writes (system-scope release).  Also the same with
// hipDeviceScheduleSpin set before the first HIP call (argv[1] == "spin").
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>
#include <algorithm>

__global__ void tiny(uint32_t *out, volatile uint32_t *flag, uint32_t v) {
  out[threadIdx.x] = v + threadIdx.x;
  if (flag) {
    __syncthreads();
    if (threadIdx.x == 0) {
      __threadfence_system();
      *flag = v;
    }
  }
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
  if (argc > 1 && !std::strcmp(argv[1], "spin")) (void)hipSetDeviceFlags(hipDeviceScheduleSpin);
  uint32_t *d_out, *h_flag;
  (void)hipMalloc(&d_out, 4096);
  (void)hipHostMalloc(reinterpret_cast<void **>(&h_flag), 64, hipHostMallocDefault);
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipEvent_t ev;
  (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  const int N = 2000;
  auto run = [&](const char *name, auto wait) {
    std::vector<double> t;
    for (int i = 0; i < N + 50; ++i) {
      const double t0 = now_us();
      wait(uint32_t(i + 1));
      const double t1 = now_us();
      if (i >= 50) t.push_back(t1 - t0);
    }
    std::sort(t.begin(), t.end());
    double m = 0;
    for (double x : t) m += x;
    std::printf("%-34s median %6.2f us  mean %6.2f us  p90 %6.2f us\n", name, t[t.size() / 2], m / t.size(),
                t[t.size() * 9 / 10]);
  };
  run("launch + hipStreamSynchronize", [&](uint32_t v) {
    hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d_out, nullptr, v);
    (void)hipStreamSynchronize(s);
  });
  run("launch + spin hipStreamQuery", [&](uint32_t v) {
    hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d_out, nullptr, v);
    while (hipStreamQuery(s) == hipErrorNotReady) {
    }
  });
  run("launch + event + hipEventSynchronize", [&](uint32_t v) {
    hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d_out, nullptr, v);
    (void)hipEventRecord(ev, s);
    (void)hipEventSynchronize(ev);
  });
  run("launch + host spin on pinned flag", [&](uint32_t v) {
    hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d_out, h_flag, v);
    while (__atomic_load_n(h_flag, __ATOMIC_ACQUIRE) != v) {
    }
  });
  (void)hipStreamSynchronize(s);
  run("launch only (enqueue cost)", [&](uint32_t v) {
    hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d_out, nullptr, v);
  });
  (void)hipStreamSynchronize(s);
  return 0;
}
