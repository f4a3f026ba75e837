// PCIe copy rates between pinned host memory and HBM (256 MB): SDMA copies
// (one, or split over 4 streams) and a copy kernel reading / writing the
// device-mapped host buffer directly; each direction alone and both at once.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
__global__ void copyk(uint4 *__restrict__ dst, const uint4 *__restrict__ src, size_t n16) {
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n16; i += size_t(gridDim.x) * blockDim.x)
    dst[i] = src[i];
}
int main() {
  const size_t n = 256ull << 20;
  void *h1, *h2, *d1, *d2, *m1, *m2;
  CK(hipHostMalloc(&h1, n, hipHostMallocMapped)); CK(hipHostMalloc(&h2, n, hipHostMallocMapped));
  CK(hipHostGetDevicePointer(&m1, h1, 0)); CK(hipHostGetDevicePointer(&m2, h2, 0));
  CK(hipMalloc(&d1, n)); CK(hipMalloc(&d2, n));
  hipStream_t s[8];
  for (auto &x : s) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  // h2d / d2h: 0 none, 1 one SDMA copy, 4 four SDMA copies, 9 copy kernel
  auto run = [&](const char *name, int h2d, int d2h, int grid) -> int {
    float ms = 0;
    const int reps = 4;
    for (int r = 0; r < reps + 1; ++r) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(a, 0));
      if (h2d == 9) hipLaunchKernelGGL(copyk, dim3(grid), dim3(256), 0, s[0], (uint4 *)d1, (const uint4 *)m1, n / 16);
      else for (int i = 0; i < h2d; ++i)
        CK(hipMemcpyAsync((char *)d1 + i * (n / h2d), (char *)h1 + i * (n / h2d), n / h2d, hipMemcpyHostToDevice, s[i]));
      if (d2h == 9) hipLaunchKernelGGL(copyk, dim3(grid), dim3(256), 0, s[4], (uint4 *)m2, (const uint4 *)d2, n / 16);
      else for (int i = 0; i < d2h; ++i)
        CK(hipMemcpyAsync((char *)h2 + i * (n / d2h), (char *)d2 + i * (n / d2h), n / d2h, hipMemcpyDeviceToHost, s[4 + i]));
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(b, 0)); CK(hipEventSynchronize(b));
      float x; CK(hipEventElapsedTime(&x, a, b));
      if (r) ms += x;
    }
    ms /= reps;
    const double bytes = double(n) * ((h2d > 0) + (d2h > 0));
    printf("%-34s grid %4d  %7.3f ms  %6.1f GB/s total\n", name, grid, ms, bytes / ms / 1e6);
    return 0;
  };
  // stream pairs: one H2D on stream i, one D2H on stream j (which pairs share a copy engine?)
  for (int j = 1; j < 8; ++j) {
    float ms = 0;
    for (int r = 0; r < 3; ++r) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(a, 0));
      CK(hipMemcpyAsync(d1, h1, n, hipMemcpyHostToDevice, s[0]));
      CK(hipMemcpyAsync(h2, d2, n, hipMemcpyDeviceToHost, s[j]));
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(b, 0)); CK(hipEventSynchronize(b));
      float x; CK(hipEventElapsedTime(&x, a, b));
      if (r) ms += x / 2;
    }
    printf("H2D on stream 0, D2H on stream %d: %.3f ms  %.1f GB/s total\n", j, ms, 2.0 * n / ms / 1e6);
  }
  run("H2D sdma x1", 1, 0, 0);
  run("H2D sdma x4", 4, 0, 0);
  run("H2D kernel", 9, 0, 256);
  run("H2D kernel", 9, 0, 1024);
  run("D2H sdma x1", 0, 1, 0);
  run("D2H sdma x4", 0, 4, 0);
  run("D2H kernel", 0, 9, 256);
  run("D2H kernel", 0, 9, 1024);
  run("both: sdma x1 / sdma x1", 1, 1, 0);
  run("both: sdma x4 / sdma x4", 4, 4, 0);
  run("both: sdma x1 / kernel", 1, 9, 256);
  run("both: sdma x4 / kernel", 4, 9, 256);
  run("both: kernel / kernel", 9, 9, 256);
  return 0;
}
