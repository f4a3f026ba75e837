// FETCH_SIZE calibration for the reconstruct kernel's read widths
// (MI355X_MICROARCH.md: only 16-B/lane streaming reads are calibrated).
// Each kernel reads exactly `bytes` distinct bytes once:
//   k16:  16 B per lane, lanes contiguous (the calibrated case)
//   k64:  64 B per lane (4 x dwordx4), lane = row, rows 3968 B apart (phase 1)
//   k8:   8 B per lane, lanes contiguous (phase-5 shard re-reads)
//   k96:  96 B per lane (6 x dwordx4), lane = row, rows 3968 B apart
//         (reconstruct_n1024x's gather, round 5; reads rows x 40 x 96 B)
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k16(const uint4 *p, size_t n, uint32_t *out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}
__global__ void k64(const uint8_t *p, size_t rows, size_t stride, size_t cols64, uint32_t *out) {
  uint32_t acc = 0;
  const size_t total = rows * cols64;
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += size_t(gridDim.x) * blockDim.x) {
    const size_t r = i % rows, c = i / rows;  // consecutive lanes: consecutive rows
    const uint4 *q = reinterpret_cast<const uint4 *>(p + r * stride + 64 * c);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint4 v = q[j];
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}
__global__ void k8(const uint2 *p, size_t n, uint32_t *out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
    const uint2 v = p[i];
    acc ^= v.x ^ v.y;
  }
  if (acc == 0x12345678u) out[0] = acc;
}
__global__ void k96(const uint8_t *p, size_t rows, size_t stride, size_t cols96, uint32_t *out) {
  uint32_t acc = 0;
  const size_t total = rows * cols96;
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += size_t(gridDim.x) * blockDim.x) {
    const size_t r = i % rows, c = i / rows;  // consecutive lanes: consecutive rows
    const uint4 *q = reinterpret_cast<const uint4 *>(p + r * stride + 96 * c);
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const uint4 v = q[j];
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}
int main() {
  const size_t stride = 3968, cols64 = 61, rows = (size_t(1) << 30) / (64 * cols64);
  const size_t bytes = rows * cols64 * 64;
  uint8_t *p;
  uint32_t *out;
  const size_t cols96 = 40, rows96 = (size_t(1) << 30) / (96 * cols96);
  const size_t alloc = (rows > rows96 ? rows : rows96) * stride + 4096;  // every kernel's rows in bounds
  if (hipMalloc(&p, alloc) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
  (void)hipMemset(p, 1, alloc);
  hipLaunchKernelGGL(k16, dim3(4096), dim3(256), 0, 0, (const uint4 *)p, bytes / 16, out);
  hipLaunchKernelGGL(k64, dim3(4096), dim3(256), 0, 0, p, rows, stride, cols64, out);
  hipLaunchKernelGGL(k8, dim3(4096), dim3(256), 0, 0, (const uint2 *)p, bytes / 8, out);
  hipLaunchKernelGGL(k96, dim3(4096), dim3(256), 0, 0, p, rows96, stride, cols96, out);
  (void)hipDeviceSynchronize();
  printf("bytes per kernel: %zu (k96: %zu)\n", bytes, rows96 * cols96 * 96);
  return 0;
}
