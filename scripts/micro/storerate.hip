// storerate.hip — store throughput of the encode's shard-row store shape:
// 16 waves per workgroup (one workgroup per CU), each global_store_dwordx4
// writes 4 rows x 256 contiguous bytes (lane = row-in-4 x 16-B chunk), rows
// ROWB bytes apart.  Grid sizes 16 .. 256 workgroups separate the per-CU rate
// from the chip-wide rate.  Also a variant with VALU work between the stores.
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int ROWB = 3968;  // the bench's shard pitch (3908 B rows rounded up to 64 B)

template <int WORK>
__global__ void __launch_bounds__(1024) rows(uint8_t *buf, int iters, uint64_t span) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint8_t *base = buf + uint64_t(blockIdx.x) * span;
  uint32_t x = lane * 0x9E3779B9u;
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  for (int i = 0; i < iters; ++i) {
    // tile i: 256 rows x 256 B at column (i % 15) * 256 of a 4 MB row block
    const uint64_t row = uint64_t(wave * 4 + (lane >> 4));
    uint8_t *dst = base + uint64_t((i % 15) * 256 + (lane & 15) * 16) + row * ROWB;
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      v4u v = {x, x + 1, x + 2, x + 3};
      __builtin_nontemporal_store(v, reinterpret_cast<v4u *>(dst + uint64_t(it) * 64 * ROWB));
    }
#pragma unroll
    for (int w = 0; w < WORK; ++w) x = __builtin_amdgcn_perm(x, x ^ w, 0x05040100u + w);
  }
  if (x == 0x12345678u) buf[0] = 1;
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const uint64_t span = uint64_t(256) * ROWB + 16 * 256;  // per workgroup
  uint8_t *buf;
  if (hipMalloc(&buf, span * 256) != hipSuccess) return 1;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int iters = 2000;
  for (int work : {0, 1}) {
    for (int grid : {16, 32, 64, 128, 256}) {
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(a);
        if (work) hipLaunchKernelGGL(rows<64>, dim3(grid), dim3(1024), 0, nullptr, buf, iters, span);
        else hipLaunchKernelGGL(rows<0>, dim3(grid), dim3(1024), 0, nullptr, buf, iters, span);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        const double bytes = double(grid) * iters * 16 * 4 * 1024;
        if (rep) printf("work=%d grid=%3d  %.3f ms  %.2f TB/s  %.1f B/clk per active CU at 2.4 GHz\n", work, grid,
                        ms, bytes / ms / 1e9, bytes / grid / (ms * 1e-3 * 2.4e9));
      }
    }
  }
  printf("cus=%d\n", cus);
  return 0;
}
