// mul_acc butterfly throughput at the kernels' occupancy: one workgroup per CU
// (grid = 256), WAVES waves per workgroup, CHAINS independent butterflies per lane.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../erasure-coding-crust_amd/csrc/ec_device.hpp"
using namespace ecamd;

template <int CHAINS, int THREADS>
__global__ void __launch_bounds__(THREADS) k(const uint32_t *tab, uint32_t *out, int iters) {
  Tab T;
  for (int i = 0; i < 20; ++i) T.t[i] = tab[i] ^ threadIdx.x;
  uint32_t al[CHAINS], ah[CHAINS], bl[CHAINS], bh[CHAINS];
  for (int c = 0; c < CHAINS; ++c) { al[c] = threadIdx.x * (c + 1); ah[c] = al[c] ^ 0x5555; bl[c] = al[c] + 7; bh[c] = ah[c] + 9; }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
      mul_acc(bl[c], bh[c], T, al[c], ah[c]);
      bl[c] ^= al[c]; bh[c] ^= ah[c];
    }
  }
  uint32_t r = 0;
  for (int c = 0; c < CHAINS; ++c) r ^= al[c] ^ ah[c] ^ bl[c] ^ bh[c];
  out[blockIdx.x * THREADS + threadIdx.x] = r;
}

template <int CHAINS, int THREADS>
void run(uint32_t *tab, uint32_t *out) {
  const int blocks = 256, iters = 40000 / CHAINS;
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  hipLaunchKernelGGL((k<CHAINS, THREADS>), dim3(blocks), dim3(THREADS), 0, 0, tab, out, iters);
  (void)hipEventRecord(a);
  hipLaunchKernelGGL((k<CHAINS, THREADS>), dim3(blocks), dim3(THREADS), 0, 0, tab, out, iters);
  (void)hipEventRecord(b); (void)hipEventSynchronize(b);
  float ms; (void)hipEventElapsedTime(&ms, a, b);
  double bfly = double(blocks) * THREADS * iters * CHAINS * 4;
  printf("waves/SIMD=%d chains=%d  %.3e symbol-butterflies/s\n", THREADS / 256, CHAINS, bfly / (ms * 1e-3));
}

int main() {
  uint32_t *tab, *out; (void)hipMalloc(&tab, 80); (void)hipMalloc(&out, 256 * 1024 * 4);
  (void)hipMemset(tab, 0x37, 80);
  run<1, 512>(tab, out); run<2, 512>(tab, out); run<4, 512>(tab, out); run<8, 512>(tab, out);
  run<1, 1024>(tab, out); run<2, 1024>(tab, out); run<4, 1024>(tab, out); run<8, 1024>(tab, out);
  run<4, 256>(tab, out); run<8, 256>(tab, out);
  return 0;
}
