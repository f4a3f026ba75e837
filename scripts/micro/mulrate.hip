// Microbenchmark: throughput of the byte-planar v_perm multiply-accumulate
// (ec_device.hpp mul_acc) with CHAINS independent accumulators per lane.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../erasure-coding-crust_amd/csrc/ec_device.hpp"
using namespace ecamd;

template <int CHAINS>
__global__ void __launch_bounds__(256) k(const uint32_t *tab, uint32_t *out, int iters) {
  Tab T;
  for (int i = 0; i < 20; ++i) T.t[i] = tab[i] ^ threadIdx.x;
  uint32_t al[CHAINS], ah[CHAINS], bl[CHAINS], bh[CHAINS];
  for (int c = 0; c < CHAINS; ++c) { al[c] = threadIdx.x * (c + 1); ah[c] = al[c] ^ 0x5555; bl[c] = al[c] + 7; bh[c] = ah[c] + 9; }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {  // one forward butterfly per chain
      mul_acc(bl[c], bh[c], T, al[c], ah[c]);
      bl[c] ^= al[c]; bh[c] ^= ah[c];
    }
  }
  uint32_t r = 0;
  for (int c = 0; c < CHAINS; ++c) r ^= al[c] ^ ah[c] ^ bl[c] ^ bh[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int CHAINS>
void run(uint32_t *tab, uint32_t *out, int blocks, int iters) {
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  hipLaunchKernelGGL(k<CHAINS>, dim3(blocks), dim3(256), 0, 0, tab, out, iters);
  hipEventRecord(a);
  hipLaunchKernelGGL(k<CHAINS>, dim3(blocks), dim3(256), 0, 0, tab, out, iters);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  double bfly = double(blocks) * 256 * iters * CHAINS * 4;  // symbol butterflies
  double instr = double(blocks) * 4 * iters * CHAINS * 32;  // wave-instrs (approx 32/bfly-group)
  printf("chains=%d blocks=%d  %.3f ms  %.3e symbol-butterflies/s  %.3e wave-instr/s (~%.0f%% of 2/clk/CU @2.4GHz)\n",
         CHAINS, blocks, ms, bfly / (ms * 1e-3), instr / (ms * 1e-3),
         100.0 * instr / (ms * 1e-3) / (256 * 2 * 2.4e9));
}

int main() {
  uint32_t *tab, *out; hipMalloc(&tab, 80); hipMalloc(&out, 4096 * 256 * 4);
  hipMemset(tab, 0x37, 80);
  for (int blocks : {1024, 2048, 4096}) {
    run<1>(tab, out, blocks, 2000);
    run<2>(tab, out, blocks, 1000);
    run<4>(tab, out, blocks, 500);
    run<8>(tab, out, blocks, 250);
  }
  return 0;
}
