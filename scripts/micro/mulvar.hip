// mul_acc formulation variants: selector extraction with 32-bit vs 64-bit shifts.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../erasure-coding-crust_amd/csrc/ec_device.hpp"
using namespace ecamd;

__device__ __forceinline__ void mul_acc64(uint32_t xl, uint32_t xh, const Tab &T, uint32_t &yl,
                                          uint32_t &yh) {
  const uint64_t x = (uint64_t(xh) << 32) | xl;
  uint64_t t3, t6;
  asm volatile("v_lshrrev_b64 %0, 3, %1" : "=v"(t3) : "v"(x));
  asm volatile("v_lshrrev_b64 %0, 6, %1" : "=v"(t6) : "v"(x));
  const uint32_t s0 = xl & 0x07070707u, s3 = xh & 0x07070707u;
  const uint32_t s1 = uint32_t(t3) & 0x07070707u, s4 = uint32_t(t3 >> 32) & 0x07070707u;
  const uint32_t s2 = uint32_t(t6) & 0x03030303u, s5 = uint32_t(t6 >> 32) & 0x03030303u;
  uint32_t l = xor3(yl, vperm(T.t[1], T.t[0], s0), vperm(T.t[5], T.t[4], s1));
  l = xor3(l, vperm(T.t[9], T.t[8], s3), vperm(T.t[13], T.t[12], s4));
  l = xor3(l, vperm(T.t[16], T.t[16], s2), vperm(T.t[18], T.t[18], s5));
  uint32_t h = xor3(yh, vperm(T.t[3], T.t[2], s0), vperm(T.t[7], T.t[6], s1));
  h = xor3(h, vperm(T.t[11], T.t[10], s3), vperm(T.t[15], T.t[14], s4));
  h = xor3(h, vperm(T.t[17], T.t[17], s2), vperm(T.t[19], T.t[19], s5));
  yl = l;
  yh = h;
}

template <int V, int CHAINS>
__global__ void __launch_bounds__(256) k(const uint32_t *tab, uint32_t *out, int iters) {
  Tab T;
  for (int i = 0; i < 20; ++i) T.t[i] = tab[i] ^ threadIdx.x;
  uint32_t al[CHAINS], ah[CHAINS], bl[CHAINS], bh[CHAINS];
  for (int c = 0; c < CHAINS; ++c) { al[c] = threadIdx.x * (c + 1); ah[c] = al[c] ^ 0x5555; bl[c] = al[c] + 7; bh[c] = ah[c] + 9; }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
      if (V == 0) mul_acc(bl[c], bh[c], T, al[c], ah[c]);
      else mul_acc64(bl[c], bh[c], T, al[c], ah[c]);
      bl[c] ^= al[c]; bh[c] ^= ah[c];
    }
  }
  uint32_t r = 0;
  for (int c = 0; c < CHAINS; ++c) r ^= al[c] ^ ah[c] ^ bl[c] ^ bh[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int V>
void run(const char *nm, uint32_t *tab, uint32_t *out) {
  const int blocks = 4096, iters = 250;
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  hipLaunchKernelGGL((k<V, 8>), dim3(blocks), dim3(256), 0, 0, tab, out, iters);
  hipEventRecord(a);
  hipLaunchKernelGGL((k<V, 8>), dim3(blocks), dim3(256), 0, 0, tab, out, iters);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  double bfly = double(blocks) * 256 * iters * 8 * 4;
  printf("%-8s %.3f ms  %.3e symbol-butterflies/s\n", nm, ms, bfly / (ms * 1e-3));
}

int main() {
  uint32_t *tab, *out; hipMalloc(&tab, 80); hipMalloc(&out, 4096 * 256 * 4);
  hipMemset(tab, 0x37, 80);
  run<0>("shift32", tab, out); run<1>("shift64", tab, out);
  run<0>("shift32", tab, out); run<1>("shift64", tab, out);
  return 0;
}
