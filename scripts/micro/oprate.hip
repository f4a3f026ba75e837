// Per-opcode VALU throughput on gfx950: 16 independent chains per lane.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CH 16
template <int OP>
__global__ void __launch_bounds__(256) k(uint32_t *out, int iters, uint32_t c0) {
  uint32_t x[CH];
  for (int i = 0; i < CH; ++i) x[i] = threadIdx.x * (i + 3) + c0;
  uint32_t y = c0 ^ threadIdx.x, z = c0 + threadIdx.x * 7;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      if (OP == 0) x[i] = __builtin_amdgcn_perm(y, z, x[i]);                 // v_perm
      if (OP == 1) x[i] = __builtin_amdgcn_bitop3_b32(x[i], y, z, 0x96);      // v_bitop3
      if (OP == 2) x[i] = x[i] ^ y;                                           // v_xor
      if (OP == 3) x[i] = (x[i] >> 3) & 0x07070707u;                          // shr + and
      if (OP == 4) x[i] = __builtin_amdgcn_perm(x[i], z, y);                  // perm, table dep
      if (OP == 5) x[i] = x[i] * 0x9E3779B1u + y;                             // v_mad_u32_u24? (mul_lo)
      if (OP == 6) {                                                           // v_lshrrev_b64 (pairs)
        if (i % 2 == 0) {
          uint64_t v = (uint64_t(x[i + 1]) << 32) | x[i];
          asm volatile("v_lshrrev_b64 %0, 3, %0" : "+v"(v));
          x[i] = uint32_t(v);
          x[i + 1] = uint32_t(v >> 32);
        }
      }
      if (OP == 7) x[i] = __builtin_amdgcn_alignbit(x[i], y, 3);              // v_alignbit_b32
      if (OP == 8) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(x[i]));     // v_lshrrev_b32 alone
    }
  }
  uint32_t r = 0;
  for (int i = 0; i < CH; ++i) r ^= x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
template <int OP>
void run(const char *name, uint32_t *out, double ninstr_per_iter) {
  const int blocks = 4096, iters = 2000;
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, iters, 12345u);
  hipEventRecord(a);
  hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, iters, 12345u);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  double wi = double(blocks) * 4 * iters * CH * ninstr_per_iter;
  printf("%-10s %.3f ms  %.3e wave-instr/s  = %.2f wave-instr/clk/CU at 2.4GHz\n", name, ms,
         wi / (ms * 1e-3), wi / (ms * 1e-3) / 256 / 2.4e9);
}
int main() {
  uint32_t *out; hipMalloc(&out, 4096 * 256 * 4);
  run<0>("perm", out, 1); run<1>("bitop3", out, 1); run<2>("xor", out, 1);
  run<3>("shr+and", out, 2); run<4>("perm-tab", out, 1); run<5>("mul+add", out, 2);
  // round 5: the 64-bit selector shift of mul_acc against 32-bit forms (the
  // b64 run issues CH / 2 instructions per iteration)
  run<6>("shr_b64", out, 0.5); run<7>("alignbit", out, 1); run<8>("shr_b32", out, 1);
  return 0;
}
