// occ_probe.hip — workgroups per CU the runtime reports for a kernel of a
// given block size and dynamic LDS (the two-workgroup reconstruct question,
// profiles/r06/NOTES.md).  Build: hipcc --offload-arch=gfx950 -O2 occ_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int T>
__global__ void __launch_bounds__(T, 2) probe(unsigned *p) {
  extern __shared__ unsigned lds[];
  lds[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (p) p[threadIdx.x] = lds[(threadIdx.x + 1) % T];
}

template <int T>
void q(int lds) {
  const void *fn = reinterpret_cast<const void *>(&probe<T>);
  hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  int n = -1;
  const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, probe<T>, T, lds);
  printf("threads %d lds %d -> %d workgroups per CU (%s)\n", T, lds, n, hipGetErrorString(e));
}

int main() {
  hipDeviceProp_t pr;
  hipGetDeviceProperties(&pr, 0);
  printf("%s sharedMemPerMultiprocessor %zu maxSharedMemoryPerMultiProcessor %zu sharedMemPerBlock %zu\n",
         pr.gcnArchName, pr.sharedMemPerBlock, pr.maxSharedMemoryPerMultiProcessor, pr.sharedMemPerBlock);
  q<384>(81920);
  q<384>(81920 - 512);
  q<320>(73728);
  q<512>(65552);
  q<768>(159760);
  return 0;
}
