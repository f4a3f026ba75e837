// n = 4096 reconstruct timer (+ -DDEC4_STAMP phase split) for dec_n4096.hip
// 512 x 1 MB payloads, n_validators = 4096, ~1/3 of the shards present.
#include "../../erasure-coding-crust_amd/csrc/dec_n4096.hip"

#include <cstdio>

#include "../../erasure-coding-crust_amd/csrc/ec_runtime.hpp"
#include <vector>

int main() {
  using namespace ecamd;
  const Field &F = field();
  CodeParams p;
  code_params(4096, &p);
  DevTables t = device_tables(device_state());  // includes the LDS table images
  const size_t B = 512, plen = 1000000, sl = shard_len(p.k, plen), ss = (sl + 63) / 64 * 64;
  std::vector<uint8_t> pres(B * 4096, 0);
  std::vector<uint16_t> el(B * 4096);
  for (size_t b = 0; b < B; ++b)
    for (int v = 0; v < 4096; ++v) {
      pres[b * 4096 + v] = ((v * 2654435761u + b * 97) >> 7) % 3 == 0;  // ~1/3 present
      el[b * 4096 + v] = uint16_t((v * 40503u + b) % 65535);
    }
  uint8_t *sh, *dp, *out;
  uint16_t *de;
  (void)hipMalloc(&sh, B * 4096 * ss);
  (void)hipMalloc(&dp, B * 4096);
  (void)hipMalloc(&de, B * 4096 * 2);
  (void)hipMalloc(&out, B * sl * 1024);
  (void)hipMemset(sh, 0x3c, B * 4096 * ss);
  (void)hipMemcpy(dp, pres.data(), pres.size(), hipMemcpyHostToDevice);
  (void)hipMemcpy(de, el.data(), el.size() * 2, hipMemcpyHostToDevice);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int i = 0; i < 2; ++i) launch_reconstruct_n4096(p, t, sh, sl, ss, dp, de, B, out, sl * 1024, nullptr);
  (void)hipEventRecord(a);
  const int reps = 10;
  for (int i = 0; i < reps; ++i) launch_reconstruct_n4096(p, t, sh, sl, ss, dp, de, B, out, sl * 1024, nullptr);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  if (hipGetLastError() != hipSuccess) printf("launch error\n");
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  printf("n4096 reconstruct  %.4f ms per launch (512 x 1 MB)\n", ms / reps);
#ifdef DEC4_STAMP
  unsigned long long st[16];
  (void)hipMemcpyFromSymbol(st, HIP_SYMBOL(g_dec4_stamp), sizeof(st));
  unsigned long long tot = 0;
  for (int i = 1; i <= 11; ++i) tot += st[i];
  const char *nm[12] = {"", "qsync0", "q-gather", "qsync1", "q-ifft", "cross", "deriv", "fft", "esync0", "e-gather", "esync1", "output"};
  for (int i = 1; i <= 11; ++i) printf("  %-8s %5.1f%%\n", nm[i], 100.0 * st[i] / tot);
#endif
  return 0;
}
