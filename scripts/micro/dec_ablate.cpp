// Reconstruct-kernel timer (+ -DDEC_STAMP phase split): dec_n1024.hip compiled in
// (switch list there); 512 x 1 MB payloads, n_validators = 1024, 342 present.
#include "../../erasure-coding-crust_amd/csrc/dec_n1024.hip"

#include <cstdio>
#include <vector>

int main() {
  using namespace ecamd;
  const Field &F = field();
  CodeParams p;
  code_params(1024, &p);
  uint16_t *sk;
  MulTab *mt;
  (void)hipMalloc(&sk, F.skews.size() * 2);
  (void)hipMalloc(&mt, F.mtab.size() * sizeof(MulTab));
  (void)hipMemcpy(sk, F.skews.data(), F.skews.size() * 2, hipMemcpyHostToDevice);
  (void)hipMemcpy(mt, F.mtab.data(), F.mtab.size() * sizeof(MulTab), hipMemcpyHostToDevice);
  DevTables t;
  t.skews = sk;
  t.mtab = mt;
  const size_t B = 512, plen = 1000000, sl = shard_len(p.k, plen), ss = (sl + 63) / 64 * 64;
  std::vector<uint8_t> pres(B * 1024, 0);
  std::vector<uint16_t> el(B * 1024);
  for (size_t b = 0; b < B; ++b)
    for (int v = 0; v < 1024; ++v) {
      pres[b * 1024 + v] = ((v * 2654435761u + b * 97) >> 7) % 3 == 0;  // ~1/3 present
      el[b * 1024 + v] = uint16_t((v * 40503u + b) % 65535);
    }
  uint8_t *sh, *dp, *out;
  uint16_t *de;
  (void)hipMalloc(&sh, B * 1024 * ss);
  (void)hipMalloc(&dp, B * 1024);
  (void)hipMalloc(&de, B * 1024 * 2);
  (void)hipMalloc(&out, B * sl * 256);
  (void)hipMemset(sh, 0x3c, B * 1024 * ss);
  (void)hipMemcpy(dp, pres.data(), pres.size(), hipMemcpyHostToDevice);
  (void)hipMemcpy(de, el.data(), el.size() * 2, hipMemcpyHostToDevice);
  void *order = nullptr;
  (void)hipMalloc(&order, gather_order_bytes(p, B));
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int i = 0; i < 2; ++i) launch_reconstruct_n1024(p, t, sh, sl, ss, dp, de, nullptr, B, out, sl * 256, order, nullptr);
  (void)hipEventRecord(a);
  const int reps = 10;
  for (int i = 0; i < reps; ++i) launch_reconstruct_n1024(p, t, sh, sl, ss, dp, de, nullptr, B, out, sl * 256, order, nullptr);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  printf("reconstruct_n1024  %.4f ms per launch (512 x 1 MB)\n", ms / reps);
#ifdef DEC_STAMP
  unsigned long long st[16];
  (void)hipMemcpyFromSymbol(st, HIP_SYMBOL(g_dec_stamp), sizeof(st));
  unsigned long long tot = 0;
  for (int i = 1; i <= 10; ++i) tot += st[i];
  const char *nm[11] = {"", "sync0", "gather", "sync1", "ifft", "deriv", "-", "-", "fft7-0", "-", "output"};
  for (int i = 1; i <= 10; ++i) printf("  %-8s %5.1f%%\n", nm[i], 100.0 * st[i] / tot);
#endif
  return 0;
}
