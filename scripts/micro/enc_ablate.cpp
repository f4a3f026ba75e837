// Encode-kernel timer: enc_k256.hip compiled in
// (see the switch list there); 512 x 1 MB payloads, n_validators = 1024.
// Outputs are NOT correct for a nonzero mask; only the time is of interest.
#include "../../erasure-coding-crust_amd/csrc/enc_k256.hip"

#include <cstdio>

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
  uint8_t *pay, *sh;
  (void)hipMalloc(&pay, B * plen);
  (void)hipMalloc(&sh, B * 1024 * ss);
  (void)hipMemset(pay, 0x5a, B * plen);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int i = 0; i < 2; ++i) launch_encode_k256(p, t, pay, plen, plen, B, sh, ss, nullptr);
  (void)hipEventRecord(a);
  const int reps = 10;
  for (int i = 0; i < reps; ++i) launch_encode_k256(p, t, pay, plen, plen, B, sh, ss, nullptr);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  printf("encode_k256  %.4f ms per launch (512 x 1 MB)\n", ms / reps);
  return 0;
}
