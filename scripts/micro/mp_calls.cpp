// Per-call times of ECCR_Test_MeasurePerformance (n_validators = 6, the
// reference benchmark's shape) for the first calls of a process and in steady
// state: where the first 100-call case's extra time goes.
// build: g++ -O2 -std=c++17 -I include scripts/micro/mp_calls.cpp -L erasure-coding-crust_amd/lib \
//   -lerasure_coding_crust -Wl,-rpath,'$ORIGIN/../../../erasure-coding-crust_amd/lib' -o scripts/micro/bin/mp_calls
#include <cstdio>
#include <cstring>
#include <vector>

#include "erasure_coding/erasure_coding.h"

int main() {
  for (size_t len : {15, 300, 15}) {
    std::vector<unsigned char> d(len, 7);
    DataBlock b;
    b.array = d.data();
    b.length = len;
    unsigned long se = 0, sd = 0;
    std::printf("%zu B:", len);
    for (int i = 0; i < 100; ++i) {
      unsigned long e = 0, dd = 0;
      ECCR_Test_MeasurePerformance(&b, 6, &e, &dd);
      se += e;
      sd += dd;
      if (i < 12) std::printf(" %lu/%lu", e, dd);
    }
    std::printf("  | 100 calls: encode %lu us, decode %lu us\n", se, sd);
  }
  return 0;
}
