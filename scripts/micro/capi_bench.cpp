// Per-call latency of the erasure_coding.h C ABI on the GPU path, at the
// payload sizes of the reference's benchmark/benchmark.cpp (BASELINE.md §1:
// 100 calls of ECCR_Test_MeasurePerformance = encode + reconstruct from all
// shards), plus ECCR_obtain_chunks / ECCR_reconstruct with only
// threshold-many random shards (a real erasure decode).  One JSON line per
// case on stdout.
//
// build: g++ -O2 -std=c++17 -I include scripts/micro/capi_bench.cpp \
//          -L erasure-coding-crust_amd/lib -lerasure_coding_crust \
//          -Wl,-rpath,$PWD/erasure-coding-crust_amd/lib -o scripts/micro/capi_bench
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

extern "C" {
#include <erasure_coding/erasure_coding.h>
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

int main(int argc, char **argv) {
  // optional: argv[1] = one payload size, argv[2] = calls (traces of one size)
  std::vector<unsigned long> sizes = {15, 300, 5000, 100000, 1000000, 10000000};
  if (argc > 1) sizes = {std::strtoul(argv[1], nullptr, 10)};
  const int calls = argc > 2 ? std::atoi(argv[2]) : 0;
  const unsigned long nvs[] = {6, 1024};
  for (unsigned long nv : nvs) {
    unsigned long thr = 0;
    if (ECCR_get_recovery_threshold(nv, &thr).tag != NPRS_RESULT_OK) return 1;
    for (unsigned long sz : sizes) {
      std::vector<uint8_t> payload(sz);
      for (unsigned long i = 0; i < sz; ++i) payload[i] = uint8_t(97 + i % 24);
      DataBlock msg{payload.data(), sz};
      const int reps = calls ? calls : sz >= 10000000 ? 10 : 100;
      // (1) the reference benchmark's call: MeasurePerformance (decode from all shards)
      unsigned long e = 0, d = 0, se = 0, sd = 0;
      for (int i = 0; i < 3; ++i) ECCR_Test_MeasurePerformance(&msg, nv, &e, &d);  // warm-up
      for (int i = 0; i < reps; ++i) {
        if (ECCR_Test_MeasurePerformance(&msg, nv, &e, &d).tag != NPRS_RESULT_OK) return 2;
        se += e;
        sd += d;
      }
      // (2) obtain_chunks + reconstruct from threshold-many random shards
      std::mt19937 rng(unsigned(nv * 131 + sz));
      double t_enc = 0, t_dec = 0;
      for (int i = 0; i < reps + 2; ++i) {
        ChunksList list{};
        const double t0 = now_us();
        if (ECCR_obtain_chunks(nv, &msg, &list).tag != NPRS_RESULT_OK) return 3;
        const double t1 = now_us();
        std::vector<unsigned long> idx(nv);
        for (unsigned long v = 0; v < nv; ++v) idx[v] = v;
        std::shuffle(idx.begin(), idx.end(), rng);
        std::vector<Chunk> keep(thr);
        for (unsigned long j = 0; j < thr; ++j) keep[j] = list.data[idx[j]];
        ChunksList in{keep.data(), thr};
        DataBlock out{};
        const double t2 = now_us();
        if (ECCR_reconstruct(nv, &in, &out).tag != NPRS_RESULT_OK) return 4;
        const double t3 = now_us();
        if (out.length < sz || std::memcmp(out.array, payload.data(), sz) != 0) return 5;
        ECCR_deallocate_data_block(&out);
        ECCR_deallocate_chunk_list(&list);
        if (i >= 2) {
          t_enc += t1 - t0;
          t_dec += t3 - t2;
        }
      }
      std::printf(
          "{\"n_validators\": %lu, \"payload_bytes\": %lu, \"calls\": %d, "
          "\"measure_perf_encode_us_per_100\": %.1f, \"measure_perf_decode_us_per_100\": %.1f, "
          "\"obtain_chunks_us\": %.1f, \"reconstruct_threshold_us\": %.1f, \"threshold\": %lu}\n",
          nv, sz, reps, 100.0 * se / reps, 100.0 * sd / reps, t_enc / reps, t_dec / reps, thr);
      std::fflush(stdout);
    }
  }
  return 0;
}
