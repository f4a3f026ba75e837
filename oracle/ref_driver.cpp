// ref_driver.cpp — thin extern "C" shim over the *reference* ec-cpp, compiled
// from the sources where they lie under /root/reference (see oracle/Makefile).
//
// TEST INFRASTRUCTURE ONLY: used to pin the C restatement (ec_oracle.c) and
// to generate tests/golden/*.json, and as bench.py's "reference" CPU
// baseline.  The output library lives in oracle/_ref/ (git-ignored).  This
// file contains no reference source; it only calls the reference API
// (include/ec-cpp/ec-cpp.hpp:15-26, reed-solomon.hpp:47-179).
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include <ec-cpp/ec-cpp.hpp>

using ec_cpp::PolyEncoder_f2e16;
using RS = ec_cpp::ReedSolomon<PolyEncoder_f2e16>;
using Shard = RS::Shard;

namespace {
int err_code(ec_cpp::Error e) { return int(e) + 1; }
}  // namespace

extern "C" {

int ecref_tables(uint16_t *log, uint16_t *exp, uint16_t *log_walsh) {
  ec_cpp::f2e16_Descriptor d;
  auto &[l, e, w] = d.kTables;
  std::memcpy(log, l.data(), 65536 * 2);
  std::memcpy(exp, e.data(), 65536 * 2);
  std::memcpy(log_walsh, w.data(), 65536 * 2);
  return 0;
}

int ecref_skews(uint16_t *out) {
  ec_cpp::f2e16_Descriptor d;
  auto a = ec_cpp::AdditiveFFT<ec_cpp::f2e16_Descriptor>::initalize(d.kTables);
  std::memcpy(out, a.skews, sizeof(a.skews));
  return 0;
}

int ecref_threshold(size_t nv, size_t *thr) {
  auto r = ec_cpp::getRecoveryThreshold(nv);
  if (ec_cpp::resultHasError(r)) return err_code(ec_cpp::resultGetError(std::move(r)));
  *thr = ec_cpp::resultGetValue(std::move(r));
  return 0;
}

int ecref_params(size_t nv, size_t *n, size_t *k) {
  auto r = ec_cpp::create(nv);
  if (ec_cpp::resultHasError(r)) return err_code(ec_cpp::resultGetError(std::move(r)));
  auto rs = ec_cpp::resultGetValue(std::move(r));
  *n = rs.n();
  *k = rs.k();
  return 0;
}

// shards written shard-major: shard v at out[v * shard_len]
int ecref_encode(size_t nv, const uint8_t *p, size_t len, uint8_t *out,
                 size_t cap, size_t *shard_len) {
  auto r = ec_cpp::create(nv);
  if (ec_cpp::resultHasError(r)) return err_code(ec_cpp::resultGetError(std::move(r)));
  auto rs = ec_cpp::resultGetValue(std::move(r));
  auto e = rs.encode(ec_cpp::Slice<uint8_t>(const_cast<uint8_t *>(p), len));
  if (ec_cpp::resultHasError(e)) return err_code(ec_cpp::resultGetError(std::move(e)));
  auto shards = ec_cpp::resultGetValue(std::move(e));
  size_t sl = shards.empty() ? 0 : shards[0].size();
  *shard_len = sl;
  if (cap < shards.size() * sl) return -1;
  for (size_t v = 0; v < shards.size(); ++v)
    std::memcpy(out + v * sl, shards[v].data(), sl);
  return 0;
}

// shards[i] == nullptr or lens[i] == 0: missing
int ecref_reconstruct(size_t nv, const uint8_t *const *sh, const size_t *lens,
                      size_t nr, uint8_t *out, size_t cap, size_t *out_len) {
  auto r = ec_cpp::create(nv);
  if (ec_cpp::resultHasError(r)) return err_code(ec_cpp::resultGetError(std::move(r)));
  auto rs = ec_cpp::resultGetValue(std::move(r));
  std::vector<Shard> rec(nr);
  for (size_t i = 0; i < nr; ++i)
    if (sh[i] && lens[i]) rec[i].assign(sh[i], sh[i] + lens[i]);
  auto d = rs.reconstruct(rec);
  if (ec_cpp::resultHasError(d)) return err_code(ec_cpp::resultGetError(std::move(d)));
  auto v = ec_cpp::resultGetValue(std::move(d));
  *out_len = v.size();
  if (cap < v.size()) return -1;
  std::memcpy(out, v.data(), v.size());
  return 0;
}

int ecref_reconstruct_from_systematic(size_t nv, const uint8_t *const *ch,
                                      const size_t *lens, size_t count,
                                      uint8_t *out, size_t cap,
                                      size_t *out_len) {
  auto r = ec_cpp::create(nv);
  if (ec_cpp::resultHasError(r)) return err_code(ec_cpp::resultGetError(std::move(r)));
  auto rs = ec_cpp::resultGetValue(std::move(r));
  std::vector<Shard> c(count);
  for (size_t i = 0; i < count; ++i) c[i].assign(ch[i], ch[i] + lens[i]);
  auto d = rs.reconstruct_from_systematic(c);
  if (ec_cpp::resultHasError(d)) return err_code(ec_cpp::resultGetError(std::move(d)));
  auto v = ec_cpp::resultGetValue(std::move(d));
  *out_len = v.size();
  if (cap < v.size()) return -1;
  std::memcpy(out, v.data(), v.size());
  return 0;
}

// Timed like benchmark/benchmark.cpp:84-101: encode once, then reconstruct
// from the shards flagged present.  Times exclude marshalling.
int ecref_time(size_t nv, const uint8_t *p, size_t len, const uint8_t *present,
               double *sec_enc, double *sec_dec) {
  using clk = std::chrono::steady_clock;
  auto r = ec_cpp::create(nv);
  if (ec_cpp::resultHasError(r)) return err_code(ec_cpp::resultGetError(std::move(r)));
  auto rs = ec_cpp::resultGetValue(std::move(r));
  auto t0 = clk::now();
  auto e = rs.encode(ec_cpp::Slice<uint8_t>(const_cast<uint8_t *>(p), len));
  auto t1 = clk::now();
  if (ec_cpp::resultHasError(e)) return err_code(ec_cpp::resultGetError(std::move(e)));
  auto shards = ec_cpp::resultGetValue(std::move(e));
  for (size_t i = 0; i < shards.size(); ++i)
    if (!present[i]) shards[i].clear();
  auto t2 = clk::now();
  auto d = rs.reconstruct(shards);
  auto t3 = clk::now();
  if (ec_cpp::resultHasError(d)) return err_code(ec_cpp::resultGetError(std::move(d)));
  *sec_enc = std::chrono::duration<double>(t1 - t0).count();
  *sec_dec = std::chrono::duration<double>(t3 - t2).count();
  return 0;
}

// All-core rate: `threads` threads, each encoding the payload
// and reconstructing it from the shards flagged present, one payload per
// thread at a time, until `seconds` have passed (ec-cpp's thread_local
// scratch, reed-solomon.hpp:198-201, makes concurrent calls safe).  *done =
// payloads completed by all threads; *wall = elapsed seconds; *enc / *dec =
// encode / reconstruct seconds summed over the threads.
int ecref_time_mt(size_t nv, const uint8_t *p, size_t len, const uint8_t *present, int threads,
                  double seconds, uint64_t *done, double *wall, double *enc, double *dec) {
  using clk = std::chrono::steady_clock;
  std::atomic<uint64_t> count{0};
  std::atomic<int> err{0};
  std::vector<double> te(threads, 0.0), td(threads, 0.0);
  const auto t0 = clk::now();
  const auto stop = t0 + std::chrono::duration<double>(seconds);
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t)
    pool.emplace_back([&, t] {
      std::vector<uint8_t> mine(p, p + len);  // each thread its own input
      do {
        double a = 0, b = 0;
        const int e = ecref_time(nv, mine.data(), len, present, &a, &b);
        if (e) {
          err = e;
          return;
        }
        te[t] += a;
        td[t] += b;
        ++count;
      } while (clk::now() < stop);
    });
  for (auto &th : pool) th.join();
  *wall = std::chrono::duration<double>(clk::now() - t0).count();
  *done = count.load();
  *enc = *dec = 0;
  for (int t = 0; t < threads; ++t) {
    *enc += te[t];
    *dec += td[t];
  }
  return err.load();
}

}  // extern "C"
