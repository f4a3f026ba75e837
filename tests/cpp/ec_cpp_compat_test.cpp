// Drives the ec-cpp source-compatible header exactly as the reference's own
// tests use ec-cpp (test/erasure_coding/reconstruct.cpp): create -> encode ->
// reconstruct / reconstruct_from_systematic, plus the ec-cpp error cases.
// Usage: ec_cpp_compat_test <payload file> <n_validators> <keep file> <out dir>
//   keep file: one shard index per line (the shards handed to reconstruct)
//   writes <out>/shards.bin (all shards concatenated), rec.bin, sys.bin
// Prints "ERR <name> ok" per error case and "DONE" at the end; exit 0 on success.
#include <ec-cpp/ec-cpp.hpp>

#include <cstdio>
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

static bool expect(const char *name, bool cond) {
  std::printf("ERR %s %s\n", name, cond ? "ok" : "FAILED");
  return cond;
}

static void write_file(const std::string &path, const std::vector<uint8_t> &b) {
  std::ofstream(path, std::ios::binary).write(reinterpret_cast<const char *>(b.data()), b.size());
}

int main(int argc, char **argv) {
  if (argc != 5) return 2;
  std::ifstream pf(argv[1], std::ios::binary);
  std::vector<uint8_t> payload((std::istreambuf_iterator<char>(pf)), {});
  const size_t nv = std::stoul(argv[2]);
  std::vector<size_t> keep;
  std::ifstream kf(argv[3]);
  for (size_t v; kf >> v;) keep.push_back(v);
  const std::string out = argv[4];

  auto created = ec_cpp::create(nv);
  if (ec_cpp::resultHasError(created)) return 3;
  auto encoder = ec_cpp::resultGetValue(std::move(created));
  auto enc = encoder.encode(ec_cpp::Slice<uint8_t>(payload.data(), payload.size()));
  if (ec_cpp::resultHasError(enc)) return 4;
  auto shards = ec_cpp::resultGetValue(std::move(enc));
  std::vector<uint8_t> flat;
  for (auto &s : shards) flat.insert(flat.end(), s.begin(), s.end());
  write_file(out + "/shards.bin", flat);

  std::vector<ec_cpp::ReedSolomon<ec_cpp::PolyEncoder_f2e16>::Shard> received(nv);
  for (size_t v : keep) received[v] = shards[v];
  auto rec = encoder.reconstruct(received);
  if (ec_cpp::resultHasError(rec)) return 5;
  write_file(out + "/rec.bin", ec_cpp::resultGetValue(std::move(rec)));

  std::vector<ec_cpp::ReedSolomon<ec_cpp::PolyEncoder_f2e16>::Shard> sys(shards.begin(),
                                                                         shards.begin() + encoder.k());
  auto srec = encoder.reconstruct_from_systematic(sys);
  if (ec_cpp::resultHasError(srec)) return 6;
  write_file(out + "/sys.bin", ec_cpp::resultGetValue(std::move(srec)));

  bool ok = true;
  auto e1 = ec_cpp::create(1);
  ok &= expect("create1", ec_cpp::resultHasError(e1) &&
                              ec_cpp::resultGetError(std::move(e1)) == ec_cpp::Error::kNotEnoughValidators);
  auto e2 = ec_cpp::create(65537);
  ok &= expect("create65537", ec_cpp::resultHasError(e2) &&
                                  ec_cpp::resultGetError(std::move(e2)) == ec_cpp::Error::kTooManyValidators);
  auto e3 = encoder.encode(ec_cpp::Slice<uint8_t>(payload.data(), 0));
  ok &= expect("empty", ec_cpp::resultHasError(e3) &&
                            ec_cpp::resultGetError(std::move(e3)) == ec_cpp::Error::kPayloadSizeIsZero);
  std::vector<ec_cpp::ReedSolomon<ec_cpp::PolyEncoder_f2e16>::Shard> few(nv);
  for (size_t v = 0; v + 1 < encoder.k(); ++v) few[v] = shards[v];
  auto e4 = encoder.reconstruct(few);
  ok &= expect("fewer_than_k", ec_cpp::resultHasError(e4) &&
                                   ec_cpp::resultGetError(std::move(e4)) == ec_cpp::Error::kNeedMoreShards);
  auto bad = received;
  for (auto &s : bad)
    if (!s.empty()) {
      s.push_back(0);
      s.push_back(0);
      break;
    }
  auto e5 = encoder.reconstruct(bad);
  ok &= expect("inconsistent", ec_cpp::resultHasError(e5) &&
                                   ec_cpp::resultGetError(std::move(e5)) ==
                                       ec_cpp::Error::kInconsistentShardLengths);
  auto empty_sys = sys;
  empty_sys[0].clear();
  auto e6 = encoder.reconstruct_from_systematic(empty_sys);
  ok &= expect("empty_shard", ec_cpp::resultHasError(e6) &&
                                  ec_cpp::resultGetError(std::move(e6)) == ec_cpp::Error::kEmptyShard);
  std::printf("n=%zu k=%zu DONE\n", encoder.n(), encoder.k());
  return ok ? 0 : 7;
}
