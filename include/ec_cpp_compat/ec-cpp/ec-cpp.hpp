// ec-cpp source-compatible front end over the MI355X library (SURVEY.md §8f
// row 4).  Put `include/ec_cpp_compat` ahead of the reference's include
// directory and link `liberasure_coding_crust.so`: code written against
// ec-cpp (`ec_cpp::create`, `ReedSolomon<PolyEncoder_f2e16>::encode /
// reconstruct / reconstruct_from_systematic`, `Result` helpers) compiles
// unchanged and runs on the GPU path, byte-identical to ec-cpp.
//
// Mirrors include/ec-cpp/ec-cpp.hpp:15-26, errors.hpp, types.hpp and the
// public surface of reed-solomon.hpp:24-185, including its validation order
// and error values.  Differences, both outside ec-cpp's contract:
//  * a missing or failing HIP device throws std::runtime_error (ec-cpp has no
//    runtime failure mode; the GPU path has no CPU fallback by design);
//  * non-empty shards at positions >= n_validators (which ec-cpp's encode never
//    produces) are treated as erased.
// C++20 (std::span), as the reference.
#ifndef ERASURE_CODING_CRUST_AMD_EC_CPP_COMPAT_HPP
#define ERASURE_CODING_CRUST_AMD_EC_CPP_COMPAT_HPP

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <span>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <variant>
#include <vector>

#include "../../erasure_coding/ec_amd.h"

namespace ec_cpp {

// errors.hpp (same enumerators, same order)
enum struct Error {
  kArgsMustBePowOf2,
  kWantedShardCountTooLow,
  kWantedShardCountTooHigh,
  kWantedPayloadShardCountTooLow,
  kPayloadSizeIsZero,
  kTooManyValidators,
  kNotEnoughValidators,
  kNeedMoreShards,
  kInconsistentShardLengths,
  kEmptyShard,
};

template <typename T>
using Result = std::variant<T, Error>;

template <typename T>
bool resultHasError(const Result<T> &r) {
  return r.index() == 1;
}
template <typename T>
Error resultGetError(Result<T> &&r) {
  return std::get<Error>(std::move(r));
}
template <typename T>
T resultGetValue(Result<T> &&r) {
  return std::get<T>(std::move(r));
}

// types.hpp
template <typename T>
using Slice = std::span<std::remove_reference_t<T>>;

// The GF(2^16) field is fixed on the device path; the tag keeps the
// `ReedSolomon<PolyEncoder_f2e16>` spelling valid.
struct f2e16_Descriptor {
  static constexpr size_t kFieldSize = 65536;
};
template <typename Descriptor>
struct PolyEncoder {
  using DescriptorType = Descriptor;
};
using PolyEncoder_f2e16 = PolyEncoder<f2e16_Descriptor>;

namespace amd_detail {
[[noreturn]] inline void device_failure(const char *what) {
  throw std::runtime_error(std::string("ec_cpp (MI355X): ") + what + ": " +
                           ECCR_AMD_last_error());
}
}  // namespace amd_detail

template <typename TPolyEncoder>
struct ReedSolomon final {
  using Shard = std::vector<uint8_t>;

  // reed-solomon.hpp:24-45 (n = po2 >= wanted, k = po2 <= threshold)
  static Result<ReedSolomon> create(size_t n, size_t k, const TPolyEncoder & = TPolyEncoder{}) {
    if (n < 2) return Error::kWantedShardCountTooLow;
    if (k < 1) return Error::kWantedPayloadShardCountTooLow;
    size_t k_po2 = 1, n_po2 = 1;
    while (k_po2 * 2 <= k) k_po2 *= 2;
    while (n_po2 < n) n_po2 *= 2;
    if (n_po2 > f2e16_Descriptor::kFieldSize) return Error::kWantedShardCountTooHigh;
    return ReedSolomon{n_po2, k_po2, n};
  }

  // reed-solomon.hpp:47-81
  Result<std::vector<Shard>> encode(const Slice<uint8_t> bytes) {
    if (bytes.empty()) return Error::kPayloadSizeIsZero;
    const size_t sl = shardLen(bytes.size());
    std::vector<uint8_t> flat(wanted_n_ * sl);
    const NPRSResult r = ECCR_AMD_encode_host_batch(wanted_n_, bytes.data(), bytes.size(),
                                                    bytes.size(), 1, flat.data(), sl, 1);
    if (r.tag != NPRS_RESULT_OK) amd_detail::device_failure("encode");
    std::vector<Shard> shards(wanted_n_);
    for (size_t v = 0; v < wanted_n_; ++v)
      shards[v].assign(flat.begin() + v * sl, flat.begin() + (v + 1) * sl);
    return shards;
  }

  // reed-solomon.hpp:83-134: positional shards, empty = missing; entries past
  // the end are erased; lengths compare as size()/2 symbols
  Result<std::vector<uint8_t>> reconstruct(const std::vector<Shard> &received_shards) {
    const size_t upto = std::min(n_, received_shards.size());
    size_t existential = 0, syms = 0;
    bool have = false;
    for (size_t i = 0; i < upto; ++i) {
      const Shard &s = received_shards[i];
      if (s.empty()) continue;
      ++existential;
      if (!have) {
        syms = s.size() / 2;
        have = true;
      } else if (syms != s.size() / 2) {
        return Error::kInconsistentShardLengths;
      }
    }
    if (existential < k_) return Error::kNeedMoreShards;
    const size_t sl = syms * 2;
    std::vector<uint16_t> idx;
    std::vector<uint8_t> comp;
    idx.reserve(existential);
    comp.reserve(existential * sl);
    for (size_t i = 0; i < std::min(upto, wanted_n_); ++i) {
      const Shard &s = received_shards[i];
      if (s.empty()) continue;
      idx.push_back(static_cast<uint16_t>(i));
      comp.insert(comp.end(), s.begin(), s.begin() + sl);
    }
    std::vector<uint8_t> out(sl * k_);
    if (idx.size() < k_) return Error::kNeedMoreShards;
    if (sl == 0) return out;  // zero-symbol shards: ec-cpp returns an empty buffer
    const NPRSResult r = ECCR_AMD_reconstruct_host_batch(wanted_n_, comp.data(), sl, sl,
                                                         idx.data(), idx.size(), 1, out.data(),
                                                         out.size(), 1);
    if (r.tag != NPRS_RESULT_OK) amd_detail::device_failure("reconstruct");
    return out;
  }

  // reed-solomon.hpp:143-179: the first k entries are the systematic shards;
  // every entry's length is checked
  Result<std::vector<uint8_t>> reconstruct_from_systematic(const std::vector<Shard> &chunks) {
    if (chunks.empty() || chunks.size() < k_) return Error::kNeedMoreShards;
    const size_t syms = chunks[0].size() / 2;
    if (syms == 0) return Error::kEmptyShard;
    for (const Shard &c : chunks)
      if (c.size() / 2 != syms) return Error::kInconsistentShardLengths;
    std::vector<Chunk> list(k_);
    for (size_t y = 0; y < k_; ++y) {
      list[y].data.array = const_cast<uint8_t *>(chunks[y].data());
      list[y].data.length = syms * 2;
      list[y].index = y;
    }
    const ChunksList in{list.data(), static_cast<unsigned long>(k_)};
    DataBlock blk{nullptr, 0};
    const NPRSResult r = ECCR_reconstruct_from_systematic(wanted_n_, &in, &blk);
    if (r.tag != NPRS_RESULT_OK) amd_detail::device_failure("reconstruct_from_systematic");
    std::vector<uint8_t> out(blk.array, blk.array + blk.length);
    ECCR_deallocate_data_block(&blk);
    return out;
  }

  size_t n() const { return n_; }
  size_t k() const { return k_; }

 private:
  ReedSolomon(size_t n, size_t k, size_t wanted_n) : n_(n), k_(k), wanted_n_(wanted_n) {}

  size_t shardLen(size_t payload_size) const {  // reed-solomon.hpp:191-196
    return ((payload_size + 1) / 2 + k_ - 1) / k_ * 2;
  }

  size_t n_, k_, wanted_n_;
};

// ec-cpp.cpp:15-37
inline Result<size_t> getRecoveryThreshold(size_t n_validators) {
  if (n_validators > f2e16_Descriptor::kFieldSize) return Error::kTooManyValidators;
  if (n_validators <= 1) return Error::kNotEnoughValidators;
  return (n_validators - 1) / 3 + 1;
}

inline Result<ReedSolomon<PolyEncoder_f2e16>> create(size_t n_validators) {
  auto k = getRecoveryThreshold(n_validators);
  if (resultHasError(k)) return resultGetError(std::move(k));
  return ReedSolomon<PolyEncoder_f2e16>::create(n_validators, resultGetValue(std::move(k)));
}

}  // namespace ec_cpp

#endif  // ERASURE_CODING_CRUST_AMD_EC_CPP_COMPAT_HPP
