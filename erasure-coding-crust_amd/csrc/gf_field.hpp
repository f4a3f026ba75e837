// gf_field.hpp — host-side GF(2^16) field description for the NPB codec.
//
// The field, its relabelled LOG/EXP tables and the additive-FFT skews are
// defined by include/ec-cpp/f2e16.hpp:25-94 and additive_fft.hpp:45-97 of the
// reference; this is an independent builder that produces the same values
// (pinned by tests/test_capi_cpu.py against tests/golden/tables.json).
//
// The device never sees LOG/EXP: every multiply-by-constant runs through a
// MulTab, a 20-dword v_perm lookup table per log-domain constant (see
// ec_device.hpp for the byte-planar kernel arithmetic).
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

namespace ecamd {

constexpr uint32_t kFieldSize = 65536;
constexpr uint32_t kOneMask = 65535;

// 80-byte multiply table for one constant c (log domain).  The 16-bit symbol
// x = xH:xL is split into 3-bit groups xL[0:3) xL[3:6) xH[0:3) xH[3:6) and
// 2-bit groups xL[6:8) xH[6:8); each group value indexes an 8- (or 4-) entry
// byte table of the partial product's low (L) and high (H) byte.
//   w[0..3]  : group xL[0:3)   {L.lo, L.hi, H.lo, H.hi}
//   w[4..7]  : group xL[3:6)
//   w[8..11] : group xH[0:3)
//   w[12..15]: group xH[3:6)
//   w[16..19]: {L(xL[6:8)), H(xL[6:8)), L(xH[6:8)), H(xH[6:8))}
struct MulTab {
  uint32_t w[20];
};
static_assert(sizeof(MulTab) == 80, "MulTab layout");

// Index of the all-zero table: skews equal to 0xFFFF (log of the element 0)
// mean "no multiply" in additive_fft.hpp:110,129 == multiply by zero.
constexpr uint32_t kZeroTab = 65535;

// Tower coordinates.  The symbols < 256 are the subfield
// GF(2^8) (closed under the reference's multiplication), and with w = 0x100
// every symbol is x0 + x1 * w, x0, x1 < 256, where x1 = x >> 8 and
// x0 = (x & 0xFF) ^ L(x >> 8) for the GF(2)-linear L below; the map
// x -> x0 | x1 << 8 is therefore x ^ L(x >> 8), its own inverse.  A multiply by
// a subfield constant c acts on tower coordinates bytewise: (c x0, c x1).
// Addition (XOR) is the same in both coordinates, so an FFT runs unchanged in
// tower coordinates as long as its multiply tables are conjugated by the map.
//
// Subfield table of a constant c (log domain, g^c < 256), 5 dwords: byte e of
// w[0..1] = (e) * g^c, of w[2..3] = (e << 3) * g^c, of w[4] = (e << 6) * g^c.
// L on bit i of the high byte (w = 0x100): the device conversion
// (ec_device.hpp tower_lo) is compiled from these; build_mtab derives L from
// the field and tests/cpp/tower_check.cpp checks that the two agree
constexpr uint8_t kTowerL[8] = {0x00, 0xcf, 0xab, 0x21, 0x8a, 0x9d, 0x27, 0x1f};

struct MulTabSub {
  uint32_t w[5];
};

// "F9" table of a constant g^c whose tower coordinates are c0 + c1 w with
// c1 in {0, 1}: with w^2 = alpha w + beta,
//   (x0 + x1 w)(c0 + c1 w) = (c0 x0 + c1 beta x1) + ((c0 + c1 alpha) x1 + c1 x0) w,
// three subfield tables and a mask (9 v_perm instead of 12):
// w[0..4] = sub table of c0, w[5..9] = of c1 beta, w[10..14] = of c0 + c1 alpha,
// w[15] = c1 ? ~0 : 0.  In a tower image slot: plane q holds w[4q .. 4q + 3].
struct MulTabF9 {
  uint32_t w[16];
};

struct Field {
  std::vector<uint16_t> log, exp, log_walsh;  // 65536 each (f2e16.hpp:48-84)
  std::vector<uint16_t> skews;                // 65535 (additive_fft.hpp:47-97)
  std::vector<MulTab> mtab;                   // 65536: [c] = *g^c, [65535] = *0
  // tower-coordinate variants (65536 each, [65535] = *0): x -> T(x * g^c)
  // (symbols in, tower out) and x -> T(x) * g^c (tower in, symbols out)
  std::vector<MulTab> mtab_tin, mtab_tout;
  uint8_t tower_l[256];  // L on a high byte

  uint16_t tower(uint16_t x) const { return uint16_t(x ^ tower_l[x >> 8]); }
  // general table of x -> T(T(x) * g^c) (tower in and out)
  MulTab tower_tab(uint32_t c) const;
  MulTabSub sub_tab(uint32_t c) const;  // requires g^c < 256 (or c = 65535)
  // requires (tower(g^c) >> 8) <= 1; returns false (and leaves t) otherwise
  bool f9_tab(uint32_t c, MulTabF9 *t) const;

  uint16_t mul(uint16_t x, uint32_t log_c) const {
    if (x == 0) return 0;
    uint32_t l = uint32_t(log[x]) + log_c;
    return exp[(l & 0xffff) + (l >> 16)];
  }
  // F[lo] = sum_hi LOG_WALSH[hi*n + lo] mod 65535: folds the 65536-point
  // error-locator transform onto n points (exactness: DESIGN.md §error locator).
  std::vector<uint16_t> fold_log_walsh(uint32_t n) const;
};

const Field &field();  // built once, thread-safe

// math.hpp:25-36, ec-cpp.cpp:15-37, reed-solomon.hpp:24-45,191-196
struct CodeParams {
  uint32_t nv = 0, n = 0, k = 0, threshold = 0;
};
enum class ParamError { kOk, kTooManyValidators, kNotEnoughValidators };
ParamError code_params(unsigned long n_validators, CodeParams *out);
inline size_t shard_len(uint32_t k, size_t payload_len) {
  size_t syms = (payload_len + 1) / 2;
  return (syms + k - 1) / k * 2;
}

}  // namespace ecamd
