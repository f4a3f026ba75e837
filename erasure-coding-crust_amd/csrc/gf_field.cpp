// gf_field.cpp — builds the field tables, skews and v_perm multiply tables.
#include "gf_field.hpp"

#include <mutex>

namespace ecamd {
namespace {

// Cantor-style relabelling basis, include/ec-cpp/f2e16.hpp:36-38
constexpr uint16_t kBase[16] = {1,     44234, 15374, 5694,  50562, 60718, 37196, 16402,
                                27800, 4312,  27250, 47360, 64952, 64308, 65336, 39198};
constexpr uint32_t kGeneratorTaps = 0x2D;  // f2e16.hpp:34

void walsh_mod(std::vector<uint16_t> &d, size_t size) {  // walsh.hpp:15-39
  for (size_t h = 1; h < size; h <<= 1)
    for (size_t b = 0; b < size; b += 2 * h)
      for (size_t i = b; i < b + h; ++i) {
        uint32_t x = d[i], y = d[i + h];
        uint32_t s = x + y, t = x + kOneMask - y;
        d[i] = uint16_t((s & 0xffff) + (s >> 16));
        d[i + h] = uint16_t((t & 0xffff) + (t >> 16));
      }
}

void build_tables(Field &f) {
  f.log.assign(kFieldSize, 0);
  f.exp.assign(kFieldSize, 0);
  // discrete logs of polynomial-basis elements via the LFSR
  std::vector<uint16_t> plog(kFieldSize, 0);
  uint32_t st = 1;
  for (uint32_t e = 0; e < kOneMask; ++e) {
    plog[st] = uint16_t(e);
    st <<= 1;
    if (st >> 16) st = (st & 0xffff) ^ kGeneratorTaps;
  }
  plog[0] = uint16_t(kOneMask);
  // relabel: element x <-> polynomial element L(x) = XOR of kBase over bits of x
  std::vector<uint16_t> lin(kFieldSize, 0);
  for (uint32_t b = 0; b < 16; ++b)
    for (uint32_t j = 0; j < (1u << b); ++j) lin[j | (1u << b)] = lin[j] ^ kBase[b];
  for (uint32_t x = 0; x < kFieldSize; ++x) f.log[x] = plog[lin[x]];
  for (uint32_t x = 0; x < kFieldSize; ++x) f.exp[f.log[x]] = uint16_t(x);
  f.exp[kOneMask] = f.exp[0];
  f.log_walsh = f.log;
  f.log_walsh[0] = 0;
  walsh_mod(f.log_walsh, kFieldSize);
}

void build_skews(Field &f) {  // additive_fft.hpp:47-97
  std::vector<uint16_t> elem(kOneMask, 0);
  uint16_t basis[15];
  for (int i = 0; i < 15; ++i) basis[i] = uint16_t(2u << i);
  for (uint32_t m = 0; m < 15; ++m) {
    elem[(1u << m) - 1] = 0;
    for (uint32_t i = m; i < 15; ++i) {
      const uint32_t span = 2u << i;
      for (uint32_t j = (1u << m) - 1; j < span; j += 2u << m) elem[j + span] = elem[j] ^ basis[i];
    }
    const uint16_t v = f.mul(basis[m], f.log[basis[m] ^ 1]);
    basis[m] = uint16_t(kOneMask - f.log[v]);
    for (uint32_t i = m + 1; i < 15; ++i) {
      const uint32_t c = (uint32_t(f.log[basis[i] ^ 1]) + basis[m]) % kOneMask;
      basis[i] = f.mul(basis[i], c);
    }
  }
  f.skews.resize(kOneMask);
  for (uint32_t i = 0; i < kOneMask; ++i) f.skews[i] = f.log[elem[i]];
}

// byte table of 4 entries: entry e = selected byte of f((first + e) << pos)
template <typename F>
uint32_t pack4(F f, uint32_t pos, uint32_t first, bool high) {
  uint32_t w = 0;
  for (uint32_t e = 0; e < 4; ++e) {
    const uint16_t p = f(uint16_t((first + e) << pos));
    w |= uint32_t(high ? (p >> 8) : (p & 0xff)) << (8 * e);
  }
  return w;
}

// v_perm table set (MulTab layout) of any GF(2)-linear map f on symbols
template <typename F>
MulTab make_tab(F f) {
  MulTab t;
  const uint32_t pos3[4] = {0, 3, 8, 11};
  for (int g = 0; g < 4; ++g) {
    t.w[4 * g + 0] = pack4(f, pos3[g], 0, false);
    t.w[4 * g + 1] = pack4(f, pos3[g], 4, false);
    t.w[4 * g + 2] = pack4(f, pos3[g], 0, true);
    t.w[4 * g + 3] = pack4(f, pos3[g], 4, true);
  }
  t.w[16] = pack4(f, 6, 0, false);
  t.w[17] = pack4(f, 6, 0, true);
  t.w[18] = pack4(f, 14, 0, false);
  t.w[19] = pack4(f, 14, 0, true);
  return t;
}

void build_mtab(Field &f) {
  // L(bit i of the high byte) = 2^(8+i) + 2^i * w, w = 0x100 (gf_field.hpp)
  uint8_t lb[8];
  for (uint32_t i = 0; i < 8; ++i) {
    const uint32_t v = (1u << (8 + i)) ^ f.mul(uint16_t(1u << i), f.log[0x100]);
    lb[i] = uint8_t(v);  // v < 256: the subfield part (checked by tests/cpp/tower_check.cpp)
  }
  for (uint32_t h = 0; h < 256; ++h) {
    uint8_t l = 0;
    for (uint32_t i = 0; i < 8; ++i)
      if ((h >> i) & 1) l ^= lb[i];
    f.tower_l[h] = l;
  }
  f.mtab.resize(kFieldSize);
  f.mtab_tin.resize(kFieldSize);
  f.mtab_tout.resize(kFieldSize);
  for (uint32_t c = 0; c < kFieldSize; ++c) {
    const bool zero = (c == kZeroTab);
    const Field &cf = f;
    f.mtab[c] = make_tab([&](uint16_t x) { return zero ? uint16_t(0) : cf.mul(x, c); });
    f.mtab_tin[c] = make_tab([&](uint16_t x) { return zero ? uint16_t(0) : cf.tower(cf.mul(x, c)); });
    f.mtab_tout[c] = make_tab([&](uint16_t x) { return zero ? uint16_t(0) : cf.mul(cf.tower(x), c); });
  }
}

}  // namespace

MulTab Field::tower_tab(uint32_t c) const {
  if (c == kZeroTab) return mtab[kZeroTab];
  return make_tab([&](uint16_t x) { return tower(mul(tower(x), c)); });
}

MulTabSub Field::sub_tab(uint32_t c) const {
  MulTabSub t;
  const auto f = [&](uint16_t x) { return c == kZeroTab ? uint16_t(0) : mul(x, c); };  // < 256 for x < 256
  t.w[0] = pack4(f, 0, 0, false);
  t.w[1] = pack4(f, 0, 4, false);
  t.w[2] = pack4(f, 3, 0, false);
  t.w[3] = pack4(f, 3, 4, false);
  t.w[4] = pack4(f, 6, 0, false);
  return t;
}

bool Field::f9_tab(uint32_t c, MulTabF9 *t) const {
  const uint16_t e = c == kZeroTab ? uint16_t(0) : exp[c];
  const uint16_t te = tower(e), w2 = tower(mul(0x100, log[0x100]));  // tower(0x100) = 0x100
  const uint32_t c0 = te & 0xff, c1 = te >> 8, beta = w2 & 0xff, alpha = w2 >> 8;
  if (c1 > 1) return false;
  const auto lg = [&](uint32_t v) { return v == 0 ? kZeroTab : uint32_t(log[v]); };
  const MulTabSub a = sub_tab(lg(c0)), b = sub_tab(lg(c1 ? beta : 0)), d = sub_tab(lg(c0 ^ (c1 ? alpha : 0)));
  for (int i = 0; i < 5; ++i) {
    t->w[i] = a.w[i];
    t->w[5 + i] = b.w[i];
    t->w[10 + i] = d.w[i];
  }
  t->w[15] = c1 ? 0xffffffffu : 0u;
  return true;
}

std::vector<uint16_t> Field::fold_log_walsh(uint32_t n) const {
  std::vector<uint16_t> F(n);
  for (uint32_t lo = 0; lo < n; ++lo) {
    uint64_t s = 0;
    for (uint32_t hi = 0; hi < kFieldSize / n; ++hi) s += log_walsh[hi * n + lo];
    F[lo] = uint16_t(s % kOneMask);
  }
  return F;
}

const Field &field() {
  static Field f;
  static std::once_flag once;
  std::call_once(once, [] {
    build_tables(f);
    build_skews(f);
    build_mtab(f);
  });
  return f;
}

ParamError code_params(unsigned long nv, CodeParams *out) {
  if (nv > kFieldSize) return ParamError::kTooManyValidators;
  if (nv <= 1) return ParamError::kNotEnoughValidators;
  const uint32_t thr = uint32_t((nv - 1) / 3 + 1);
  uint32_t n = 1;
  while (n < nv) n <<= 1;
  uint32_t k = 1;
  while ((k << 1) <= thr) k <<= 1;  // largest power of two <= thr
  out->nv = uint32_t(nv);
  out->n = n;
  out->k = k;
  out->threshold = thr;
  return ParamError::kOk;
}

}  // namespace ecamd
