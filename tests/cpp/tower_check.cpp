// tower_check.cpp — CPU check of the tower-coordinate multiply tables
// (gf_field.hpp), built by tests/test_tower.py with g++ against
// erasure-coding-crust_amd/csrc/gf_field.cpp.  Emulates the device multiply
// forms (mul_acc: 12 v_perm, mul_acc_sub: 6 v_perm, mul_acc_f9: 9 v_perm,
// ec_device.hpp) byte for
// byte and checks every table kind against the field, and runs the additive
// FFT / IFFT (additive_fft.hpp:99-141) in tower coordinates with the tower
// image rule (ec_kernels.hpp tower_sub_min) against the plain transform.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "gf_field.hpp"

using namespace ecamd;

static int fails = 0;
#define CHECK(c, ...)                     \
  do {                                    \
    if (!(c)) {                           \
      if (fails++ < 10) {                 \
        std::printf("FAIL %s: ", #c);     \
        std::printf(__VA_ARGS__);         \
        std::printf("\n");                \
      }                                   \
    }                                     \
  } while (0)

// v_perm_b32(hi, lo, sel) for selector bytes 0..7
static uint32_t vperm(uint32_t hi, uint32_t lo, uint32_t sel) {
  const uint64_t t = (uint64_t(hi) << 32) | lo;
  uint32_t r = 0;
  for (int b = 0; b < 4; ++b) r |= uint32_t((t >> (8 * ((sel >> (8 * b)) & 7))) & 0xff) << (8 * b);
  return r;
}

static void mul_acc(uint32_t xl, uint32_t xh, const MulTab &T, uint32_t &yl, uint32_t &yh) {
  const uint64_t x = (uint64_t(xh) << 32) | xl, t3 = x >> 3, t6 = x >> 6;
  const uint32_t s0 = xl & 0x07070707u, s1 = uint32_t(t3) & 0x07070707u, s2 = uint32_t(t6) & 0x03030303u;
  const uint32_t s3 = xh & 0x07070707u, s4 = uint32_t(t3 >> 32) & 0x07070707u, s5 = uint32_t(t6 >> 32) & 0x03030303u;
  const uint32_t *w = T.w;
  yl ^= vperm(w[1], w[0], s0) ^ vperm(w[5], w[4], s1) ^ vperm(w[9], w[8], s3) ^ vperm(w[13], w[12], s4) ^
        vperm(w[16], w[16], s2) ^ vperm(w[18], w[18], s5);
  yh ^= vperm(w[3], w[2], s0) ^ vperm(w[7], w[6], s1) ^ vperm(w[11], w[10], s3) ^ vperm(w[15], w[14], s4) ^
        vperm(w[17], w[17], s2) ^ vperm(w[19], w[19], s5);
}

static void mul_acc_sub(uint32_t xl, uint32_t xh, const MulTabSub &T, uint32_t &yl, uint32_t &yh) {
  const uint64_t x = (uint64_t(xh) << 32) | xl, t3 = x >> 3, t6 = x >> 6;
  const uint32_t s0 = xl & 0x07070707u, s1 = uint32_t(t3) & 0x07070707u, s2 = uint32_t(t6) & 0x03030303u;
  const uint32_t s3 = xh & 0x07070707u, s4 = uint32_t(t3 >> 32) & 0x07070707u, s5 = uint32_t(t6 >> 32) & 0x03030303u;
  const uint32_t *w = T.w;
  yl ^= vperm(w[1], w[0], s0) ^ vperm(w[3], w[2], s1) ^ vperm(w[4], w[4], s2);
  yh ^= vperm(w[1], w[0], s3) ^ vperm(w[3], w[2], s4) ^ vperm(w[4], w[4], s5);
}

// F9 form (ec_device.hpp mul_acc_f9): low ^= c0 x0 ^ c1 beta x1,
// high ^= (c0 + c1 alpha) x1 ^ (x0 & m)
static void mul_acc_f9(uint32_t xl, uint32_t xh, const MulTabF9 &T, uint32_t &yl, uint32_t &yh) {
  const uint64_t x = (uint64_t(xh) << 32) | xl, t3 = x >> 3, t6 = x >> 6;
  const uint32_t s0 = xl & 0x07070707u, s1 = uint32_t(t3) & 0x07070707u, s2 = uint32_t(t6) & 0x03030303u;
  const uint32_t s3 = xh & 0x07070707u, s4 = uint32_t(t3 >> 32) & 0x07070707u, s5 = uint32_t(t6 >> 32) & 0x03030303u;
  const uint32_t *w = T.w;
  yl ^= vperm(w[1], w[0], s0) ^ vperm(w[3], w[2], s1) ^ vperm(w[4], w[4], s2) ^ vperm(w[6], w[5], s3) ^
        vperm(w[8], w[7], s4) ^ vperm(w[9], w[9], s5);
  yh ^= vperm(w[11], w[10], s3) ^ vperm(w[13], w[12], s4) ^ vperm(w[14], w[14], s5) ^ (xl & w[15]);
}

// one symbol through a multiply form (lane 0 of a byte-planar group)
template <typename T, typename M>
static uint16_t apply(M m, const T &tab, uint16_t x) {
  uint32_t yl = 0, yh = 0;
  m(x & 0xff, x >> 8, tab, yl, yh);
  return uint16_t((yl & 0xff) | ((yh & 0xff) << 8));
}

int main() {
  const Field &f = field();
  std::mt19937_64 rng(7);
  // the device constants of L equal the field's
  for (uint32_t i = 0; i < 8; ++i) CHECK(f.tower_l[1u << i] == kTowerL[i], "L bit %u", i);
  // the map is an involution, and the subfield is closed
  for (uint32_t x = 0; x < kFieldSize; ++x) CHECK(f.tower(f.tower(uint16_t(x))) == x, "x=%u", x);
  for (uint32_t a = 1; a < 256; a += 7)
    for (uint32_t b = 1; b < 256; ++b) CHECK(f.mul(uint16_t(a), f.log[b]) < 256, "a=%u b=%u", a, b);
  // every table kind against the field, at random symbols
  for (uint32_t c = 0; c < kFieldSize; c += (c < 300 ? 1 : 97)) {
    const uint32_t cl = c == 0 ? kZeroTab : c;  // also the zero table
    const MulTab tt = f.tower_tab(cl);
    for (int it = 0; it < 64; ++it) {
      const uint16_t x = uint16_t(rng());
      const uint16_t p = cl == kZeroTab ? 0 : f.mul(x, cl);
      CHECK(apply(mul_acc, f.mtab[cl], x) == p, "mtab c=%u", cl);
      CHECK(apply(mul_acc, f.mtab_tin[cl], x) == f.tower(p), "tin c=%u", cl);
      CHECK(apply(mul_acc, f.mtab_tout[cl], f.tower(x)) == p, "tout c=%u", cl);
      CHECK(apply(mul_acc, tt, f.tower(x)) == f.tower(p), "tower c=%u", cl);
    }
  }
  for (uint32_t e = 0; e < 256; ++e) {  // every subfield constant (e = 0: the zero table)
    const uint32_t cl = e == 0 ? kZeroTab : f.log[e];
    const MulTabSub st = f.sub_tab(cl);
    for (int it = 0; it < 256; ++it) {
      const uint16_t x = uint16_t(rng());
      const uint16_t p = e == 0 ? 0 : f.mul(x, cl);
      CHECK(apply(mul_acc_sub, st, f.tower(x)) == f.tower(p), "sub e=%u x=%u", e, x);
    }
  }
  // F9 tables: every constant whose high tower coordinate is 0 or 1
  int nf9 = 0;
  for (uint32_t e = 0; e < kFieldSize; e += (e < 1024 ? 1 : 61)) {  // by element value
    const uint32_t cl = e == 0 ? kZeroTab : f.log[e];
    MulTabF9 t9;
    const bool ok = f.f9_tab(cl, &t9);
    CHECK(ok == ((f.tower(uint16_t(e)) >> 8) <= 1), "f9 domain e=%u", e);
    if (!ok) continue;
    ++nf9;
    for (int it = 0; it < 16; ++it) {
      const uint16_t x = uint16_t(rng());
      const uint16_t p = cl == kZeroTab ? 0 : f.mul(x, cl);
      CHECK(apply(mul_acc_f9, t9, f.tower(x)) == f.tower(p), "f9 c=%u x=%u", cl, x);
    }
  }
  CHECK(nf9 >= 512, "f9 constants %d", nf9);
  // the F9 image rule (ec_kernels.hpp f9_slot): image 0's stage-1 entries
  // (i = 1 mod 4) and, in the encode's image, its stage-0 entries 256..510
  // have high tower coordinate <= 1
  for (uint32_t i = 0; i < 1023; ++i) {
    MulTabF9 t9;
    if (i % 4 == 1 || (i % 2 == 0 && i >= 256 && i < 512)) CHECK(f.f9_tab(f.skews[i], &t9), "f9 slot %u", i);
  }
  // the tower image rule: every entry at a stage >= tower_sub_min(q) is a
  // subfield skew (ec_kernels.hpp; mirrored here)
  const auto sub_min = [](int q) { return q == 0 ? 2 : q == 1 ? 3 : 4; };
  for (int q = 0; q < 4; ++q)
    for (uint32_t i = 0; i < 1023; ++i) {
      const uint32_t idx = 1024 * q + i, c = f.skews[idx];
      if (__builtin_ctz(idx + 1) >= sub_min(q)) CHECK(c == kZeroTab || f.exp[c] < 256, "q=%d i=%u", q, i);
    }
  // alias slots (enc_k256.hip PassIdx, dec_n1024.hip sub_alias): the skew of
  // position p at stage m of the transform at index off (a multiple of 2^(m+1))
  // has element 2 ((off | p) >> (m + 1)); the stage-2 slot
  // ((off | p) >> (m + 1)) << 3 | 3 holds the same element
  for (uint32_t m = 0; m < 10; ++m)
    for (uint32_t off = 0; off < 1024; off += (2u << m))
      for (uint32_t p = 0; p < 1024 && off + p < 1024; ++p) {
        const uint32_t h = (off | p) >> (m + 1);
        if (h >= 128 || (off & p)) continue;
        const uint32_t d = 1u << m, idx = ((off | p) & ~(2 * d - 1)) + d - 1, al = (h << 3) | 3;
        const uint32_t c0 = f.skews[idx], c1 = f.skews[al];
        const uint32_t e0 = c0 == kZeroTab ? 0 : f.exp[c0], e1 = c1 == kZeroTab ? 0 : f.exp[c1];
        CHECK(e0 == e1 && e0 == 2 * h && __builtin_ctz(al + 1) == 2, "alias m=%u off=%u p=%u", m, off, p);
      }
  // reconstruct_n4096's cross-quarter skews (dec_n4096.hip n4096_lin) are subfield
  for (uint32_t i : {1023u, 2047u, 3071u}) CHECK(f.skews[i] == kZeroTab || f.exp[f.skews[i]] < 256, "skew %u", i);
  // IFFT / FFT of size 1024 at index 1024 q (additive_fft.hpp:99-141), in
  // symbols with mtab and in tower coordinates with the image rule
  for (int q = 0; q < 4; ++q)
    for (int inverse = 0; inverse < 2; ++inverse) {
      const uint32_t n = 1024, index = 1024 * q;
      std::vector<uint16_t> a(n), t(n);
      for (uint32_t i = 0; i < n; ++i) {
        a[i] = uint16_t(rng());
        t[i] = f.tower(a[i]);
      }
      std::vector<uint16_t> t9 = t;  // tower coordinates, F9 tables at the encode image's F9 slots
      const auto mulp = [&](uint16_t x, uint32_t skew_i, int tower) -> uint16_t {
        const uint32_t c = f.skews[skew_i], i = skew_i - index;
        if (!tower) return apply(mul_acc, f.mtab[c], x);
        if (__builtin_ctz(skew_i + 1) >= sub_min(q)) return apply(mul_acc_sub, f.sub_tab(c), x);
        MulTabF9 tf;
        if (tower == 2 && q == 0 && (i % 4 == 1 || (i % 2 == 0 && i >= 256 && i < 512)) && f.f9_tab(c, &tf))
          return apply(mul_acc_f9, tf, x);
        return apply(mul_acc, f.tower_tab(c), x);
      };
      for (int tw = 0; tw < 3; ++tw) {
        std::vector<uint16_t> &d = tw == 2 ? t9 : tw ? t : a;
        if (inverse) {
          for (uint32_t dep = 1; dep < n; dep <<= 1)
            for (uint32_t j = dep; j < n; j += 2 * dep) {
              for (uint32_t i = j - dep; i < j; ++i) d[i + dep] ^= d[i];
              for (uint32_t i = j - dep; i < j; ++i) d[i] ^= mulp(d[i + dep], j + index - 1, tw);
            }
        } else {
          for (uint32_t dep = n >> 1; dep > 0; dep >>= 1)
            for (uint32_t j = dep; j < n; j += 2 * dep) {
              for (uint32_t i = j - dep; i < j; ++i) d[i] ^= mulp(d[i + dep], j + index - 1, tw);
              for (uint32_t i = j - dep; i < j; ++i) d[i + dep] ^= d[i];
            }
        }
      }
      for (uint32_t i = 0; i < n; ++i) CHECK(f.tower(t[i]) == a[i], "fft q=%d inv=%d i=%u", q, inverse, i);
      for (uint32_t i = 0; i < n; ++i) CHECK(t9[i] == t[i], "f9 fft q=%d inv=%d i=%u", q, inverse, i);
    }
  if (fails) {
    std::printf("%d failures\n", fails);
    return 1;
  }
  std::printf("tower tables ok\n");
  return 0;
}
