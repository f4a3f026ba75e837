#!/usr/bin/env python3
"""A/B variant of encode_k256w: the subfield tables' last dword (plane 1,
dword 0 of a 16-B slot, kCImgSub1) read from a packed 4-B-stride copy after
the LDS slot word, so that the ds_read_b32 of pass A's 32 distinct entries is
conflict free instead of 4-way (one extra shift per table).  Valid only for
the k = 256, n = 1024 encode (the other encodes read the unpacked plane).

  enc_sub1p.py OUT_DIR   -> OUT_DIR/enc_k256w.hip, OUT_DIR/cimg.hpp
Build: scripts/build_var.sh NAME "" enc_k256w.hip=OUT_DIR/enc_k256w.hip cimg.hpp=OUT_DIR/cimg.hpp"""
import sys

ROOT = __file__.rsplit("/scripts/", 1)[0]
out = sys.argv[1]


def rep(s, old, new):
    assert old in s, old[:80]
    return s.replace(old, new, 1)


c = open(f"{ROOT}/erasure-coding-crust_amd/csrc/cimg.hpp").read()
c = rep(c, "  T.t[4] = lds_r32(a + kCImgSub1);", "  T.t[4] = lds_r32(kSub1Packed + (a >> 2));")
c = rep(c, "namespace {\n", "namespace {\n\nconstexpr uint32_t kSub1Packed = kCImgBytes + 8 * 4096 + 16;\n")
open(f"{out}/cimg.hpp", "w").write(c)

k = open(f"{ROOT}/erasure-coding-crust_amd/csrc/enc_k256w.hip").read()
k = rep(k, "constexpr int LDS_BYTES = int(SLOT + 16);", "constexpr int LDS_BYTES = int(SLOT + 16 + 512);\n"
        "static_assert(SLOT + 16 == kSub1Packed, \"packed plane after the slot\");")
k = rep(k, "    for (int k = 0; k < kPer; ++k) reinterpret_cast<v4u *>(lds)[tid0 + k * THREADS] = v[k];\n",
        "    for (int k = 0; k < kPer; ++k) reinterpret_cast<v4u *>(lds)[tid0 + k * THREADS] = v[k];\n"
        "    if (tid0 < 128) reinterpret_cast<uint32_t *>(lds + kSub1Packed)[tid0] =\n"
        "        reinterpret_cast<const uint32_t *>(cimg + kCImgSub1)[4 * tid0];\n")
open(f"{out}/enc_k256w.hip", "w").write(k)
