#!/usr/bin/env python3
"""A/B variant of reconstruct_n1024x: phase 5's received rows staged in LDS by
the gather (the raw 96-B row segment of every present row y < 256, in the
32 KB the compact image freed) instead of re-read from the shards into
registers held across the IFFT.  Row slot ((y & 3) << 6 | y >> 2) at a 112-B
pitch: phase 5's reads (y = 4 lane + q) are 2-way at most.

  n1024x_stage.py OUT.hip
Build: scripts/build_var.sh NAME "" dec_n1024x.hip=OUT.hip"""
import sys

ROOT = __file__.rsplit("/scripts/", 1)[0]
s = open(f"{ROOT}/erasure-coding-crust_amd/csrc/dec_n1024x.hip").read()


def rep(s, old, new):
    assert old in s, old[:80]
    return s.replace(old, new, 1)


s = rep(s, "constexpr uint32_t SLOT = uint32_t(TAB_REGION + WAVES * REG_BYTES);",
        "constexpr uint32_t STG = uint32_t(TAB_REGION + WAVES * REG_BYTES);  // phase 5's received rows\n"
        "constexpr uint32_t STG_PITCH = 112;\n"
        "__device__ __forceinline__ uint32_t stg_row(uint32_t y) { return STG + (((y & 3) << 6) | (y >> 2)) * STG_PITCH; }\n"
        "constexpr uint32_t SLOT = STG + 256 * STG_PITCH;")
s = rep(s, """        if (on) {  // one divergent branch for the 12 groups
#pragma unroll""", """        if (on) {  // one divergent branch for the 12 groups
          if (v < uint32_t(K)) {  // phase 5's copy of a received data row
#pragma unroll
            for (int j = 0; j < ROW_WORDS / 4; ++j)
              *reinterpret_cast<__attribute__((address_space(3))) v4u *>(uintptr_t(stg_row(v) + 16 * j)) =
                  v4u{w[4 * j], w[4 * j + 1], w[4 * j + 2], w[4 * j + 3]};
          }
#pragma unroll""")
a = s.index("    // phase 5's received rows y = 4 lane + q < 256 (8 B of the row: this")
b = s.index("    S16 s;\n    // ---- phase 2")
s = s[:a] + s[b:]
s = rep(s, """          oh[q] = vperm(rv[q].y, rv[q].x, 0x06040200u);
          ol[q] = vperm(rv[q].y, rv[q].x, 0x07050301u);""", """          const uint2 rv = lds_ld2(stg_row(4 * lane + uint32_t(q)) + 8 * wave_s);
          oh[q] = vperm(rv.y, rv.x, 0x06040200u);
          ol[q] = vperm(rv.y, rv.x, 0x07050301u);""")
open(sys.argv[1], "w").write(s)
