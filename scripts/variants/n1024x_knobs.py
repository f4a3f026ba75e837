#!/usr/bin/env python3
"""A/B variants of reconstruct_n1024x's tuning choices (moved out of the
product source; results in profiles/r05/NOTES.md):

  n1024x_knobs.py KNOB=VALUE[,KNOB=VALUE...] OUT.hip
    RB=N         table-ring depth of IFFT pass B' (product: 3; pass A' has no
                 ring since round 6's relayout)
    PRIO=1|2     issue priority by transform phase: 1 lets waves 8-11 lead
                 pass A, 4-7 pass B, 0-3 pass C and the FFT; 2 the reverse
                 (product: equal priority)

Build: scripts/build_var.sh NAME "" dec_n1024x.hip=OUT.hip"""
import sys

ROOT = __file__.rsplit("/scripts/", 1)[0]
knobs = dict(kv.split("=") for kv in sys.argv[1].split(",") if kv)
out = sys.argv[2]
s = open(f"{ROOT}/erasure-coding-crust_amd/csrc/dec_n1024x.hip").read()


def rep(s, old, new):
    assert old in s, old[:80]
    return s.replace(old, new, 1)


if "RB" in knobs:
    s = rep(s, "constexpr int RING_B = 3;", f"constexpr int RING_B = {knobs['RB']};")
if knobs.get("PRIO") in ("1", "2"):
    lead = "2u - uint32_t(phase)" if knobs["PRIO"] == "1" else "uint32_t(phase)"
    s = rep(s, "}  // namespace\n\n__global__",
            "__device__ __forceinline__ void prio3(uint32_t wave_s, int phase) {\n"
            f"  const uint32_t lead = {lead};\n"
            "  if (phase < 3 && (wave_s >> 2) == lead) __builtin_amdgcn_s_setprio(2);\n"
            "  else __builtin_amdgcn_s_setprio(0);\n}\n\n}  // namespace\n\n__global__")
    s = rep(s, "      ipassA2(s, lane);", "      prio3(wave_s, 0);\n      ipassA2(s, lane);")
    s = rep(s, "      ipassB2(s, lane);", "      prio3(wave_s, 1);\n      ipassB2(s, lane);")
    s = rep(s, "    // layout C: r bit0", "    prio3(wave_s, 2);\n    // layout C: r bit0")
    s = rep(s, "    // ---- phase 5: y = 4*lane", "    prio3(wave_s, 3);\n    // ---- phase 5: y = 4*lane")
open(out, "w").write(s)
