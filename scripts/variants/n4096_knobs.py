#!/usr/bin/env python3
"""A/B variants of reconstruct_n4096's schedule choices (round 6; results in
profiles/r06/NOTES.md):

  n4096_knobs.py KNOB=VALUE[,KNOB=VALUE...] OUT.hip
    PRIO4=1   at n = 4096 too, the two waves of a SIMD alternate the higher
              issue priority from quarter to quarter (product: only n = 2048)
    DYN2=1    dynamic tiles at n = 2048 too (product: only n = 4096)
    PRIO2=0   no alternation at n = 2048 either

Build: scripts/build_var.sh NAME "" dec_n4096.hip=OUT.hip"""
import sys

ROOT = __file__.rsplit("/scripts/", 1)[0]
knobs = dict(kv.split("=") for kv in sys.argv[1].split(",") if kv)
out = sys.argv[2]
s = open(f"{ROOT}/erasure-coding-crust_amd/csrc/dec_n4096.hip").read()


def rep(s, old, new):
    assert old in s, old[:80]
    return s.replace(old, new, 1)


if knobs.get("PRIO4") == "1":
    s = rep(s, "if (NQ == 2 && (((wave >> 2) ^ uint32_t(q)) & 1))", "if ((((wave >> 2) ^ uint32_t(q)) & 1))")
if knobs.get("PRIO2") == "0":
    s = rep(s, "if (NQ == 2 && (((wave >> 2) ^ uint32_t(q)) & 1))", "if (false && (((wave >> 2) ^ uint32_t(q)) & 1))")
if knobs.get("DYN2") == "1":
    s = rep(s, "constexpr bool DYN = NQ == 4;", "constexpr bool DYN = true;")
open(out, "w").write(s)
