#!/usr/bin/env python3
"""Instruction mix of one kernel in a hipcc -save-temps .s file:
   isa_mix.py FILE.s KERNEL_SYMBOL_PREFIX  -> total + per-opcode counts."""
import collections
import re
import sys

path, prefix = sys.argv[1], sys.argv[2]
ops, on = collections.Counter(), False
for line in open(path):
    if not on and line.startswith(prefix) and ":" in line.split()[0]:
        on = True
        continue
    if on:
        m = re.match(r"\s+([a-z_0-9]+)\b", line)
        if m and m.group(1)[:2] in ("v_", "s_", "ds", "gl", "bu", "sc"):
            ops[m.group(1)] += 1
        if "s_endpgm" in line:
            break
print("total", sum(ops.values()))
for k, v in ops.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 12):
    print(f"{v:6d} {k}")
