#!/usr/bin/env python3
"""Per-basic-block instruction counts of one kernel in a hipcc -save-temps .s
file:  asm_blocks.py FILE.s KERNEL_SYMBOL_PREFIX"""
import collections
import re
import sys

lines = open(sys.argv[1]).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith(sys.argv[2]) and ":" in l.split()[0])
end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
blocks, cur = [], None
for l in lines[start:end + 1]:
    m = re.match(r"^(\.LBB\w+|_Z\w+):", l)
    if m:
        cur = [m.group(1), collections.Counter(), []]
        blocks.append(cur)
        continue
    m = re.match(r"\s+([a-z_0-9]+)\b(.*)", l)
    if m and cur and m.group(1)[:2] in ("v_", "s_", "ds", "gl", "bu"):
        op = m.group(1)
        cur[1][op] += 1
        if op.startswith("s_cbranch") or op == "s_branch":
            cur[2].append(f"{op} {m.group(2).strip()}")
for name, c, br in blocks:
    tot = sum(c.values())
    valu = sum(v for k, v in c.items() if k.startswith("v_"))
    ds = sum(v for k, v in c.items() if k.startswith("ds_"))
    print(f"{name:28s} tot={tot:5d} valu={valu:5d} perm={c['v_perm_b32']:4d} ds={ds:4d} {' | '.join(br)}")
