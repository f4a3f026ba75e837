#!/usr/bin/env python3
"""Dynamic instruction account of one kernel's hot path from a hipcc
-save-temps .s file: sums the opcode counts of the named basic blocks, each
weighted by how often it runs per tile (the caller knows the control flow:
read it off scripts/asm_blocks.py), and prints them per category.
  isa_account.py FILE.s KERNEL_PREFIX BLOCK:WEIGHT [BLOCK:WEIGHT ...]"""
import collections
import re
import sys

path, prefix = sys.argv[1], sys.argv[2]
weights = {b: float(w) for b, w in (x.rsplit(":", 1) for x in sys.argv[3:])}
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith(prefix) and ":" in l.split()[0])
end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
cur, ops = None, collections.Counter()
for l in lines[start:end + 1]:
    m = re.match(r"^(\.LBB\w+|_Z\w+):", l)
    if m:
        cur = m.group(1)
        continue
    m = re.match(r"\s+([a-z_0-9]+)\b", l)
    if m and cur in weights and m.group(1)[:2] in ("v_", "s_", "ds", "gl", "bu", "sc"):
        ops[m.group(1)] += weights[cur]
CATS = [
    ("v_perm", lambda o: o == "v_perm_b32"),
    ("v_and/or (selectors, masks)", lambda o: o.startswith(("v_and_b32", "v_or_b32", "v_and_or"))),
    ("v_lshrrev_b64 (selectors)", lambda o: o == "v_lshrrev_b64"),
    ("xor / bitop3 (accumulate, butterfly)", lambda o: o.startswith(("v_xor", "v_bitop3"))),
    ("32-bit shifts", lambda o: o.startswith(("v_lshrrev_b32", "v_lshlrev_b32"))),
    ("moves", lambda o: o.startswith(("v_mov", "v_cndmask", "v_readlane", "v_writelane", "v_readfirstlane"))),
    ("address / integer", lambda o: o.startswith(("v_add", "v_sub", "v_lshl_", "v_mad", "v_mul", "v_cmp", "v_bfe", "v_bcnt", "v_alignbyte"))),
    ("other VALU", lambda o: o.startswith("v_")),
    ("LDS", lambda o: o.startswith("ds_")),
    ("global / scratch", lambda o: o.startswith(("global_", "buffer_", "scratch_"))),
    ("s_waitcnt", lambda o: o == "s_waitcnt"),
    ("SALU / branch / other", lambda o: True),
]
done, tot = set(), sum(ops.values())
valu = sum(v for o, v in ops.items() if o.startswith("v_"))
print(f"total {tot:.0f} per tile, VALU {valu:.0f}")
for name, f in CATS:
    sel = {o: v for o, v in ops.items() if o not in done and f(o)}
    done |= set(sel)
    if sel:
        top = ", ".join(f"{o} {v:.0f}" for o, v in sorted(sel.items(), key=lambda x: -x[1])[:4])
        print(f"  {name:38s} {sum(sel.values()):7.0f}   ({top})")
