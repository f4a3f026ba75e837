#!/usr/bin/env python3
"""Bank-conflict check / search for the compact element-indexed multiply-table
image of the n = 1024 encode: entry x (element 2x) at
((x >> 4) << 8) | (sw(x) << 4) per 16-B plane, and the subfield tables' fifth
dword at 4 * sw1(x).  Every table read of the kernel must be conflict free:
ds_read_b128 in its four 16-lane groups, ds_read_b32 in its two 32-lane groups
(MI355X_MICROARCH.md, LDS).  Lane q (0..31) of either instance reads
x = 4q | c, 2q | c or q | c (layout A, stages 0 / 1 / 2) or a function of q >> 3
(layout B), c wave-uniform (sw linear: c does not change distinctness)."""
import itertools

B128 = [[0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27],
        [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31]]
PATTERNS = {"A0": lambda q: 4 * q, "A1": lambda q: 2 * q, "A2": lambda q: q,
            "B3": lambda q: 4 * (q >> 3), "B4": lambda q: 2 * (q >> 3), "B5": lambda q: q >> 3}


def lin(rows):  # rows[i] = mask of x bits feeding output bit i
    return lambda x: sum(((bin(x & r).count("1") & 1) << i) for i, r in enumerate(rows))


def ok128(sw):
    for f in PATTERNS.values():
        for g in B128:
            xs = {f(q) for q in g}
            if len({((x >> 4), sw(x)) for x in xs}) != len(xs):
                return False  # (x >> 4 distinct blocks differ in address bits >= 8: never the same bank quad? no:)
    return True


def banks128(sw):
    """max over patterns / groups of the conflict degree (16-B bank quads)"""
    worst = 1
    for f in PATTERNS.values():
        for g in B128:
            xs = {f(q) for q in g}
            slots = [sw(x) for x in xs]
            worst = max(worst, max(slots.count(s) for s in set(slots)))
    return worst


def banks32(sw1):
    worst = 1
    for f in PATTERNS.values():
        xs = {f(q) for q in range(32)}
        b = [sw1(x) % 32 for x in xs]
        worst = max(worst, max(b.count(s) for s in set(b)))
    return worst


if __name__ == "__main__":
    # 16-B slot swizzle: sw(x) = (x & 15) ^ G(x >> 4), G linear 5 -> 4 bits
    best = None
    for cols in itertools.product(range(16), repeat=5):
        rows = [(1 << i) | sum(((cols[j] >> i) & 1) << (4 + j) for j in range(5)) for i in range(4)]
        d = banks128(lin(rows))
        if d == 1:
            best = rows
            break
    print("sw rows", [bin(r) for r in best] if best else None)
    # dword swizzle for the subfield tables' fifth word: sw1(x) = x ^ H(x >> 5) on 7 bits
    best1 = None
    for cols in itertools.product(range(32), repeat=2):
        rows = [(1 << i) | sum(((cols[j] >> i) & 1) << (5 + j) for j in range(2)) for i in range(5)] + [1 << 5, 1 << 6]
        if banks32(lin(rows)) == 1:
            best1 = rows
            break
    print("sw1 rows", [bin(r) for r in best1] if best1 else None)
    cur = lambda x: (x ^ (x >> 4) ^ (x >> 8)) & 15  # noqa: E731  (the current image's f)
    print("current f on x: worst", banks128(cur))
