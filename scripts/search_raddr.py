#!/usr/bin/env python3
"""Search a GF(2)-linear 8-B-cell swizzle of the 1024 positions of a wave's
LDS region (the two-workgroup reconstruct_n1024w of round 4, since removed:
profiles/r04/NOTES.md) under which every exchange
access is bank-conflict free (MI355X_MICROARCH.md, LDS): ds_read_b64 in two
32-lane groups (256 B: cell mod 32 distinct), ds_write_b64 in four 16-lane
groups (128 B: cell mod 16 distinct).  Layouts (lane bits -> position bits):
  A' lane = p2..p7                    (registers p0 p1 p8 p9)
  B' lane = p0 p1 p6 p7 p8 p9         (registers p2..p5)
  C  lane = p0..p5                    (registers p8 p9 p6 p7)"""
import random

LAYOUT_LANE_BITS = {"A'": [2, 3, 4, 5, 6, 7], "B'": [0, 1, 6, 7, 8, 9], "C": [0, 1, 2, 3, 4, 5]}


def apply(M, v):
    c = 0
    for i, row in enumerate(M):
        c |= (bin(row & v).count("1") & 1) << i
    return c


def rank(rows, n=10):
    rows = list(rows)
    r = 0
    for bit in range(n):
        piv = next((i for i in range(r, len(rows)) if (rows[i] >> bit) & 1), None)
        if piv is None:
            continue
        rows[r], rows[piv] = rows[piv], rows[r]
        for i in range(len(rows)):
            if i != r and (rows[i] >> bit) & 1:
                rows[i] ^= rows[r]
        r += 1
    return r


def ok(M):
    for bits in LAYOUT_LANE_BITS.values():
        for lo, width in ((0, 32), (32, 32)):  # reads
            cells = set()
            for l in range(lo, lo + width):
                v = sum(((l >> i) & 1) << b for i, b in enumerate(bits))
                cells.add(apply(M, v) % 32)
            if len(cells) != 32:
                return False
        for lo in range(0, 64, 16):  # writes
            cells = set()
            for l in range(lo, lo + 16):
                v = sum(((l >> i) & 1) << b for i, b in enumerate(bits))
                cells.add(apply(M, v) % 16)
            if len(cells) != 16:
                return False
    return True


if __name__ == "__main__":
    random.seed(1)
    for it in range(200000):
        # low 5 output bits random functions of all 10 bits; high 5 = p5..p9 (kept simple)
        M = [random.randrange(1, 1024) for _ in range(5)] + [1 << b for b in (5, 6, 7, 8, 9)]
        if rank(M) == 10 and ok(M):
            print("found after", it, [bin(r) for r in M])
            break
    else:
        print("none")
