#!/usr/bin/env python3
"""Diagnostic (wrong-result) variants of encode_k256w for the time account of
the headline encode.  Each removes one kind of work and
keeps every instruction of the rest, so the kernel-time difference is what
that work costs in the real interleaving:

  enc_diag.py KIND OUTDIR   writes OUTDIR/enc_k256w.hip and OUTDIR/cimg.hpp
    nobar   the per-tile workgroup barriers dropped (LDS races: garbage rows)
    static  tiles by a static grid stride instead of the ticket counter: with
            barriers dropped the tickets are read unsynchronised (lagging
            waves skip or repeat tiles), so combine nobar / cmp with static
            for a time account (nobar+static, cmp+static)
    wdyn    every wave takes its own tiles (its 8-piece group of the tile) from a
            counter of its own: no cross-wave tile hand-off, so nobar / cmp
            stay balanced and valid for timing (nobar+wdyn, cmp+wdyn)
    nbread  only the "regions read out" barriers dropped (tile start, after
            IFFT pass A, before each coset's first exchange)
    nbstg   only the "rows staged" barriers dropped (before each store phase)
    nost    the row stores dropped (LDS reads kept; nothing written)
    nold    payload loads replaced by lane-derived words
    nostg   row stores dropped, their LDS reads and addresses kept (asm-consumed)
    stplain row stores without the nontemporal hint
    noprio  no s_setprio around the store phases
    notab   multiply tables from VALU-derived words instead of LDS reads
    cmp     nobar + nost + nold: the transforms alone
    cmpt    cmp + notab: the register-only instruction stream
    dnobar  reconstruct_n1024: the two per-tile workgroup barriers dropped
    dnogat  reconstruct_n1024: the gather's row loads and E[v] multiplies dropped
    dnoout  reconstruct_n1024: the output stores dropped (values asm-consumed)
    xnobar, xnogat, xnoout  the same three for reconstruct_n1024x (writes
            OUTDIR/dec_n1024x.hip)
    xnorv   reconstruct_n1024x: phase 5's read of the staged present rows dropped
    xwdyn   reconstruct_n1024x: every wave takes its own tiles (its 4-column
            group) from a counter of its own (one 128-B line each): with
            xnobar / xnogat the waves stay balanced and the timing valid
    kclk:F  the clk probe in the kernel of csrc file F (its first kernel with
            dynamic LDS), e.g. kclk:enc_k1024.hip (writes OUTDIR/F)
    dclk    the clk probe in reconstruct_n1024 instead (writes OUTDIR/dec_n1024.hip;
            clk_run.py dec)
    clk     wave 0 of every workgroup sums s_memtime (shader clock) and
            s_memrealtime (100 MHz) over its lifetime: the clock under load
            (scripts/variants/clk_run.py); combine as e.g. clk+nostg

Build: scripts/build_var.sh diag_KIND "" enc_k256w.hip=OUT/enc_k256w.hip cimg.hpp=OUT/cimg.hpp"""
import os
import sys

ROOT = __file__.rsplit("/scripts/", 1)[0]
CS = f"{ROOT}/erasure-coding-crust_amd/csrc"
kind, out = sys.argv[1], sys.argv[2]
os.makedirs(out, exist_ok=True)
enc = open(f"{CS}/enc_k256w.hip").read()
cim = open(f"{CS}/cimg.hpp").read()
dec = open(f"{CS}/dec_n1024.hip").read()
decx = open(f"{CS}/dec_n1024x.hip").read()


READER = '''
extern "C" int ECCR_DIAG_stamps(unsigned long long *out, int n, int reset) {
  if (n > 16) n = 16;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(ecamd::g_stamp), n * sizeof(unsigned long long)) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[16] = {};
    z[2] = z[4] = ~0ull;  // atomicMin slots
    (void)hipMemcpyToSymbol(HIP_SYMBOL(ecamd::g_stamp), z, sizeof(z));
  }
  return n;
}
'''


CLK_END = ("  if (threadIdx.x == 0) {\n"
           "    atomicAdd(&g_stamp[0], (unsigned long long)(__builtin_amdgcn_s_memtime() - clk_t0));\n"
           "    atomicAdd(&g_stamp[1], (unsigned long long)(__builtin_amdgcn_s_memrealtime() - clk_r0));\n"
           "    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();\n"
           "    atomicMin(&g_stamp[2], (unsigned long long)clk_r0);\n"
           "    atomicMax(&g_stamp[3], (unsigned long long)clk_r0);\n"
           "    atomicMin(&g_stamp[4], r1);\n"
           "    atomicMax(&g_stamp[5], r1);\n"
           "    atomicAdd(&g_stamp[6], 1ull);\n  }\n")


def rep(s, old, new):
    assert s.count(old) == 1, old[:70]
    return s.replace(old, new)


ALIAS = {"cmp": ["nobar", "nost", "nold"], "cmpt": ["nobar", "nost", "nold", "notab"]}
extra = {}
kinds = [x for part in kind.split("+") for x in ALIAS.get(part, [part])]
for k in kinds:
    if k == "nobar":
        enc = rep(enc, "const auto rsync = [&]() __attribute__((always_inline)) { lds_barrier(); };",
                  "const auto rsync = [&]() __attribute__((always_inline)) { asm volatile(\"\" ::: \"memory\"); };")
    elif k == "static":
        enc = rep(enc, "  uint32_t cur = __builtin_amdgcn_readfirstlane(*slot);", "  uint32_t cur = blockIdx.x;")
        enc = rep(enc, "      next = __builtin_amdgcn_readfirstlane(*slot);", "      next = cur + gridDim.x;")
    elif k == "wdyn":
        take = ("[&]() { uint32_t v_ = 0; if ((tid0 & 63) == 0) v_ = atomicAdd(tick + 32 + 32 * (tid0 >> 6), 1u);"
                " return __builtin_amdgcn_readfirstlane(v_); }()")
        enc = rep(enc, "  uint32_t cur = __builtin_amdgcn_readfirstlane(*slot);", f"  uint32_t cur = {take};")
        # the next tile's ticket taken at the tile start (lane 0 of each wave),
        # read at its end: the atomic's latency hidden as in the product
        enc = rep(enc, "    if (tid0 == 0) taken = tick ? atomicAdd(tick, 1u) : cur + gridDim.x;",
                  "    if ((tid0 & 63) == 0) taken = atomicAdd(tick + 32 + 32 * (tid0 >> 6), 1u);")
        enc = rep(enc, "      next = __builtin_amdgcn_readfirstlane(*slot);", "      next = __builtin_amdgcn_readfirstlane(taken);")
        # one counter per wave index, each on its own 128-B line (8 on one
        # line serialise in L2: ~6 ns per atomic); 1152 B of scratch
        enc = rep(enc, "launch_zero_counters(tick, sizeof(uint32_t), s)", "launch_zero_counters(tick, 1152, s)")
        extra["enc_k256.hip"] = rep(open(f"{CS}/enc_k256.hip").read(),
                                    "size_t k256_scratch_bytes(const CodeParams &) { return 256; }",
                                    "size_t k256_scratch_bytes(const CodeParams &) { return 1152; }")
    elif k == "nbread":
        for old in ("    rsync();  // the other waves are done reading this region (last tile)\n",
                    "    rsync();  // systematic rows read out of the regions\n",
                    "      rsync();  // previous coset's rows read out\n",
                    "      rsync();  // tile start\n", "      rsync();  // after IFFT pass A\n",
                    "        rsync();  // after pass C\n"):
            enc = rep(enc, old, "")
    elif k == "nbstg":
        for old, new in (("    rsync();\n    store_sys();", "    store_sys();"),
                         ("      rsync();\n      if constexpr (decltype(last)::value)", "      if constexpr (decltype(last)::value)"),
                         ("      rsync();  // systematic rows staged\n", ""),
                         ("        rsync();  // rows staged\n", "")):
            enc = rep(enc, old, new)
    elif k == "nost":
        enc = rep(enc, "  asm volatile(\"\" : \"+v\"(lane));  // recomputed here, not kept live across the FFTs\n",
                  "  asm volatile(\"\" : \"+v\"(lane));\n  if (s0 != 0xFFFFFFFFu) {\n    then();\n    return;\n  }\n")
    elif k == "nostg":
        enc = rep(enc, "      __builtin_nontemporal_store(val, reinterpret_cast<v4u *>(dst + it * dstep));  // written once\n",
                  "      asm volatile(\"\" :: \"v\"(val), \"v\"(dst + it * dstep));\n")
    elif k == "stplain":
        enc = rep(enc, "      __builtin_nontemporal_store(val, reinterpret_cast<v4u *>(dst + it * dstep));  // written once\n",
                  "      *reinterpret_cast<v4u *>(dst + it * dstep) = val;\n")
    elif k == "noprio":
        enc = enc.replace("__builtin_amdgcn_s_setprio(1);", "").replace("__builtin_amdgcn_s_setprio(0);", "")
    elif k == "clk":
        enc = rep(enc, "namespace ecamd {\nnamespace {", "namespace ecamd {\n__device__ unsigned long long g_stamp[16];\nnamespace {")
        enc = rep(enc, "  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];\n",
                  "  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];\n"
                  "  const uint64_t clk_t0 = __builtin_amdgcn_s_memtime(), clk_r0 = __builtin_amdgcn_s_memrealtime();\n")
        enc = rep(enc, "  }\n}\n\nhipError_t launch_encode_k256w", "  }\n" + CLK_END + "}\n\nhipError_t launch_encode_k256w")
        enc += READER
    elif k == "dnobar":
        dec = rep(dec, "    lds_barrier();  // previous tile's readers of the regions are done (LDS only)\n", "")
        dec = rep(dec, "    if constexpr (!PACKED) __syncthreads();  // packed: the wave's own region and staging only\n", "")
    elif k == "dnogat":
        dec = rep(dec, "    if ((meta[0] & 0xffffu) != 0xffffu) load_row(0);\n    lds_barrier();",
                  "    lds_barrier();")
        dec = rep(dec, "      if ((meta[half] & 0xffffu) != 0xffffu) {\n", "      if (meta[half] == 0x12345678u) {\n")
    elif k == "dnoout":
        dec = rep(dec, "        *reinterpret_cast<uint2 *>(O + (col * K + 4 * lane) * 2) = make_uint2(w0, w1);\n",
                  "        asm volatile(\"\" :: \"v\"(w0), \"v\"(w1), \"v\"(O + (col * K + 4 * lane) * 2));\n")
    elif k == "xnobar":
        decx = rep(decx, "      lds_barrier();  // the previous tile's readers of the regions are done\n", "")
        decx = rep(decx, "    __syncthreads();  // (every wave has read SLOT)\n    const uint64_t cbase", "    const uint64_t cbase")
        extra["dec_n1024x.hip"] = decx
    elif k == "xnogat":
        decx = rep(decx, "      if ((meta[0] & 0xffffu) != 0xffffu) load_row(0);\n", "")
        decx = rep(decx, "        if (half == 1 && on) load_row(1);\n", "")
        decx = rep(decx, "        if (on) {  // one divergent branch", "        if (meta[half] == 0x12345678u) {  //")
        extra["dec_n1024x.hip"] = decx
    elif k == "xnorv":
        decx = rep(decx, "          const uint2 rv = lds_ld2(stg_row(4 * lane + uint32_t(q)) + 8 * wave_s);\n",
                   "          const uint2 rv = make_uint2(lane, uint32_t(q));\n")
        extra["dec_n1024x.hip"] = decx
    elif k == "xwdyn":
        W = "(tid0 & 63) == 0"
        decx = rep(decx, "  if (tid0 == 0) taken = gridDim.x + atomicAdd(tick, 1u);\n",
                   f"  if ({W}) taken = gridDim.x + atomicAdd(tick + 32 + 32 * (tid0 >> 6), 1u);\n")
        decx = rep(decx, "  if (tid0 == 0) *slot = taken;  // read after the first tile's region barrier\n", "")
        decx = rep(decx, "      nxt = __builtin_amdgcn_readfirstlane(*slot);\n"
                         "      if (tid0 == 0) taken = gridDim.x + atomicAdd(tick, 1u);  // the tile after nxt\n",
                   "      nxt = __builtin_amdgcn_readfirstlane(taken);\n"
                   f"      if ({W}) taken = gridDim.x + atomicAdd(tick + 32 + 32 * (tid0 >> 6), 1u);\n")
        decx = rep(decx, "    if (tid0 == 0) *slot = taken;\n", "")
        decx = rep(decx, "return n1024_tick_offset(p, batch) + 256; }", "return n1024_tick_offset(p, batch) + 2048; }")
        decx = rep(decx, "launch_zero_counters(tick, sizeof(uint32_t), s)", "launch_zero_counters(tick, 2048, s)")
        extra["dec_n1024x.hip"] = decx
    elif k == "xnoout":
        decx = rep(decx, "        *reinterpret_cast<uint2 *>(O + (col * K + 4 * lane) * 2) = make_uint2(w0, w1);\n",
                   "        asm volatile(\"\" :: \"v\"(w0), \"v\"(w1), \"v\"(O + (col * K + 4 * lane) * 2));\n")
        extra["dec_n1024x.hip"] = decx
    elif k.startswith("kclk:"):
        fname = k.split(":", 1)[1]
        src = open(f"{CS}/{fname}").read()
        src = rep(src, "namespace ecamd {\nnamespace {", "namespace ecamd {\n__device__ unsigned long long g_stamp[16];\nnamespace {")
        i = src.index("  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];\n")
        body = src.rindex("{\n", 0, i) + 2  # the kernel's opening brace
        j = i + len("  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];\n")
        depth, e = 1, body
        while depth:
            c = src[e]
            depth += (c == "{") - (c == "}")
            e += 1
        close = e - 1  # the kernel's closing brace
        src = (src[:j] + "  const uint64_t clk_t0 = __builtin_amdgcn_s_memtime(), clk_r0 = __builtin_amdgcn_s_memrealtime();\n"
               + src[j:close] + CLK_END + src[close:]) + READER
        extra[fname] = src
    elif k == "dclk":
        dec = rep(dec, "namespace ecamd {\nnamespace {", "namespace ecamd {\n__device__ unsigned long long g_stamp[16];\nnamespace {")
        dec = rep(dec, "  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];\n  uint8_t *tabs = lds;\n",
                  "  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];\n  uint8_t *tabs = lds;\n"
                  "  const uint64_t clk_t0 = __builtin_amdgcn_s_memtime(), clk_r0 = __builtin_amdgcn_s_memrealtime();\n")
        dec = rep(dec, "    __builtin_amdgcn_s_setprio(0);  // the next tile's gather: equal\n  }\n}\n",
                  "    __builtin_amdgcn_s_setprio(0);  // the next tile's gather: equal\n  }\n" + CLK_END + "}\n")
        dec += READER
    elif k == "nold":
        enc = rep(enc, "      for (int u = 0; u < 4; ++u) d[u] = *reinterpret_cast<const v4u *>(src + u * 2 * K);\n",
                  "      for (int u = 0; u < 4; ++u) d[u] = v4u{uint32_t(pw) * 0x9E3779B1u + u, uint32_t(fb) ^ 0x5bd1e995u, q * 77u, inst};\n")
    elif k == "notab":
        for typ, n in (("SubTab", 5), ("F9Tab", 16), ("Tab", 20)):
            start = cim.index(f"__device__ __forceinline__ void ctab(uint32_t lt, uint32_t u, {typ} &T) {{")
            end = cim.index("\n}\n", start) + 3
            body = (f"__device__ __forceinline__ void ctab(uint32_t lt, uint32_t u, {typ} &T) {{\n"
                    f"  const uint32_t a = lt ^ u;\n"
                    f"#pragma unroll\n  for (int i = 0; i < {n}; ++i) T.t[i] = (a + uint32_t(i) * 0x01010101u) & 0x3F3F3F3Fu;\n}}\n")
            cim = cim[:start] + body + cim[end:]
    else:
        raise SystemExit(f"unknown kind {k}")
open(f"{out}/enc_k256w.hip", "w").write(enc)
open(f"{out}/cimg.hpp", "w").write(cim)
open(f"{out}/dec_n1024.hip", "w").write(dec)
for fname, src in extra.items():
    open(f"{out}/{fname}", "w").write(src)
print("wrote", out, kinds)
