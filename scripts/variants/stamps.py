#!/usr/bin/env python3
"""Diagnostic variants with per-phase s_memtime stamps (results unchanged; the
product sources carry no switches: this script writes patched copies).

  stamps.py enc OUT.hip   encode_k256: load / barrier wait / row stores / compute
  stamps.py dec OUT.hip   reconstruct_n1024: gather / barrier waits / IFFT /
                          derivative+FFT / output

Each variant sums the cycles of every wave into a __device__ array and exports
ECCR_DIAG_stamps(out, n, reset) (scripts/variants/stamp_run.py reads it).
Build with scripts/build_var.sh NAME "" enc_k256.hip=OUT.hip (or dec_n1024.hip)."""
import sys

ROOT = __file__.rsplit("/scripts/", 1)[0]
kind, out = sys.argv[1], sys.argv[2]
READER = '''
namespace ecamd {
__device__ unsigned long long g_stamp[16];
}
extern "C" int ECCR_DIAG_stamps(unsigned long long *out, int n, int reset) {
  if (n > 16) n = 16;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(ecamd::g_stamp), n * sizeof(unsigned long long)) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[16] = {};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(ecamd::g_stamp), z, sizeof(z));
  }
  return n;
}
'''
DECL = ('namespace ecamd {\n__device__ unsigned long long g_stamp[16];\n}\n')
STAMP = ('  uint64_t st_last_ = __builtin_amdgcn_s_memtime(), acc_[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};\n'
         '  const auto STAMP = [&](int i) __attribute__((always_inline)) {\n'
         '    const uint64_t now_ = __builtin_amdgcn_s_memtime();\n'
         '    acc_[i] += now_ - st_last_;\n'
         '    st_last_ = now_;\n'
         '  };\n')
FLUSH = ('  if ((threadIdx.x & 63) == 0)\n'
         '    for (int i = 0; i < 12; ++i) atomicAdd(&g_stamp[i], (unsigned long long)acc_[i]);\n')


def rep(s, old, new, count=1):
    assert s.count(old) >= count, old[:80]
    return s.replace(old, new, count)


if kind == "enc":
    s = open(f"{ROOT}/erasure-coding-crust_amd/csrc/enc_k256.hip").read()
    s = rep(s, "namespace ecamd {\nnamespace {", "namespace ecamd {\n__device__ unsigned long long g_stamp[16];\nnamespace {")
    s = rep(s, "  Tabs::copy_image<THREADS>(tabs, img0, tid0);\n  __syncthreads();\n",
            "  Tabs::copy_image<THREADS>(tabs, img0, tid0);\n  __syncthreads();\n" + STAMP)
    s = rep(s, "    } else {\n      lds_barrier();\n    }\n  };",
            "    } else {\n      STAMP(3);\n      lds_barrier();\n      STAMP(1);\n    }\n  };")
    s = rep(s, "      __builtin_amdgcn_s_setprio(1);\n",
            "      STAMP(3);\n      __builtin_amdgcn_s_setprio(1);\n")
    s = rep(s, "      __builtin_amdgcn_s_setprio(0);\n    };",
            "      __builtin_amdgcn_s_setprio(0);\n      STAMP(2);\n    };")
    s = rep(s, "    // ---- systematic shards 0..255 = the data symbols (poly_encoder.hpp:239)\n",
            "    STAMP(0);\n    // ---- systematic shards 0..255 = the data symbols (poly_encoder.hpp:239)\n")
    # end of the tile loop body of the kernel: the two closing braces before k256_applicable
    s = rep(s, "  }\n}\n\nbool k256_applicable", "  }\n" + FLUSH + "}\n\nbool k256_applicable")
    names = ["load", "barrier", "stores", "compute"]
elif kind == "dec":
    s = open(f"{ROOT}/erasure-coding-crust_amd/csrc/dec_n1024.hip").read()
    s = rep(s, "namespace ecamd {\nnamespace {", "namespace ecamd {\n__device__ unsigned long long g_stamp[16];\nnamespace {")
    s = rep(s, "  Tabs::copy_image<THREADS>(tabs, kF9 ? t.timg_f9 : t.timg_t, tid0);  // F9 kind 0\n  __syncthreads();\n",
            "  Tabs::copy_image<THREADS>(tabs, kF9 ? t.timg_f9 : t.timg_t, tid0);  // F9 kind 0\n  __syncthreads();\n" + STAMP)
    s = rep(s, "    if ((meta[0] & 0xffffu) != 0xffffu) load_row(0);\n    lds_barrier();",
            "    if ((meta[0] & 0xffffu) != 0xffffu) load_row(0);\n    STAMP(0);\n    lds_barrier();\n    STAMP(1);")
    s = rep(s, "    if constexpr (!PACKED) __syncthreads();  // packed",
            "    STAMP(0);\n    if constexpr (!PACKED) __syncthreads();\n    STAMP(1);  // packed")
    s = rep(s, "    prio_lead(wave_s & 4);\n    // ---- phases 3 + 4a", "    prio_lead(wave_s & 4);\n    STAMP(2);\n    // ---- phases 3 + 4a")
    s = rep(s, "    // the output at equal priority", "    STAMP(3);\n    // the output at equal priority")
    s = rep(s, "    __builtin_amdgcn_s_setprio(0);  // the next tile's gather: equal\n  }\n",
            "    __builtin_amdgcn_s_setprio(0);  // the next tile's gather: equal\n    STAMP(4);\n  }\n" + FLUSH)
    names = ["gather", "barriers", "ifft", "deriv+fft", "output"]
elif kind == "encw":
    s = open(f"{ROOT}/erasure-coding-crust_amd/csrc/enc_k256w.hip").read()
    s = rep(s, "namespace ecamd {\nnamespace {", "namespace ecamd {\n__device__ unsigned long long g_stamp[16];\nnamespace {")
    s = rep(s, "  __syncthreads();\n\n  const uint64_t npieces", "  __syncthreads();\n" + STAMP + "\n  const uint64_t npieces")
    s = rep(s, "    const auto rsync = [&]() __attribute__((always_inline)) { lds_barrier(); };",
            "    const auto rsync = [&]() __attribute__((always_inline)) { STAMP(3); lds_barrier(); STAMP(1); };")
    # both store lambdas (store, store_last)
    s = rep(s, "      __builtin_amdgcn_s_setprio(1);\n", "      STAMP(3);\n      __builtin_amdgcn_s_setprio(1);\n", 3)
    s = rep(s, "      __builtin_amdgcn_s_setprio(0);\n    };", "      __builtin_amdgcn_s_setprio(0);\n      STAMP(2);\n    };", 3)
    s = rep(s, "    // ---- systematic shards 0..255 = the data symbols (poly_encoder.hpp:239)\n",
            "    STAMP(0);\n    // ---- systematic shards 0..255 = the data symbols (poly_encoder.hpp:239)\n")
    s = rep(s, "  }\n}\n\nhipError_t launch_encode_k256w", "  }\n" + FLUSH + "}\n\nhipError_t launch_encode_k256w")
    names = ["load", "barrier", "stores", "compute"]
elif kind == "decw":
    # the two-workgroup reconstruct_n1024w: in dec_n1024.hip as of commit
    # 0ececd2 only (removed in 9c0fece); check that version out to rerun it
    s = open(f"{ROOT}/erasure-coding-crust_amd/csrc/dec_n1024.hip").read()
    s = rep(s, "namespace ecamd {\nnamespace {", "namespace ecamd {\n__device__ unsigned long long g_stamp[16];\nnamespace {")
    i = s.index("reconstruct_n1024w(")
    head, tail = s[:i], s[i:]
    tail = rep(tail, "  __syncthreads();\n\n  const uint64_t ncols", "  __syncthreads();\n" + STAMP + "\n  const uint64_t ncols")
    tail = rep(tail, "    if ((meta[0] & 0xffffu) != 0xffffu) load_row(0, w0, RT0);\n    lds_barrier();",
               "    if ((meta[0] & 0xffffu) != 0xffffu) load_row(0, w0, RT0);\n    STAMP(0);\n    lds_barrier();\n    STAMP(1);")
    tail = rep(tail, "    __syncthreads();\n    const uint64_t cbase", "    STAMP(0);\n    __syncthreads();\n    STAMP(1);\n    const uint64_t cbase")
    tail = rep(tail, "    // ---- phases 3 + 4a", "    STAMP(2);\n    // ---- phases 3 + 4a")
    tail = rep(tail, "    // ---- phase 5: y = 4 lane + q", "    STAMP(3);\n    // ---- phase 5: y = 4 lane + q")
    tail = rep(tail, "    for (int i = 0; i < NM; ++i) meta[i] = meta_next[i];\n    __builtin_amdgcn_s_setprio(0);  // the next tile's gather: equal\n  }\n}",
               "    for (int i = 0; i < NM; ++i) meta[i] = meta_next[i];\n    __builtin_amdgcn_s_setprio(0);\n    STAMP(4);\n  }\n" + FLUSH + "}")
    s = head + tail
    names = ["gather", "barriers", "ifft", "deriv+fft", "output"]
elif kind == "enc4":
    s = open(f"{ROOT}/erasure-coding-crust_amd/csrc/enc_k1024.hip").read()
    s = rep(s, "namespace ecamd {\nnamespace {", "namespace ecamd {\n__device__ unsigned long long g_stamp[16];\nnamespace {")
    s = rep(s, "  Tabs::copy_image<THREADS>(tabs, t.timg_t, tid0);  // index 0 (the IFFT)\n  __syncthreads();\n",
            "  Tabs::copy_image<THREADS>(tabs, t.timg_t, tid0);  // index 0 (the IFFT)\n  __syncthreads();\n" + STAMP)
    s = rep(s, "    // systematic shards 0..1023 = the data symbols (poly_encoder.hpp:239)\n",
            "    STAMP(0);\n    // systematic shards 0..1023 = the data symbols (poly_encoder.hpp:239)\n")
    s = rep(s, "    // the index-0 tables (the last tile's DMA, issued before the systematic\n",
            "    STAMP(1);\n    // the index-0 tables (the last tile's DMA, issued before the systematic\n")
    s = rep(s, "    lds_barrier();\n    if (!idle) {\n      to_tower(g);",
            "    lds_barrier();\n    STAMP(2);\n    if (!idle) {\n      to_tower(g);")
    s = rep(s, "    if (tid0 == 0) *slot = taken;  // (issued at the tile start: long returned)\n",
            "    STAMP(3);\n    if (tid0 == 0) *slot = taken;  // (issued at the tile start: long returned)\n")
    s = rep(s, "      constexpr uint32_t s = decltype(cs)::value;\n",
            "      constexpr uint32_t s = decltype(cs)::value;\n      STAMP(4);\n")
    s = rep(s, "      lds_barrier();\n      if (!idle) {\n        if constexpr (s > 1) {",
            "      lds_barrier();\n      STAMP(2);\n      if (!idle) {\n        if constexpr (s > 1) {")
    s = rep(s, "        stage_rows(g, my, lane);\n      }\n      lds_barrier();",
            "        stage_rows(g, my, lane);\n      }\n      STAMP(5);\n      lds_barrier();")
    s = rep(s, "      store_rows(regions, SH, sstride, s * K, nv, piece0, npieces, wave, lane);\n    };",
            "      STAMP(6);\n      store_rows(regions, SH, sstride, s * K, nv, piece0, npieces, wave, lane);\n      STAMP(7);\n    };")
    s = rep(s, "    cur = next;\n  }\n  asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");  // no LDS-DMA outlives the workgroup\n",
            "    STAMP(1);\n    cur = next;\n  }\n" + FLUSH + "  asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");  // no LDS-DMA outlives the workgroup\n")
    names = ["load", "sys+stage+stores", "vmcnt+barrier", "ifft", "coset start", "fft+stage", "barrier+dma", "stores"]
elif kind == "dec4":
    s = open(f"{ROOT}/erasure-coding-crust_amd/csrc/dec_n4096.hip").read()
    s = rep(s, "namespace ecamd {\nnamespace {", "namespace ecamd {\n__device__ unsigned long long g_stamp[16];\nnamespace {")
    s = rep(s, "  const uint64_t ncols = slen / 2;\n  const uint32_t tiles_pp = uint32_t((ncols + COLS - 1) / COLS);\n",
            STAMP + "  const uint64_t ncols = slen / 2;\n  const uint32_t tiles_pp = uint32_t((ncols + COLS - 1) / COLS);\n")
    s = rep(s, "      if (qnext >= 0) load_meta(qnext, tq);\n      asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");  // table image landed\n      lds_barrier();\n",
            "      if (qnext >= 0) load_meta(qnext, tq);\n      STAMP(0);\n      asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");  // table image landed\n      lds_barrier();\n      STAMP(1);\n")
    s = rep(s, "        ifft1024<q == 0, tower_sub_min(q)>(Qq, tabs, my, lq);\n      }\n",
            "        ifft1024<q == 0, tower_sub_min(q)>(Qq, tabs, my, lq);\n      }\n      STAMP(2);\n")
    s = rep(s, "        Tabs::dma_image<THREADS>(tabs, t.timg_t + qnext * kTabImageBytes, tq);\n        __builtin_amdgcn_sched_barrier(0);\n      }\n",
            "        Tabs::dma_image<THREADS>(tabs, t.timg_t + qnext * kTabImageBytes, tq);\n        __builtin_amdgcn_sched_barrier(0);\n      }\n      STAMP(3);\n")
    s = rep(s, "        asm volatile(\"\" : \"+v\"(P.l[r]), \"+v\"(P.h[r]), \"+v\"(Qa.l[r]), \"+v\"(Qa.h[r]));\n      __builtin_amdgcn_sched_barrier(0);\n    };",
            "        asm volatile(\"\" : \"+v\"(P.l[r]), \"+v\"(P.h[r]), \"+v\"(Qa.l[r]), \"+v\"(Qa.h[r]));\n      __builtin_amdgcn_sched_barrier(0);\n      STAMP(4);\n    };")
    s = rep(s, "    lds_barrier();  // every wave is done with the FFT tables\n",
            "    STAMP(5);\n    lds_barrier();  // every wave is done with the FFT tables\n")
    s = rep(s, "    lds_barrier();\n    if (idle) {\n", "    lds_barrier();\n    STAMP(6);\n    if (idle) {\n")
    s = rep(s, "        reinterpret_cast<uint4 *>(dst)[1] = make_uint4(wd[4], wd[5], wd[6], wd[7]);\n      }\n    }\n    tile = nxt;\n  }\n}",
            "        reinterpret_cast<uint4 *>(dst)[1] = make_uint4(wd[4], wd[5], wd[6], wd[7]);\n      }\n    }\n    STAMP(7);\n    tile = nxt;\n  }\n" + FLUSH + "}")
    names = ["gather", "wait_tab+bar", "ifft", "bar+dma", "accum", "deriv+fft", "outtab", "output"]
else:
    sys.exit("kind: enc | dec | encw | decw | enc4 | dec4")
s += READER.replace('namespace ecamd {\n__device__ unsigned long long g_stamp[16];\n}\n', '')
open(out, "w").write(s)
print(",".join(names))
