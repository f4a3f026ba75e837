"""Static checks of the built kernel code that hand-written waits rely on
(ADVICE r04): the encode kernels wait for their table LDS-DMA / payload loads
with `s_waitcnt vmcnt(N)` counted past the row stores of the fast store path,
so each fast store phase must issue exactly N global stores per lane.  If a
toolchain change merged or split those stores, the wait would under-count and
the transform would read tables still in flight; this catches it.  CPU only:
compiles the device code to assembly (hipcc -S, gfx950, ~10 s per file)."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "erasure-coding-crust_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"


def _sched_flags(name):
    """The per-source scheduler flags of the library build (Makefile
    `SCHED_<source> ?= ...`), so the checked code is the shipped code."""
    mk = open(os.path.join(ROOT, "erasure-coding-crust_amd", "Makefile")).read()
    m = re.search(r"^SCHED_" + re.escape(name) + r"\s*\??=\s*(.*)$", mk, re.M)
    return m.group(1).split() if m else []


def _asm(name, tmp_path):
    if not os.path.exists(HIPCC):
        pytest.skip("no hipcc")
    out = tmp_path / (name + ".s")
    subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                    *_sched_flags(name), "-o", str(out), os.path.join(CSRC, name)], check=True,
                   capture_output=True)
    return out.read_text()


def _nt_store_blocks(text, kernel):
    """Streaming (nt) global stores per basic block of `kernel` (the fast store
    paths are the only nt stores)."""
    lines = text.split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and kernel in l.split(":")[0] and ":" in l)
    counts, cur = [], 0
    for l in lines[start + 1:]:
        if re.match(r"^(\.LBB\w+|_Z\w+):", l) or "s_endpgm" in l:
            if cur:
                counts.append(cur)
            cur = 0
            if "s_endpgm" in l:
                break
            continue
        if re.match(r"\s+global_store_dwordx4 .* nt\b", l):
            cur += 1
    return counts


def test_sched_flags_parsed():
    assert _sched_flags("enc_k256w.hip") == ["-mllvm", "-amdgpu-sched-strategy=max-memory-clause"]
    assert _sched_flags("dec_n1024x.hip") == []


def test_enc_k1024_fast_store_count(tmp_path):
    # enc_k1024.hip: kStoreIts = 8, the vmcnt(8) waits before the IFFT and cosets 2, 3
    src = open(os.path.join(CSRC, "enc_k1024.hip")).read()
    assert "kStoreIts == 8" in src and src.count("vmcnt(8)") >= 2
    blocks = _nt_store_blocks(_asm("enc_k1024.hip", tmp_path), "encode_k1024_fused")
    assert blocks and all(c == 8 for c in blocks), blocks
    assert sum(blocks) == 8 * 4, blocks  # systematic rows + 3 cosets


def test_enc_k256w_fast_store_count(tmp_path):
    # enc_k256w.hip: store_own8's fast path, 4 stores per lane; the compiler's
    # own vmcnt(4) before the next tile's transposes depends on it too
    blocks = _nt_store_blocks(_asm("enc_k256w.hip", tmp_path), "encode_k256w")
    assert blocks and all(c == 4 for c in blocks), blocks


def test_dec_n1024x_no_spills(tmp_path):
    # dec_n1024x.hip runs 3 waves per SIMD only at <= 168 VGPRs (launch bounds
    # 768); a loop-carried table or row array (a value read on a path that did
    # not write it) pushes it into scratch spills, ~25% slower (round 5)
    text = _asm("dec_n1024x.hip", tmp_path)
    body = text[text.index("reconstruct_n1024x"):]
    body = body[:body.index("s_endpgm")]
    assert "scratch_" not in body
    assert re.search(r"NumVgprs:\s+(\d+)", text), "resource summary missing"
    assert all(int(v) <= 168 for v in re.findall(r"NumVgprs:\s+(\d+)", text))


def test_enc_k512w_fast_store_count_no_spills(tmp_path):
    # enc_k512w.hip: store_own's fast path, 4 stores per lane (the vmcnt(4)
    # before cosets 2.. counts the previous coset's stores past the extension
    # image's LDS-DMA); the coset loop keeps the next tile's payload out of
    # the loop-carried state, so no scratch spills
    src = open(os.path.join(CSRC, "enc_k512w.hip")).read()
    assert src.count("vmcnt(4)") >= 1
    text = _asm("enc_k512w.hip", tmp_path)
    blocks = _nt_store_blocks(text, "encode_k512w")
    assert blocks and all(c == 4 for c in blocks), blocks
    body = text[text.index("encode_k512w"):]
    body = body[:body.index("s_endpgm")]
    assert "scratch_" not in body


def test_enc_kw_fast_store_count_no_spills(tmp_path):
    # enc_kw.hip (k = 16 .. 256): store_own's fast path, 4 stores per lane in
    # every instantiation (the compiler's own vmcnt(4) before the next tile's
    # transposes counts them, and at k = 256 the hand-written vmcnt(4) before
    # a coset's extension tables); no spills
    text = _asm("enc_kw.hip", tmp_path)
    for m in (4, 5, 6, 7, 8):
        name = "encode_kwILi%dE" % m
        blocks = _nt_store_blocks(text, name)
        assert blocks and all(c == 4 for c in blocks), (m, blocks)
        body = text[text.index(name + "EEvPKh"):]
        body = body[:body.index("s_endpgm")]
        assert "scratch_" not in body, m
