"""The reference's own C-ABI caller, /root/reference/benchmark/benchmark.cpp,
compiled UNCHANGED (oracle/Makefile: `_ref/benchmark`, built where the source
lies, with this repo's include/erasure_coding/erasure_coding.h) and linked
against this repo's liberasure_coding_crust.so — the drop-in claim of
INTEGRATION.md.  The binary is built in the container that has the reference
and travels to the GPU box with the tree (oracle/_ref is git-ignored, not
gpurun-ignored).  CPU: it links and every ECCR_ symbol it needs is ours.
GPU: it runs to completion (benchmark.cpp:36-113: 100 cycles of
ECCR_Test_MeasurePerformance per README size, next to ec-cpp)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "oracle", "_ref", "benchmark")
LIB = os.path.join(ROOT, "erasure-coding-crust_amd", "lib", "liberasure_coding_crust.so")

needs_bin = pytest.mark.skipif(not os.path.exists(BIN),
                               reason="oracle/_ref/benchmark not built (no /root/reference here)")


@needs_bin
def test_reference_benchmark_links_against_this_library():
    ldd = subprocess.run(["ldd", BIN], capture_output=True, text=True, check=True).stdout
    line = next(l for l in ldd.splitlines() if "liberasure_coding_crust.so" in l)
    assert "not found" not in line
    assert os.path.realpath(line.split("=>")[1].split("(")[0].strip()) == os.path.realpath(LIB)
    undef = subprocess.run(["nm", "-D", "--undefined-only", BIN], capture_output=True, text=True,
                           check=True).stdout
    need = set(re.findall(r"\b(ECCR_\w+)", undef))
    assert need == {"ECCR_Test_MeasurePerformance"}
    exported = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True,
                              check=True).stdout
    assert need <= set(re.findall(r"\bT (ECCR_\w+)", exported))


@needs_bin
@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_reference_benchmark_runs_on_gpu():
    r = subprocess.run(["timeout", "-k", "10", "540", BIN], capture_output=True, text=True)
    out_dir = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out_dir, exist_ok=True)
    with open(os.path.join(out_dir, "reference_benchmark.txt"), "w") as f:
        f.write(r.stdout + r.stderr)
    assert r.returncode == 0, r.stderr[-2000:]
    cases = [int(x) for x in re.findall(r"Benchmark case: (\d+) bytes", r.stdout)]
    assert cases == [15, 300, 5000, 100000, 1000000, 10000000]
    assert len(re.findall(r"Encode RUST", r.stdout)) == 6
    assert len(re.findall(r"Decode RUST", r.stdout)) == 6
    assert "erasure_coding_crust(amd)" not in r.stderr  # no library error was reported
