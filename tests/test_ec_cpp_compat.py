"""The ec-cpp source-compatible header (include/ec_cpp_compat/ec-cpp/ec-cpp.hpp,
SURVEY.md §8f row 4): a C++ program written against the ec-cpp API compiles
with g++ -std=c++20 (CPU test) and, on the GPU, produces the oracle's shards
and reconstructions and ec-cpp's error values."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "ec_cpp_compat_test.cpp")
INC = [os.path.join(ROOT, "include", "ec_cpp_compat"), os.path.join(ROOT, "include")]
LIBDIR = os.path.join(ROOT, "erasure-coding-crust_amd", "lib")


def _cxx(args):
    return subprocess.run(["g++", "-std=c++20", "-O1", *[f"-I{i}" for i in INC], *args],
                          capture_output=True, text=True)


def test_header_compiles():
    r = _cxx(["-fsyntax-only", "-Wall", "-Wextra", SRC])
    assert r.returncode == 0, r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("nv,plen", [(6, 1000), (1024, 100_001), (100, 7)])
def test_compat_program_matches_oracle(tmp_path, oracle, nv, plen):
    import ecc_amd as E
    import synth
    E.build()
    exe = tmp_path / "compat"
    r = _cxx([SRC, "-o", str(exe), f"-L{LIBDIR}", "-lerasure_coding_crust", f"-Wl,-rpath,{LIBDIR}"])
    assert r.returncode == 0, r.stderr
    payload = synth.payload(31 + nv, plen).tobytes()
    n, k, thr = E.code_params(nv)
    keep = sorted(int(x) for x in synth.present_set(77 + nv, nv, thr))
    (tmp_path / "p.bin").write_bytes(payload)
    (tmp_path / "keep.txt").write_text("\n".join(map(str, keep)))
    run = subprocess.run([str(exe), str(tmp_path / "p.bin"), str(nv), str(tmp_path / "keep.txt"),
                          str(tmp_path)], capture_output=True, text=True, timeout=300)
    assert run.returncode == 0, run.stdout + run.stderr
    assert "FAILED" not in run.stdout and "DONE" in run.stdout
    ref = oracle.encode(nv, payload)
    assert (tmp_path / "shards.bin").read_bytes() == b"".join(ref)
    rec = oracle.reconstruct(nv, [ref[i] if i in set(keep) else None for i in range(nv)])
    assert (tmp_path / "rec.bin").read_bytes() == rec
    assert (tmp_path / "sys.bin").read_bytes() == oracle.reconstruct_from_systematic(nv, ref[:k])
