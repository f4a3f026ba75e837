"""Pin the CPU restatement (oracle/ec_oracle.c) to the reference's own golden data.

CPU only.  Mirrors test/erasure_coding/reconstruct.cpp (Cpp_Polyf2e16,
Cpp_AFFT_tables, Cpp_Encode, Cpp_Decode*, Reconstruct1_3*, Systematic*,
Cpp_RecoveryThreshold_*, Cpp_MathNext*Pow2, Cpp_EltBEEncode) and adds the
seeded sweep / BASELINE-config fixtures from tests/golden/make_golden.py.
"""
import hashlib
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
from make_golden import payload_from_spec, present_from_spec  # noqa: E402

import oracle as orc  # noqa: E402


def sha(b):
    return hashlib.sha256(b).hexdigest()



@pytest.fixture(scope="module")
def oracle(restatement):
    """This module pins the C restatement itself (not the Checker the GPU
    parity tests use): it must equal the reference's goldens on its own."""
    return restatement

def test_tables_match_reference_golden_header(oracle, golden_tables):
    g = golden_tables
    assert sha(oracle.table("log").tobytes()) == g["header_LOG_TABLE_sha256"]
    assert sha(oracle.table("exp").tobytes()) == g["header_EXP_TABLE_sha256"]
    assert sha(oracle.table("log_walsh").tobytes()) == g["header_LOG_WALSH_sha256"]
    assert g["header_LOG_TABLE_sha256"] == g["runtime_log_sha256"]


def test_skews_match_reference(oracle, golden_tables):
    sk = oracle.table("skews")
    assert sha(sk.tobytes()) == golden_tables["skews_sha256"]
    for i, v in golden_tables["samples"]["skews"].items():
        assert sk[int(i)] == v
    # skews[2^m - 1] are the "skip multiply" markers (log of element 0)
    for m in range(16):
        assert sk[(1 << m) - 1] == 0xFFFF


def test_be_symbol():  # reconstruct.cpp:227-230
    assert int.from_bytes(bytes([0x11, 0x22]), "big") == 0x1122


@pytest.mark.parametrize("nv,thr", [(5, 2), (100, 34), (6, 2), (1024, 342), (4096, 1366),
                                    (65536, 21846)])
def test_recovery_threshold(oracle, nv, thr):  # reconstruct.cpp:282-325
    assert oracle.threshold(nv) == thr


@pytest.mark.parametrize("nv,err", [(0, "NotEnoughValidators"), (1, "NotEnoughValidators"),
                                    (65537, "TooManyValidators"), (90000, "TooManyValidators")])
def test_threshold_errors(oracle, nv, err):
    with pytest.raises(orc.CodecError) as e:
        oracle.threshold(nv)
    assert e.value.name == err


@pytest.mark.parametrize("nv,n,k", [(2, 2, 1), (3, 4, 1), (6, 8, 2), (8, 8, 2), (1000, 1024, 256),
                                    (1024, 1024, 256), (1025, 2048, 256), (4096, 4096, 1024),
                                    (65536, 65536, 16384)])
def test_params(oracle, nv, n, k):  # math.hpp:25-36 via reed-solomon.hpp:24-45
    assert oracle.params(nv) == (n, k)


def test_empty_payload(oracle):
    with pytest.raises(orc.CodecError) as e:
        oracle.encode(6, b"")
    assert e.value.name == "PayloadSizeIsZero"


def test_need_more_shards(oracle):  # reconstruct.cpp:403-437
    sh = oracle.encode(6, b"x" * 93)
    with pytest.raises(orc.CodecError) as e:
        oracle.reconstruct(6, [sh[0]] + [None] * 5)
    assert e.value.name == "NeedMoreShards"


def test_inconsistent_lengths(oracle):
    sh = oracle.encode(6, b"x" * 93)
    sh[3] = sh[3] + b"\0\0"
    with pytest.raises(orc.CodecError) as e:
        oracle.reconstruct(6, sh)
    assert e.value.name == "InconsistentShardLengths"


def test_wrong_index_garbage(oracle):  # reconstruct.cpp:484-504
    data = b"This is a test string. The purpose of it is not allow the evil forces to conquer the world!!"
    sh = oracle.encode(6, data)
    out = oracle.reconstruct(6, [None, None, None, sh[1], None, sh[5]])
    assert out[: len(data)] != data


def test_golden_vectors(oracle, golden_vectors):
    big = 0
    for c in golden_vectors:
        if c["payload_len"] > 2_000_000:
            big += 1
            continue  # covered by test_golden_large (slow)
        p = payload_from_spec(c["payload"])
        nv = c["nv"]
        shards = oracle.encode(nv, p)
        assert len(shards[0]) == c["shard_len"]
        assert sha(b"".join(shards)) == c["shards_sha256"], c
        present = set(present_from_spec(nv, c["k"], c["threshold"], c["present"]))
        rec = oracle.reconstruct(nv, [shards[i] if i in present else None for i in range(nv)])
        assert sha(rec) == c["reconstructed_sha256"], c
        if "systematic_sha256" in c:
            assert sha(oracle.reconstruct_from_systematic(nv, shards[: c["k"]])) == c["systematic_sha256"]
    assert big >= 1


def test_golden_large(oracle, golden_vectors):
    for c in golden_vectors:
        if c["payload_len"] <= 2_000_000:
            continue
        p = payload_from_spec(c["payload"])
        shards = oracle.encode(c["nv"], p)
        assert sha(b"".join(shards)) == c["shards_sha256"]


@pytest.mark.parametrize("n", [2, 8, 64, 1024, 4096])
def test_error_poly_folded_equals_direct(oracle, n):
    rng = np.random.default_rng(n)
    for frac in (0.0, 0.3, 0.7):
        e = (rng.random(n) < frac).astype(np.uint8)
        d = oracle.error_poly(e, n)[:n].astype(np.int64) % 65535
        f = oracle.error_poly(e, n, folded=True).astype(np.int64) % 65535
        assert (d == f).all()


@pytest.mark.parametrize("n", [2, 8, 256, 1024])
def test_formal_derivative_closed_form(oracle, n):
    """c'[j] = c[j] ^ XOR_{b: bit b of j is 0} c[j | 2^b]  (used by the HIP decoder)."""
    rng = np.random.default_rng(n)
    c = rng.integers(0, 65536, n, dtype=np.uint16)
    ref = oracle.formal_derivative(c)
    out = c.copy()
    for j in range(n):
        b = 1
        while b < n:
            if not j & b:
                out[j] ^= c[j | b]
            b <<= 1
    assert (out == ref).all()


@pytest.mark.parametrize("size,index", [(2, 0), (8, 8), (256, 0), (256, 768), (1024, 0)])
def test_afft_roundtrip(oracle, size, index):
    rng = np.random.default_rng(size + index)
    x = rng.integers(0, 65536, size, dtype=np.uint16)
    assert (oracle.inverse_afft(oracle.afft(x, index), index) == x).all()


@pytest.mark.parametrize("nv,cnt", [(1024, 342), (4096, 1366), (100, 34)])
def test_bench_gf_mul_counts(oracle, nv, cnt):
    """bench.py's secondary-ceiling multiply counts equal the
    butterflies with a non-0xFFFF skew that the reference's transforms run
    (additive_fft.hpp:99-141), counted here from the oracle's skew table."""
    import bench
    sk = oracle.table("skews")
    n, k = 1 << (nv - 1).bit_length(), None
    thr = (nv - 1) // 3 + 1
    k = 1 << (thr.bit_length() - 1)

    def muls(size, index):
        c, d = 0, 1
        while d < size:
            c += sum(1 for j in range(0, size, 2 * d) if sk[j + d - 1 + index] != 65535) * d
            d *= 2
        return c

    enc = muls(k, 0) + sum(muls(k, s) for s in range(k, n, k))
    rec_fft = muls(n, 0)
    e, r = bench.gf_mul_counts(nv, n, k, cnt)
    assert e == enc
    assert r == pytest.approx(cnt + 2 * rec_fft + k * (1 - cnt / nv))


def test_checker_uses_reference_for_bytes(restatement):
    """the parity tests' byte outputs are checked against
    the reference ec-cpp itself whenever its build (oracle/_ref) exists; the
    restatement serves the internals the reference does not export."""
    chk = orc.Checker.default()
    if not orc.RefEC.available():
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    assert chk.kind == "reference" and chk.encode.__self__ is chk.ref
    assert chk.error_poly.__self__ is chk.restatement
    p = bytes(range(256)) * 5 + b"\x07"
    assert chk.encode(100, p) == restatement.encode(100, p)
    keep = [s if i % 3 == 0 else None for i, s in enumerate(chk.encode(100, p))]
    assert chk.reconstruct(100, keep)[:len(p)] == p
