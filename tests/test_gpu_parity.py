"""GPU parity: the HIP path (through the C ABI) against the oracle and the
reference's golden fixtures.  Bit-exact for every byte.  Needs an MI355X.

Covers the reference's own cases (test/erasure_coding/reconstruct.cpp), the
seeded sweep of tests/golden/vectors.json, edge cases (1-byte and ragged
payloads, n_validators 2..65536, exactly-k shards, systematic fast path) and,
at BASELINE sizes, size-independent properties (encode -> erase -> decode
round trips, batch == single-call equality).
"""
import hashlib
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
from make_golden import LONG_DATA, TEST_DATA, payload_from_spec, present_from_spec  # noqa: E402

import ecc_amd as E  # noqa: E402  (imports torch first)
import synth  # noqa: E402

pytestmark = pytest.mark.gpu


def sha(b):
    return hashlib.sha256(b).hexdigest()


@pytest.fixture(scope="module", autouse=True)
def _device():
    assert E.device_count() > 0, "no HIP device: -m gpu tests need an MI355X"
    r = E.lib().ECCR_AMD_init_device()
    assert r.tag == 0, E.last_error()


def decode_subset(nv, shards, keep):
    keep = set(keep)
    return E.reconstruct(nv, [(i, shards[i]) for i in range(nv) if i in keep])


@pytest.mark.gpu
def test_checker_is_the_reference(oracle):
    """Which checker the byte comparisons of this run used:
    the reference ec-cpp build travels with the tree, so it must be it."""
    import oracle as orc
    assert oracle.kind == ("reference" if orc.RefEC.available() else "restatement")
    print("checker:", oracle.kind)


# ---------------------------------------------------------------- reference KATs
def test_kat_whole_data():  # ReconstructChunksFromWholeData
    sh = E.obtain_chunks(6, TEST_DATA.encode())
    assert len(sh) == 6
    out = E.reconstruct(6, list(enumerate(sh)))
    assert out[: len(TEST_DATA)] == TEST_DATA.encode()


@pytest.mark.parametrize("keep", [[0, 1], [1, 5], [2, 3, 4, 5], [2, 5], [0, 5]])
def test_kat_subsets(keep):  # Reconstruct1_3, Reconstruct1_3_last_one, Cpp_Reconstruct1_3(_Border)
    sh = E.obtain_chunks(6, TEST_DATA.encode())
    assert decode_subset(6, sh, keep)[: len(TEST_DATA)] == TEST_DATA.encode()


def test_kat_wrong_index():  # Reconstruct_WrongIndex
    sh = E.obtain_chunks(6, TEST_DATA.encode())
    out = E.reconstruct(6, [(3, sh[1]), (5, sh[5])])
    assert out[: len(TEST_DATA)] != TEST_DATA.encode()


@pytest.mark.parametrize("text", [TEST_DATA, LONG_DATA, "1"])
def test_kat_systematic(oracle, text):  # SystematicChuncksRust(ToCpp)
    sh = E.obtain_chunks(6, text.encode())
    assert sh == oracle.encode(6, text.encode())  # Cpp_Encode (Rust == C++)
    out = E.reconstruct_from_systematic(6, [(0, sh[0]), (1, sh[1])])
    assert out[: len(text)] == text.encode()
    assert out == oracle.reconstruct_from_systematic(6, sh[:2])


def test_kat_decode_big(oracle):  # Cpp_Decode_Big: 1 MiB of (i+1) % 255, n=6
    p = synth.pattern_mod255(1 << 20).tobytes()
    sh = E.obtain_chunks(6, p)
    assert sha(b"".join(sh)) == sha(b"".join(oracle.encode(6, p)))
    assert E.reconstruct(6, list(enumerate(sh))) == oracle.reconstruct(6, sh)


# ---------------------------------------------------------------- golden vectors
def test_golden_vectors(golden_vectors):
    for c in golden_vectors:
        nv = c["nv"]
        p = payload_from_spec(c["payload"])
        sh = E.obtain_chunks(nv, p)
        assert len(sh[0]) == c["shard_len"]
        assert sha(b"".join(sh)) == c["shards_sha256"], (c["tag"], nv, len(p))
        keep = present_from_spec(nv, c["k"], c["threshold"], c["present"])
        rec = decode_subset(nv, sh, keep)
        assert sha(rec) == c["reconstructed_sha256"], (c["tag"], nv, len(p), "reconstruct")
        if "systematic_sha256" in c:
            s = E.reconstruct_from_systematic(nv, list(enumerate(sh[: c["k"]])))
            assert sha(s) == c["systematic_sha256"]


# ---------------------------------------------------------------- random sweep vs oracle
@pytest.mark.parametrize("nv", [2, 3, 5, 6, 7, 9, 16, 33, 46, 64, 65, 100, 128, 129, 200, 255, 256,
                                257, 300, 384, 512, 600, 700, 765, 1000, 1024, 1025, 1366, 1367,
                                2048, 2049, 3000, 3069, 3070, 3500, 4096])
def test_random_vs_oracle(oracle, nv):
    rng = np.random.default_rng(nv)
    n, k, thr = E.code_params(nv)
    for plen in (1, 2, 2 * k - 1, 2 * k, 2 * k + 1, int(rng.integers(1, 20000))):
        p = rng.integers(0, 256, plen, dtype=np.uint8).tobytes()
        sh = E.obtain_chunks(nv, p)
        ref = oracle.encode(nv, p)
        assert sh == ref, (nv, plen)
        for cnt in (k, thr, nv):
            keep = rng.permutation(nv)[:cnt]
            kk = set(int(x) for x in keep)
            out = decode_subset(nv, sh, kk)
            assert out == oracle.reconstruct(nv, [sh[i] if i in kk else None for i in range(nv)])
            assert out[:plen] == p


def test_tiny_encode_vs_oracle(oracle):
    """enc_tiny.hip (per-call encode, n <= 16, payload <= 2048 B in the kernel
    arguments): every n_validators it takes, payload lengths around its piece
    and size boundaries, and the first lengths past it (the staged path)."""
    rng = np.random.default_rng(32)
    for nv in range(2, 34):
        for plen in (1, 2, 3, 4, 5, 15, 16, 17, 300, 1000, 2047, 2048, 2049):
            p = rng.integers(0, 256, plen, dtype=np.uint8).tobytes()
            assert E.obtain_chunks(nv, p) == oracle.encode(nv, p), (nv, plen)


@pytest.mark.parametrize("nv", [16384, 65536])
def test_huge_n(oracle, nv):
    n, k, thr = E.code_params(nv)
    p = synth.payload(nv, 3 * k + 5).tobytes()
    sh = E.obtain_chunks(nv, p)
    assert sha(b"".join(sh)) == sha(b"".join(oracle.encode(nv, p)))
    keep = set(int(x) for x in synth.present_set(nv, nv, k))
    out = decode_subset(nv, sh, keep)
    assert out[: len(p)] == p


def test_measure_performance():
    e, d = E.measure_performance(6, b"x" * 5000)
    assert e >= 0 and d >= 0


# ---------------------------------------------------------------- device batch API
def _batch_case(nv, plen, batch, cnt_key="threshold", seed0=0, pad=0):
    """pad=0: tight rows (generic kernels); pad>0: shard rows aligned to `pad`
    bytes and payload rows to 64 (the fast kernels, ragged lengths included:
    with a payload pitch off 16 B every encode takes the generic kernel)."""
    import torch
    n, k, thr = E.code_params(nv)
    sl = E.shard_len(nv, plen)
    ss = (sl + pad - 1) // pad * pad if pad else sl
    ps = (plen + 63) // 64 * 64 if pad else plen
    pay = np.stack([synth.payload(seed0 + b, plen) for b in range(batch)])
    cnt = {"threshold": thr, "k": k}[cnt_key]
    pres = np.stack([synth.present_mask(10**6 + seed0 + b, nv, cnt, n) for b in range(batch)])
    d_pay = torch.zeros((batch, ps), dtype=torch.uint8, device="cuda")
    d_pay[:, :plen] = torch.from_numpy(pay).cuda()
    d_sh = torch.zeros((batch, nv, ss), dtype=torch.uint8, device="cuda")
    d_pr = torch.from_numpy(pres).cuda()
    d_el = torch.zeros((batch, n), dtype=torch.int16, device="cuda")
    d_out = torch.zeros((batch, sl * k), dtype=torch.uint8, device="cuda")
    E.encode_batch(nv, d_pay, plen, ps, batch, d_sh, ss)
    E.error_locator(nv, d_pr, batch, d_el)
    E.reconstruct_batch(nv, d_sh, sl, ss, d_pr, d_el, batch, d_out, sl * k)
    torch.cuda.synchronize()
    sh = d_sh.cpu().numpy()[:, :, :sl].copy()
    return pay, pres, sh, d_el.cpu().numpy().view(np.uint16), d_out.cpu().numpy()


@pytest.mark.parametrize("nv,plen,batch,pad", [
    (6, 300, 5, 0), (1024, 5000, 3, 0), (1024, 70000, 2, 0), (4096, 3001, 2, 0), (100, 1, 4, 0),
    (1024, 5000, 3, 64), (1024, 70000, 2, 16), (1024, 1, 3, 16), (1024, 511, 2, 8),
    (1024, 131073, 2, 64), (1000, 99999, 2, 64), (800, 12345, 3, 64), (4096, 3001, 2, 64),
    # k = 256 / n = 1024 encode: 9, 9 (last one partial), 8 and 7 groups of 8
    # pieces per payload (one full tile plus a partial one, one tile, a partial one)
    (1024, 36864, 4, 0), (900, 36000, 5, 16), (1024, 30000, 5, 64), (800, 28000, 3, 64),
    # k = 1024 / n = 4096 fast path (config 4): several 64-piece tiles, a partly
    # populated last coset (nv 3500), tight and 8/16/64-byte row pitches
    (4096, 300001, 2, 64), (3070, 300001, 2, 16), (3500, 131073, 2, 8), (4096, 131072, 1, 0),
    # k = 32 / 64 / 128, n <= 1024 encode (encode_kw): several tiles,
    # partly populated last cosets, 8/16/64-byte pitches
    (600, 300001, 2, 64), (700, 5000, 2, 64), (384, 131073, 2, 64), (300, 70001, 3, 16),
    (100, 12345, 3, 8), (200, 200001, 2, 64),
    # 64 <= n <= 1024, 16 <= k <= 512 register-blocked reconstruct (every n / k
    # shape): several tiles, partial last tile, 16/64-byte pitches
    (46, 70001, 2, 64), (65, 9999, 3, 16), (129, 33333, 2, 16), (257, 100001, 2, 64),
    (512, 200001, 2, 64), (765, 300001, 2, 64), (600, 1, 2, 16),
    # n = 2048 / 4096 with k = 256 / 512: encode with per-coset table images
    # (encode_k256<2048>, encode_k512w), reconstruct by halves / quarters
    # with k < 1024 outputs
    (1025, 5000, 3, 64), (1500, 200001, 2, 64), (2048, 100001, 2, 16), (2500, 300001, 2, 64),
    (3069, 4097, 2, 16)])
def test_batch_vs_oracle(oracle, nv, plen, batch, pad):
    pay, pres, sh, el, out = _batch_case(nv, plen, batch, pad=pad)
    n, k, _ = E.code_params(nv)
    for b in range(batch):
        ref = oracle.encode(nv, pay[b].tobytes())
        assert b"".join(ref) == sh[b].tobytes(), b
        erased = (pres[b][:n] == 0).astype(np.uint8)
        ep = oracle.error_poly(erased, n)[:n].astype(np.int64) % 65535
        assert ((el[b].astype(np.int64) % 65535) == ep).all()
        keep = [ref[i] if pres[b][i] else None for i in range(nv)]
        assert out[b].tobytes() == oracle.reconstruct(nv, keep)


@pytest.mark.parametrize("seed", range(12))
def test_batch_random_nv_aligned(oracle, seed):
    """n_validators drawn uniformly from 2..4096 and payload lengths
    log-uniformly from 1 B to 1.2 MB, with 64-B payload rows and 8/16/64-B
    shard pitches (so the fast encodes and reconstructs take whatever shape
    falls out, ragged tails included), encode + locator + reconstruct against
    the reference at the threshold count of random shards."""
    rng = np.random.default_rng(4321 + seed)
    for _ in range(8):
        nv = int(rng.integers(2, 4097))
        plen = int(np.exp(rng.uniform(0, np.log(1_200_000))))
        pad = int(rng.choice([8, 16, 64]))
        pay, pres, sh, el, out = _batch_case(nv, plen, 2, seed0=100 * seed + nv, pad=pad)
        n, k, _ = E.code_params(nv)
        for b in range(2):
            ref = oracle.encode(nv, pay[b].tobytes())
            assert b"".join(ref) == sh[b].tobytes(), (nv, plen, pad, b)
            keep = [ref[i] if pres[b][i] else None for i in range(nv)]
            assert out[b].tobytes() == oracle.reconstruct(nv, keep), (nv, plen, pad, b)


@pytest.mark.parametrize("nv,plen,batch,pad", [
    (1534, 70001, 3, 64), (1535, 1, 2, 16), (1536, 3 * 32768, 2, 16), (1800, 33793, 2, 8),
    (2048, 66559, 3, 64), (2049, 40001, 2, 16), (2560, 50001, 2, 64), (2561, 30001, 2, 8),
    (3000, 32769, 2, 64), (3069, 100001, 3, 16), (3069, 1024 * 31, 2, 64)])
def test_encode_k512w_vs_oracle(oracle, nv, plen, batch, pad):
    """enc_k512w.hip (k = 512, n = 2048 / 4096): the first and last
    n_validators of each coset count (J = 2..5 cosets, the last partly below
    n_validators), payloads of one piece, of whole and partial 32-piece tiles
    (waves with no pieces), 8 / 16 / 64-byte row pitches (the slow store path
    below 16), against the reference encoder."""
    import torch
    n, k, _ = E.code_params(nv)
    assert k == 512
    sl = E.shard_len(nv, plen)
    ss = (sl + pad - 1) // pad * pad
    pays = [synth.payload(nv * 3 + b, plen) for b in range(batch)]
    ps = (plen + 63) // 64 * 64  # 16-B aligned payload rows: the fast kernels take ragged lengths too
    d_pay = torch.zeros((batch, ps), dtype=torch.uint8, device="cuda")
    for b in range(batch):
        d_pay[b, :plen] = torch.from_numpy(pays[b])
    d_sh = torch.full((batch, nv, ss), 0x5C, dtype=torch.uint8, device="cuda")
    E.encode_batch(nv, d_pay, plen, ps, batch, d_sh, ss)
    torch.cuda.synchronize()
    got = d_sh.cpu().numpy()
    for b in range(batch):
        want = oracle.encode(nv, pays[b].tobytes())
        assert b"".join(want) == got[b, :, :sl].tobytes(), (nv, plen, b)
        assert (got[b, :, sl:] == 0x5C).all()  # nothing past the shard length


@pytest.mark.parametrize("nv,plen,batch,pad", [
    # k = 16 (n 64 / 128), 32 (128 / 256), 64 (256 / 512): first and last
    # n_validators of the k, the n boundary
    (46, 70001, 3, 64), (47, 1, 2, 16), (64, 32768, 2, 16), (65, 32769, 3, 8), (93, 100001, 2, 64),
    (94, 33, 3, 16), (128, 3 * 32768, 2, 64), (129, 40001, 2, 8), (189, 65, 2, 64),
    (190, 70001, 2, 16), (256, 129, 3, 64), (257, 32767, 2, 8), (300, 100001, 2, 64), (381, 32769, 2, 16),
    # k = 256 at n = 2048 (4 and 5 cosets, stage 0 of cosets 4.. from the
    # extension image)
    (1025, 70001, 3, 64), (1100, 1, 2, 16), (1280, 32768, 2, 16), (1281, 32769, 3, 8),
    (1400, 255, 2, 64), (1533, 100001, 3, 16), (1533, 1_000_000, 2, 64),
    # k = 128 (n 512 / 1024)
    (382, 70001, 3, 64), (383, 1, 2, 16), (384, 32768, 2, 16), (512, 32769, 3, 8),
    (513, 40001, 2, 64), (600, 255, 2, 16), (640, 3 * 32768, 2, 64), (641, 30001, 2, 8),
    (700, 257, 3, 64), (765, 100001, 3, 16), (765, 1_000_000, 2, 64)])
def test_encode_kw_vs_oracle(oracle, nv, plen, batch, pad):
    """enc_kw.hip (k = 16 .. 128, n <= 8 k; k = 256, n = 2048): the first and last n_validators
    of each coset count (J = 2..5 cosets, the last partly below n_validators),
    payloads of one piece, of whole and partial 32 KB tiles (waves with no
    pieces), 8 / 16 / 64-byte row pitches, against the reference encoder."""
    import torch
    n, k, _ = E.code_params(nv)
    assert 16 <= k <= 128 or (k, n) == (256, 2048)
    sl = E.shard_len(nv, plen)
    ss = (sl + pad - 1) // pad * pad
    pays = [synth.payload(nv * 5 + b, plen) for b in range(batch)]
    ps = (plen + 63) // 64 * 64  # 16-B aligned payload rows: the fast kernels take ragged lengths too
    d_pay = torch.zeros((batch, ps), dtype=torch.uint8, device="cuda")
    for b in range(batch):
        d_pay[b, :plen] = torch.from_numpy(pays[b])
    d_sh = torch.full((batch, nv, ss), 0x5C, dtype=torch.uint8, device="cuda")
    E.encode_batch(nv, d_pay, plen, ps, batch, d_sh, ss)
    torch.cuda.synchronize()
    got = d_sh.cpu().numpy()
    for b in range(batch):
        want = oracle.encode(nv, pays[b].tobytes())
        assert b"".join(want) == got[b, :, :sl].tobytes(), (nv, plen, b)
        assert (got[b, :, sl:] == 0x5C).all()


def test_batch_config2_roundtrip():
    """BASELINE config 2 shape (n_validators=1024, 1 MB payloads, 342 random shards):
    size-independent round trip + batch-vs-single equality on a batch of 8."""
    pay, pres, sh, el, out = _batch_case(1024, 1_000_000, 8, seed0=100, pad=64)
    for b in range(8):
        assert out[b][:1_000_000].tobytes() == pay[b].tobytes()
        assert not out[b][1_000_000:].any()  # zero padding, as the reference
    single = E.obtain_chunks(1024, pay[3].tobytes())
    assert b"".join(single) == sh[3].tobytes()


def test_batch_config3_k_golden(oracle, golden_vectors):
    """BASELINE config 3 read as 'reconstruct from k random shards' (10 MB,
    n_validators = 1024, c = k = 256) on the device batch path, B = 2: payload 0
    is the golden case generated by the reference ec-cpp (tests/golden, tag
    config, count k), payload 1 is checked against the oracle."""
    import torch
    case = next(c for c in golden_vectors if c["tag"] == "config" and c["nv"] == 1024
                and c["payload_len"] == 10_000_000 and c["present"]["count"] == "k")
    nv, plen, batch = 1024, 10_000_000, 2
    n, k, thr = E.code_params(nv)
    sl = E.shard_len(nv, plen)
    ss = (sl + 63) // 64 * 64
    pay = np.stack([np.frombuffer(payload_from_spec(case["payload"]), np.uint8),
                    synth.payload(4242, plen)])
    pres = np.zeros((batch, n), dtype=np.uint8)
    pres[0, present_from_spec(nv, k, thr, case["present"])] = 1
    pres[1, synth.present_set(4243, nv, k)] = 1
    assert (pres.sum(axis=1) == k).all()
    d_pay = torch.from_numpy(pay).cuda()
    d_sh = _prefilled((batch, nv, ss))
    d_pr = torch.from_numpy(pres).cuda()
    d_el = torch.zeros((batch, n), dtype=torch.int16, device="cuda")
    d_out = _prefilled((batch, sl * k))
    E.encode_batch(nv, d_pay, plen, plen, batch, d_sh, ss)
    torch.cuda.synchronize()
    for b in range(batch):  # absent rows: garbage that must never be read
        gone = np.where(pres[b][:nv] == 0)[0]
        d_sh[b, torch.from_numpy(gone).cuda()] = 0x5C
    E.error_locator(nv, d_pr, batch, d_el)
    E.reconstruct_batch(nv, d_sh, sl, ss, d_pr, d_el, batch, d_out, sl * k)
    torch.cuda.synchronize()
    sh = d_sh.cpu().numpy()
    out = d_out.cpu().numpy()
    assert sha(out[0].tobytes()) == case["reconstructed_sha256"]
    ref1 = oracle.encode(nv, pay[1].tobytes())
    keep = [ref1[i] if pres[1][i] else None for i in range(nv)]
    assert out[1].tobytes() == oracle.reconstruct(nv, keep)
    assert out[1][:plen].tobytes() == pay[1].tobytes()
    # the encode of payload 0 (present rows survive the 0x5C overwrite) vs golden
    E.encode_batch(nv, d_pay, plen, plen, batch, d_sh, ss)
    torch.cuda.synchronize()
    sh = d_sh.cpu().numpy()
    assert sha(np.ascontiguousarray(sh[0][:, :sl]).tobytes()) == case["shards_sha256"]
    assert [sh[1][v, :sl].tobytes() for v in range(nv)] == ref1


def test_batch_nv4096_1MB(oracle):
    """BASELINE config 4 shape at full payload size on the device batch path:
    n_validators = 4096 (n = 4096, k = 1024), 1 MB payloads, B = 4, so several
    k = 1024 encode tiles span payloads and the four encode_k1024 launches share
    one coefficient scratch; every shard and output byte vs the oracle."""
    nv, plen, batch = 4096, 1_000_000, 4
    pay, pres, sh, el, out = _batch_case(nv, plen, batch, seed0=40960, pad=64)
    n, k, _ = E.code_params(nv)
    for b in range(batch):
        ref = oracle.encode(nv, pay[b].tobytes())
        assert b"".join(ref) == sh[b].tobytes(), b
        keep = [ref[i] if pres[b][i] else None for i in range(nv)]
        assert out[b].tobytes() == oracle.reconstruct(nv, keep), b
        assert out[b][:plen].tobytes() == pay[b].tobytes(), b


def test_batch_systematic():
    import torch
    nv, plen, batch = 1024, 100_000, 3
    pay, pres, sh, el, out = _batch_case(nv, plen, batch, seed0=7)
    n, k, _ = E.code_params(nv)
    sl = E.shard_len(nv, plen)
    d_sh = torch.from_numpy(sh).cuda()
    d_out = torch.zeros((batch, sl * k), dtype=torch.uint8, device="cuda")
    E.systematic_batch(nv, d_sh, sl, sl, batch, d_out, sl * k)
    o = d_out.cpu().numpy()
    for b in range(batch):
        assert o[b][:plen].tobytes() == pay[b].tobytes()


# ---------------------------------------------------------------- host batches (row f2)
@pytest.mark.parametrize("nv,plen,batch,chunk", [(1024, 70001, 7, 2), (100, 5000, 5, 0),
                                                 (1024, 1_000_000, 4, 3),
                                                 # k = 1024: chunks on the 3 slot streams
                                                 # share the encode's coefficient scratch
                                                 (4096, 60001, 7, 1),
                                                 # the round-6 encodes (encode_kw<4>, <6>, <8>,
                                                 # encode_k512w) on the slot streams, their
                                                 # tile counters in the slots' scratch
                                                 (64, 30001, 5, 2), (300, 50001, 5, 2),
                                                 (1500, 70001, 5, 2), (3069, 100001, 4, 0)])
def test_host_batch_roundtrip(oracle, nv, plen, batch, chunk):
    n, k, thr = E.code_params(nv)
    sl = E.shard_len(nv, plen)
    pay = np.stack([synth.payload(500 + b, plen) for b in range(batch)])
    sh = np.zeros((batch, nv, sl), dtype=np.uint8)
    E.encode_host_batch(nv, pay, plen, plen, batch, sh, sl, chunk)
    for b in range(batch):
        assert b"".join(oracle.encode(nv, pay[b].tobytes())) == sh[b].tobytes(), b
    cnt = thr
    idx = np.stack([np.sort(synth.present_set(700 + b, nv, cnt)) for b in range(batch)]).astype(np.uint16)
    idx[0, -1] = idx[0, 0]  # a repeated index counts once (cnt - 1 >= k distinct)
    comp = np.stack([sh[b][idx[b]] for b in range(batch)])
    out = np.zeros((batch, sl * k), dtype=np.uint8)
    E.reconstruct_host_batch(nv, comp, sl, sl, idx, cnt, batch, out, sl * k, chunk)
    for b in range(batch):
        assert out[b][:plen].tobytes() == pay[b].tobytes(), b
        assert not out[b][plen:].any()


@pytest.mark.parametrize("nv", [600, 1024, 2500, 4096])
def test_encode_shard_base_8_aligned(oracle, nv):
    """Fast encodes with an 8-B (not 16-B) aligned shard base: 8-B stores."""
    import torch
    n, k, _ = E.code_params(nv)
    plen, batch = 70001, 2
    sl = E.shard_len(nv, plen)
    ss = (sl + 15) // 16 * 16
    ps = (plen + 15) // 16 * 16  # 16-B payload pitch: the fast kernels apply
    pay = np.zeros((batch, ps), dtype=np.uint8)
    for b in range(batch):
        pay[b, :plen] = synth.payload(50 + b, plen)
    d_pay = torch.from_numpy(pay).cuda()
    raw = torch.zeros(batch * nv * ss + 8, dtype=torch.uint8, device="cuda")
    d_sh = raw[8:]  # base 8 bytes past a 256-B aligned allocation
    assert d_sh.data_ptr() % 16 == 8
    E.encode_batch(nv, d_pay, plen, ps, batch, d_sh, ss)
    torch.cuda.synchronize()
    sh = d_sh.cpu().numpy().reshape(batch, nv, ss)[:, :, :sl]
    for b in range(batch):
        assert b"".join(oracle.encode(nv, pay[b, :plen].tobytes())) == sh[b].tobytes(), b


def test_capi_concurrent_threads(oracle):
    """The C ABI is reentrant like the reference (thread_local scratch,
    reed-solomon.hpp:198-201): host threads encoding / reconstructing at once,
    including k = 1024 encodes (the shared coefficient scratch), give the
    single-threaded results."""
    import threading
    cases = [(4096, 30001), (4096, 50001), (1024, 40001), (600, 20001), (3070, 30001), (100, 9999)]
    want = {}
    for nv, plen in cases:
        p = synth.payload(nv + plen, plen).tobytes()
        want[(nv, plen)] = (p, b"".join(oracle.encode(nv, p)))
    errors = []

    def worker(tid):
        try:
            for rep in range(3):
                nv, plen = cases[(tid + rep) % len(cases)]
                p, ref = want[(nv, plen)]
                sh = E.obtain_chunks(nv, p)
                if b"".join(sh) != ref:
                    errors.append(("encode", tid, nv))
                    continue
                n, k, thr = E.code_params(nv)
                keep = set(int(x) for x in synth.present_set(tid * 7 + rep, nv, thr))
                if decode_subset(nv, sh, keep)[:plen] != p:
                    errors.append(("reconstruct", tid, nv))
        except Exception as e:  # surfaced below
            errors.append(("exception", tid, repr(e)))

    threads = [threading.Thread(target=worker, args=(i,)) for i in range(6)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(120)
    assert not any(t.is_alive() for t in threads)
    assert not errors, errors


def test_batch_concurrent_default_stream(oracle):
    """host threads issuing the plain device-batch calls at once on
    the SAME stream (torch's default stream, handle 0) with mixed shapes, so
    the stream's scratch is shared, grown and handed to several callers: every
    call holds it until its kernels are enqueued, so each payload's gather
    order and coefficient slots are its own.  Every shard and output byte vs
    the oracle."""
    import threading
    shapes = [(1024, 100_001, 3), (4096, 60_001, 2), (1024, 5000, 5), (600, 70_001, 3),
              (2500, 20_001, 2), (1024, 300_001, 2)]
    got, errors = {}, []

    def worker(tid):
        try:
            for rep in range(3):
                nv, plen, batch = shapes[(tid + rep) % len(shapes)]
                got[(tid, rep)] = (nv, plen, batch,
                                   _batch_case(nv, plen, batch, seed0=1000 * tid + 10 * rep, pad=64))
        except Exception as e:  # surfaced below
            errors.append((tid, repr(e)))

    threads = [threading.Thread(target=worker, args=(i,)) for i in range(6)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(180)
    assert not any(t.is_alive() for t in threads)
    assert not errors, errors
    assert len(got) == 18
    for (tid, rep), (nv, plen, batch, (pay, pres, sh, el, out)) in sorted(got.items()):
        for b in range(batch):
            ref = oracle.encode(nv, pay[b].tobytes())
            assert b"".join(ref) == sh[b].tobytes(), (tid, rep, b)
            keep = [ref[i] if pres[b][i] else None for i in range(nv)]
            assert out[b].tobytes() == oracle.reconstruct(nv, keep), (tid, rep, b)


def test_release_stream_scratch():
    """ECCR_AMD_release_stream_scratch frees a stream's batch scratch; the next
    call on that stream allocates it again and is still correct."""
    import torch
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        pay, pres, sh, el, out = _batch_case(1024, 100_001, 2, seed0=55, pad=64)
    assert E.release_stream_scratch(s)
    assert not E.release_stream_scratch(s)
    with torch.cuda.stream(s):
        pay2, pres2, sh2, el2, out2 = _batch_case(1024, 100_001, 2, seed0=55, pad=64)
    torch.cuda.synchronize()
    assert (out2 == out).all() and (out2[:, :100_001] == pay2).all()
    E.release_stream_scratch(s)


@pytest.mark.parametrize("nv", [1024, 4096])
def test_batch_past_4GiB(oracle, nv):
    """both headline workloads address shard bytes beyond
    2^32 (config 2: 16.6 GB of shards).  B = 1100 x 1 MB with 64-B rows puts
    4.47 GB (nv = 1024) / 4.6 GB (nv = 4096) of shards on the device; payloads
    0 and B - 1 and the payloads on either side of (and straddling) the 2^32
    byte offset are compared byte for byte with the oracle (encode and
    reconstruct, reed-solomon.hpp:73-78,116-127); every payload round-trips."""
    import torch
    plen, batch = 1_000_000, 1100
    n, k, thr = E.code_params(nv)
    sl = E.shard_len(nv, plen)
    ss = (sl + 63) // 64 * 64
    row = nv * ss  # shard bytes per payload
    assert batch * row > (1 << 32)
    seeds = list(range(77_000, 77_000 + batch))
    d_pay = torch.empty((batch, plen), dtype=torch.uint8, device="cuda")
    for c0 in range(0, batch, 256):
        d_pay[c0:c0 + 256] = synth.payloads_torch(seeds[c0:c0 + 256], plen)
    pres = synth.present_masks([10**6 + s for s in seeds], nv, thr, n)
    d_pr = torch.from_numpy(pres).cuda()
    d_sh = _prefilled((batch, nv, ss))
    d_el = torch.zeros((batch, n), dtype=torch.int16, device="cuda")
    d_out = _prefilled((batch, sl * k))
    E.encode_batch(nv, d_pay, plen, plen, batch, d_sh, ss)
    E.error_locator(nv, d_pr, batch, d_el)
    E.reconstruct_batch(nv, d_sh, sl, ss, d_pr, d_el, batch, d_out, sl * k)
    torch.cuda.synchronize()
    assert torch.equal(d_out[:, :plen], d_pay)
    assert not d_out[:, plen:].any()
    edge = (1 << 32) // row  # the payload whose shard rows reach / straddle 2^32
    check = sorted({0, batch - 1, edge - 1, edge, edge + 1})
    assert any(b * row < (1 << 32) <= (b + 1) * row for b in check)
    for b in check:
        p = synth.payload(seeds[b], plen).tobytes()
        assert d_pay[b].cpu().numpy().tobytes() == p
        ref = oracle.encode(nv, p)
        assert b"".join(ref) == d_sh[b, :, :sl].cpu().numpy().tobytes(), b
        keep = [ref[i] if pres[b][i] else None for i in range(nv)]
        assert d_out[b].cpu().numpy().tobytes() == oracle.reconstruct(nv, keep), b
    del d_pay, d_sh, d_out
    torch.cuda.empty_cache()


@pytest.mark.parametrize("nv,plen,batch", [(3069, 1_000_000, 67), (4096, 300_001, 411)])
def test_batch_xcd_spans(oracle, nv, plen, batch):
    """reconstruct_n4096's XCD-affine tile spans (ec_device.hpp xcd_span): with
    at least 8 x grid tiles the tiles are cut into 8 contiguous spans; these
    shapes give spans of unequal length (2,077 tiles at k = 512, 2,055 at
    k = 1024) and spans that start and end inside a payload.  Every payload
    round-trips (a skipped tile would leave the 0xAA prefill); the first, the
    last and one mid-batch payload are compared with the oracle."""
    import torch
    n, k, thr = E.code_params(nv)
    sl = E.shard_len(nv, plen)
    ss = (sl + 63) // 64 * 64
    tiles = (sl // 2 + 31) // 32 * batch
    assert tiles >= 8 * 256 and tiles % 8 != 0  # the span path on a 256-CU part, unequal spans
    seeds = list(range(91_000, 91_000 + batch))
    d_pay = synth.payloads_torch(seeds, plen)
    pres = synth.present_masks([10**6 + s for s in seeds], nv, thr, n)
    d_pr = torch.from_numpy(pres).cuda()
    d_sh = _prefilled((batch, nv, ss))
    d_el = torch.zeros((batch, n), dtype=torch.int16, device="cuda")
    d_out = _prefilled((batch, sl * k))
    E.encode_batch(nv, d_pay, plen, plen, batch, d_sh, ss)
    E.error_locator(nv, d_pr, batch, d_el)
    E.reconstruct_batch(nv, d_sh, sl, ss, d_pr, d_el, batch, d_out, sl * k)
    torch.cuda.synchronize()
    assert torch.equal(d_out[:, :plen], d_pay)
    assert not d_out[:, plen:].any()
    for b in (0, batch // 2, batch - 1):
        p = synth.payload(seeds[b], plen).tobytes()
        ref = oracle.encode(nv, p)
        assert b"".join(ref) == d_sh[b, :, :sl].cpu().numpy().tobytes(), b
        keep = [ref[i] if pres[b][i] else None for i in range(nv)]
        assert d_out[b].cpu().numpy().tobytes() == oracle.reconstruct(nv, keep), b
    del d_pay, d_sh, d_out
    torch.cuda.empty_cache()


# ------------------------------------------- erasure patterns per reconstruct kernel
def _pattern_rows(nv, n, k, thr, rng):
    """One present mask per pattern the reference's gap / erased-index handling
    distinguishes (reed-solomon.hpp:83-134): exactly k, threshold, every shard
    (E == 0 erasures), all systematic rows present with some y >= k erased,
    only the systematic rows, only non-systematic rows."""
    rows = {}

    def mask(idx):
        m = np.zeros(n, dtype=np.uint8)
        m[np.asarray(sorted(idx), dtype=np.int64)] = 1
        return m

    rows["k"] = mask(rng.permutation(nv)[:k])
    rows["threshold"] = mask(rng.permutation(nv)[:thr])
    rows["all"] = mask(range(nv))
    if nv > k:
        extra = rng.permutation(np.arange(k, nv))[: max(1, (nv - k) // 2)]
        rows["systematic+some"] = mask(list(range(k)) + [int(x) for x in extra])
        rows["systematic_only"] = mask(range(k))
    if nv - k >= k:
        rows["parity_only"] = mask(k + rng.permutation(nv - k)[:k])
    return rows


def _prefilled(shape, fill=0xAA):
    import torch
    return torch.full(shape, fill, dtype=torch.uint8, device="cuda")


@pytest.mark.parametrize("seed", range(8))
def test_batch_random_shapes_and_runs(oracle, seed):
    """Random n_validators (every fast reconstruct and the generic kernel) with
    present sets shaped against the gather order (gather_order: present rows
    first, wave-major): a random subset of random size in [k, nv], one
    contiguous run, a strided set and the last rows only -- so whole waves
    of slots are full, empty or partly present -- on the device batch path,
    compared with the oracle; outputs prefilled with 0xAA."""
    import torch
    rng = np.random.default_rng(1234 + seed)
    for nv in [int(x) for x in rng.choice(
            [46, 70, 129, 200, 257, 383, 513, 700, 800, 1000, 1024, 1100, 1700, 2049, 2700, 3071, 4000],
            3, replace=False)]:
        n, k, thr = E.code_params(nv)
        plen = int(rng.integers(1, 3 * 2 * k))
        sl = E.shard_len(nv, plen)
        ss = (sl + 15) // 16 * 16

        def mask(idx):
            m = np.zeros(n, dtype=np.uint8)
            m[np.asarray(sorted(set(int(x) for x in idx)), dtype=np.int64)] = 1
            return m

        cnt = int(rng.integers(k, nv + 1))
        start = int(rng.integers(0, nv - k + 1))
        step = int(rng.integers(2, 4))
        strided = list(range(0, nv, step))[:max(k, 1)]
        strided += [i for i in range(nv) if i % step][: max(0, k - len(strided))]
        rows = [mask(rng.permutation(nv)[:cnt]), mask(range(start, start + k)), mask(strided),
                mask(range(nv - k, nv))]
        batch = len(rows)
        pay = np.stack([synth.payload(777 + 31 * seed + b + nv, plen) for b in range(batch)])
        pres = np.stack(rows)
        d_pay = torch.from_numpy(pay).cuda()
        d_sh = _prefilled((batch, nv, ss))
        d_pr = torch.from_numpy(pres).cuda()
        d_el = torch.zeros((batch, n), dtype=torch.int16, device="cuda")
        d_out = _prefilled((batch, sl * k))
        E.encode_batch(nv, d_pay, plen, plen, batch, d_sh, ss)
        torch.cuda.synchronize()
        sh_np = d_sh.cpu().numpy()
        for b in range(batch):
            gone = np.where(pres[b][:nv] == 0)[0]
            if len(gone):
                d_sh[b, torch.from_numpy(gone).cuda()] = 0x5C
        E.error_locator(nv, d_pr, batch, d_el)
        E.reconstruct_batch(nv, d_sh, sl, ss, d_pr, d_el, batch, d_out, sl * k)
        torch.cuda.synchronize()
        out = d_out.cpu().numpy()
        for b in range(batch):
            shards = [sh_np[b, i, :sl].tobytes() if pres[b][i] else None for i in range(nv)]
            want = oracle.reconstruct(nv, shards)
            assert out[b].tobytes() == want, (nv, plen, b)
            assert out[b, :plen].tobytes() == pay[b].tobytes()


@pytest.mark.parametrize("nv,plen,pad", [
    (1024, 70001, 64), (800, 33333, 16),                # reconstruct_n1024x, k = 256 (nv = n and nv < n)
    (1500, 70001, 64), (2048, 40001, 16),               # reconstruct_n4096, 2 halves, k = 256 / 512
    (2500, 70001, 64), (3070, 90001, 16), (4096, 70001, 64),  # 4 quarters, k = 512 / 1024
    (600, 50001, 64), (513, 70001, 64), (765, 40001, 16),  # reconstruct_gen, n = 1024, k = 128
    (600, 9001, 64), (300, 20001, 16), (100, 9999, 16), (46, 5001, 64),  # reconstruct_gen
    (6, 3001, 0), (20, 999, 0), (5000, 40001, 0)])     # generic kernels (incl. n = 8192)
def test_batch_patterns_every_kernel(oracle, nv, plen, pad):
    """Device batch reconstruct through ECCR_AMD_reconstruct_batch with every
    pattern class, outputs and shard padding prefilled with 0xAA (a missed
    write or a read of an absent row shows up), compared with the oracle."""
    import torch
    n, k, thr = E.code_params(nv)
    rng = np.random.default_rng(nv * 7 + plen)
    rows = _pattern_rows(nv, n, k, thr, rng)
    names = list(rows)
    batch = len(names)
    sl = E.shard_len(nv, plen)
    ss = (sl + pad - 1) // pad * pad if pad else sl
    pay = np.stack([synth.payload(9000 + nv + b, plen) for b in range(batch)])
    pres = np.stack([rows[x] for x in names])
    d_pay = torch.from_numpy(pay).cuda()
    d_sh = _prefilled((batch, nv, ss))
    d_pr = torch.from_numpy(pres).cuda()
    d_el = torch.zeros((batch, n), dtype=torch.int16, device="cuda")
    d_out = _prefilled((batch, sl * k))
    E.encode_batch(nv, d_pay, plen, plen, batch, d_sh, ss)
    torch.cuda.synchronize()
    # absent shards: garbage bytes (must never be read)
    sh_np = d_sh.cpu().numpy()
    for b in range(batch):
        gone = np.where(pres[b][:nv] == 0)[0]
        d_sh[b, torch.from_numpy(gone).cuda()] = 0x5C
    E.error_locator(nv, d_pr, batch, d_el)
    E.reconstruct_batch(nv, d_sh, sl, ss, d_pr, d_el, batch, d_out, sl * k)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    for b, name in enumerate(names):
        ref = oracle.encode(nv, pay[b].tobytes())
        assert b"".join(ref) == sh_np[b][:, :sl].tobytes(), (name, "encode")
        keep = [ref[i] if pres[b][i] else None for i in range(nv)]
        assert out[b].tobytes() == oracle.reconstruct(nv, keep), name
        assert out[b][:plen].tobytes() == pay[b].tobytes(), name


@pytest.mark.parametrize("nv,plen,pad", [(1024, 40001, 64), (600, 30001, 64), (4096, 50001, 64),
                                         (1500, 30001, 16), (20, 999, 0)])
def test_shared_patterns(oracle, nv, plen, pad):
    """Per-pattern locator dedup: many payloads share a
    few erasure patterns.  ECCR_AMD_error_locator computes each distinct one
    once (its rows still equal oracle.error_poly), ECCR_AMD_dedup_patterns
    finds the leaders, and ECCR_AMD_reconstruct_batch_patterns reads the shared
    rows; every output equals the oracle's."""
    import torch
    n, k, thr = E.code_params(nv)
    base = [synth.present_mask(77 + j, nv, thr, n) for j in range(3)]
    # same sets also arrive as bytes other than 1 and with flags past nv set
    alt = base[1].copy()
    alt[alt == 1] = 7
    if n > nv:
        alt[nv:] = 1
    which = [0, 1, 0, 0, 2, 1, 2, 0, 1, 0, 0, 2]
    batch = len(which)
    pres = np.stack([alt if (w == 1 and b % 2) else base[w] for b, w in enumerate(which)])
    d_pr = torch.from_numpy(pres).cuda()
    d_el = torch.zeros((batch, n), dtype=torch.int16, device="cuda")
    E.error_locator(nv, d_pr, batch, d_el)
    d_pat = torch.zeros(batch, dtype=torch.int32, device="cuda")
    E.dedup_patterns(nv, d_pr, batch, d_pat)
    torch.cuda.synchronize()
    el = d_el.cpu().numpy().view(np.uint16)
    first = {}
    want = [first.setdefault(w, b) for b, w in enumerate(which)]
    assert d_pat.cpu().numpy().tolist() == want
    for b in range(batch):
        erased = (pres[b][:n] == 0).astype(np.uint8)
        erased[nv:] = 1
        ep = oracle.error_poly(erased, n)[:n].astype(np.int64) % 65535
        assert ((el[b].astype(np.int64) % 65535) == ep).all(), b
    # reconstruct with ONE present row / locator per distinct pattern
    sl = E.shard_len(nv, plen)
    ss = (sl + pad - 1) // pad * pad if pad else sl
    pay = np.stack([synth.payload(4000 + b, plen) for b in range(batch)])
    d_pay = torch.from_numpy(pay).cuda()
    d_sh = _prefilled((batch, nv, ss))
    E.encode_batch(nv, d_pay, plen, plen, batch, d_sh, ss)
    d_rows = torch.from_numpy(np.stack(base)).cuda()
    d_rel = torch.zeros((3, n), dtype=torch.int16, device="cuda")
    E.error_locator_patterns(nv, d_rows, None, 3, d_rel)
    d_idx = torch.tensor(which, dtype=torch.int32, device="cuda")
    d_out = _prefilled((batch, sl * k))
    E.reconstruct_batch_patterns(nv, d_sh, sl, ss, d_rows, d_rel, d_idx, batch, d_out, sl * k)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    sh = d_sh.cpu().numpy()[:, :, :sl]
    for b, w in enumerate(which):
        shards = [sh[b][i].tobytes() for i in range(nv)]
        keep = [shards[i] if base[w][i] else None for i in range(nv)]
        assert out[b].tobytes() == oracle.reconstruct(nv, keep), b


def test_locator_cache_eviction(oracle):
    """More distinct patterns than the per-call locator cache holds (64): every
    miss past the cap recycles the least recent entry's device buffers; results
    stay bit-exact, a re-used recent pattern hits, an evicted one misses."""
    import time
    nv, plen = 1024, 3000
    n, k, thr = E.code_params(nv)
    p = synth.payload(99, plen).tobytes()
    sh = E.obtain_chunks(nv, p)
    sets = [set(int(x) for x in synth.present_set(50_000 + j, nv, thr)) for j in range(80)]
    h0, m0 = E.locator_cache_stats()
    t0 = time.perf_counter()
    for j, keep in enumerate(sets):
        out = decode_subset(nv, sh, keep)
        if j % 9 == 0 or j >= 70:
            assert out == oracle.reconstruct(nv, [sh[i] if i in keep else None for i in range(nv)]), j
        assert out[:plen] == p
    per_miss_ms = (time.perf_counter() - t0) / len(sets) * 1e3
    h1, m1 = E.locator_cache_stats()
    assert (h1 - h0, m1 - m0) == (0, 80)
    assert decode_subset(nv, sh, sets[79])[:plen] == p  # recent: hit
    assert decode_subset(nv, sh, sets[0])[:plen] == p   # evicted: miss
    h2, m2 = E.locator_cache_stats()
    assert (h2 - h1, m2 - m1) == (1, 1)
    print(f"per-call reconstruct with a locator miss: {per_miss_ms:.3f} ms")


def test_locator_cache_per_call(oracle):
    """ECCR_reconstruct computes a pattern's locator once per device and then
    reuses it (the same validators missing for every block)."""
    nv = 1024
    n, k, thr = E.code_params(nv)
    keep = set(int(x) for x in synth.present_set(31337, nv, thr))
    h0, m0 = E.locator_cache_stats()
    for rep in range(4):
        p = synth.payload(600 + rep, 20000 + rep).tobytes()
        sh = E.obtain_chunks(nv, p)
        out = decode_subset(nv, sh, keep)
        assert out == oracle.reconstruct(nv, [sh[i] if i in keep else None for i in range(nv)])
    h1, m1 = E.locator_cache_stats()
    assert m1 - m0 == 1 and h1 - h0 == 3


# ----------------------------------------- host batches at the config-5 sizes (row f2)
README_SIZES = [15, 300, 5000, 100_000, 1_000_000, 10_000_000]  # README.md:50-84


def _pinned_like(a):
    """a copy of numpy array `a` in pinned host memory (ECCR_AMD_host_alloc),
    viewed as numpy; freed with the returned handle"""
    import ctypes
    ptr = E.lib().ECCR_AMD_host_alloc(a.nbytes)
    assert ptr
    buf = (ctypes.c_uint8 * a.nbytes).from_address(ptr)
    v = np.frombuffer(buf, dtype=a.dtype).reshape(a.shape)
    v[...] = a
    return v, ptr


def _host_roundtrip(oracle, nv, plen, batch, chunk, seed, shared=False, check_all=True,
                    pinned=False):
    n, k, thr = E.code_params(nv)
    sl = E.shard_len(nv, plen)
    pay = np.stack([synth.payload(seed + b, plen) for b in range(batch)])
    sh = np.full((batch, nv, sl), 0xAA, dtype=np.uint8)
    if pinned:  # pinned host buffers (device-mapped): the pipeline's fast paths
        return _host_roundtrip_pinned(oracle, nv, plen, batch, chunk, seed, pay, sh)
    E.encode_host_batch(nv, pay, plen, plen, batch, sh, sl, chunk)
    for b in (range(batch) if check_all else [0, batch - 1]):
        assert b"".join(oracle.encode(nv, pay[b].tobytes())) == sh[b].tobytes(), (plen, b)
    if shared:  # one validator set for every payload, listed in different orders
        s0 = synth.present_set(seed, nv, thr)
        idx = np.stack([np.random.default_rng(b).permutation(s0) for b in range(batch)]).astype(np.uint16)
    else:
        idx = np.stack([synth.present_set(seed + 7 * b, nv, thr) for b in range(batch)]).astype(np.uint16)
    comp = np.stack([sh[b][idx[b]] for b in range(batch)])
    out = np.full((batch, sl * k), 0xAA, dtype=np.uint8)
    E.reconstruct_host_batch(nv, comp, sl, sl, idx, thr, batch, out, sl * k, chunk)
    for b in range(batch):
        assert out[b][:plen].tobytes() == pay[b].tobytes(), (plen, b)
        assert not out[b][plen:].any(), (plen, b)
    for b in (range(batch) if check_all else [0]):
        kk = set(int(x) for x in idx[b])
        keep = [sh[b][i].tobytes() if i in kk else None for i in range(nv)]
        assert out[b].tobytes() == oracle.reconstruct(nv, keep), (plen, b)


def _host_roundtrip_pinned(oracle, nv, plen, batch, chunk, seed, pay, sh):
    n, k, thr = E.code_params(nv)
    sl = E.shard_len(nv, plen)
    held = []
    try:
        pay_p, q = _pinned_like(pay)
        held.append(q)
        sh_p, q = _pinned_like(sh)
        held.append(q)
        E.encode_host_batch(nv, pay_p, plen, plen, batch, sh_p, sl, chunk)
        for b in range(batch):
            assert b"".join(oracle.encode(nv, pay[b].tobytes())) == sh_p[b].tobytes(), (plen, b)
        idx = np.stack([synth.present_set(seed + 7 * b, nv, thr) for b in range(batch)]).astype(np.uint16)
        comp_p, q = _pinned_like(np.stack([sh_p[b][idx[b]] for b in range(batch)]))
        held.append(q)
        idx_p, q = _pinned_like(idx)
        held.append(q)
        out_p, q = _pinned_like(np.full((batch, sl * k), 0xAA, dtype=np.uint8))
        held.append(q)
        E.reconstruct_host_batch(nv, comp_p, sl, sl, idx_p, thr, batch, out_p, sl * k, chunk)
        for b in range(batch):
            kk = set(int(x) for x in idx[b])
            keep = [sh_p[b][i].tobytes() if i in kk else None for i in range(nv)]
            assert out_p[b].tobytes() == oracle.reconstruct(nv, keep), (plen, b)
            assert out_p[b][:plen].tobytes() == pay[b].tobytes(), (plen, b)
    finally:
        for q in held:
            E.lib().ECCR_AMD_host_free(q)


@pytest.mark.parametrize("nv,plen,batch,chunk", [(1024, 1_000_000, 7, 2), (1024, 300, 50, 0),
                                                  (600, 100_001, 9, 4), (4096, 65_537, 5, 0)])
def test_host_batch_pinned(oracle, nv, plen, batch, chunk):
    """Host batches in pinned memory (ECCR_AMD_host_alloc, as a real caller
    allocates them for full PCIe rate), odd sizes included, vs the oracle."""
    _host_roundtrip(oracle, nv, plen, batch, chunk, seed=plen + nv, pinned=True)


@pytest.mark.parametrize("plen,batch", [(15, 300), (300, 100), (10_000_000, 2)])
def test_host_batch_config5_sizes(oracle, plen, batch):
    """The 15 B, 300 B and 10 MB classes of the config-5 stream through the
    host-batch pipeline with automatic chunking (chunk = 0), nv = 1024."""
    _host_roundtrip(oracle, 1024, plen, batch, 0, seed=plen, check_all=plen < 10_000_000)


def test_host_batch_shared_patterns(oracle):
    """Every payload of the host batch has the same validator set (in different
    orders): one locator per chunk, results unchanged."""
    _host_roundtrip(oracle, 1024, 5000, 40, 0, seed=17, shared=True)
    _host_roundtrip(oracle, 600, 5000, 9, 4, seed=18, shared=True)


def test_host_batch_mixed_stream(oracle):
    """Config 5 shape on one GPU: the six README sizes round-robin through the
    host-batch pipeline (chunk = 0), every result checked."""
    for rnd in range(2):
        for j, plen in enumerate(README_SIZES):
            batch = {15: 64, 300: 32, 5000: 16, 100_000: 8, 1_000_000: 3, 10_000_000: 1}[plen]
            _host_roundtrip(oracle, 1024, plen, batch, 0, seed=1000 * rnd + j,
                            check_all=plen <= 100_000)


@pytest.mark.parametrize("nv,lo,hi", [(4096, 0, 2048), (4096, 1024, 3072), (4096, 3000, 4096),
                                       (3500, 0, 1500), (2048, 1024, 2048), (1500, 0, 1024),
                                       (2500, 1024, 2048)])
def test_batch_empty_quarters(oracle, nv, lo, hi):
    """n = 2048 / 4096 reconstruct with every present shard in [lo, hi), so
    whole 1024-row quarters hold no present row (clustered outages: a quarter's
    gather is all-absent, its IFFT zero), mixed in one batch with payloads
    whose shards span every quarter; every output byte vs the oracle."""
    import torch
    n, k, thr = E.code_params(nv)
    plen, batch = 20_011, 4
    sl = E.shard_len(nv, plen)
    ss = (sl + 63) // 64 * 64
    rng = np.random.default_rng(nv + lo)
    pay = np.stack([synth.payload(31 * nv + b, plen) for b in range(batch)])
    pres = np.zeros((batch, n), dtype=np.uint8)
    for b in range(batch):
        cnt = [thr, k, min(hi - lo, thr + 5), thr][b]
        pool = np.arange(lo, min(hi, nv)) if b != 3 else np.arange(nv)
        pres[b, rng.choice(pool, size=min(cnt, len(pool)), replace=False)] = 1
    d_pay = torch.from_numpy(pay).cuda()
    d_sh = torch.zeros((batch, nv, ss), dtype=torch.uint8, device="cuda")
    d_pr = torch.from_numpy(pres).cuda()
    d_el = torch.zeros((batch, n), dtype=torch.int16, device="cuda")
    d_out = torch.full((batch, sl * k), 0xAA, dtype=torch.uint8, device="cuda")
    E.encode_batch(nv, d_pay, plen, plen, batch, d_sh, ss)
    E.error_locator(nv, d_pr, batch, d_el)
    E.reconstruct_batch(nv, d_sh, sl, ss, d_pr, d_el, batch, d_out, sl * k)
    torch.cuda.synchronize()
    sh = d_sh.cpu().numpy()
    out = d_out.cpu().numpy()
    for b in range(batch):
        keep = [sh[b, v, :sl].tobytes() if pres[b, v] else None for v in range(nv)]
        assert out[b].tobytes() == oracle.reconstruct(nv, keep), (nv, lo, hi, b)
        assert out[b, :plen].tobytes() == pay[b].tobytes()


# ------------------------------------------------------- caller-owned scratch / hipGraph
@pytest.mark.parametrize("use_ws", [True, False])
@pytest.mark.parametrize("nv,plen,batch", [(1024, 100_003, 6), (4096, 30_001, 3), (600, 50_001, 4),
                                           (20000, 9_001, 2)])
def test_graph_capture_ws(oracle, nv, plen, batch, use_ws):
    """The batch calls captured into a hipGraph (torch.cuda.CUDAGraph) and
    replayed on new inputs: encode + error locator + reconstruct, every shard
    and every output byte vs the oracle.  use_ws: the *_ws calls on one
    caller-owned workspace (stream order); else the plain calls, whose scratch
    is private to the stream they were warmed up on (no allocation, event or
    host sync once warm: ec_amd.h)."""
    import torch
    n, k, thr = E.code_params(nv)
    sl = E.shard_len(nv, plen)
    ss = (sl + 63) // 64 * 64
    need = E.workspace_bytes(nv, plen, batch)
    # the shapes do need scratch; the locator only where it deduplicates (n > 4096)
    assert (need[1] > 0) == (n > 4096) and (nv > 4096 or need[2] > 0)
    ws = torch.empty(max(need), dtype=torch.uint8, device="cuda")
    d_pay = torch.empty((batch, plen), dtype=torch.uint8, device="cuda")
    d_sh = torch.full((batch, nv, ss), 0xAA, dtype=torch.uint8, device="cuda")
    d_pr = torch.empty((batch, n), dtype=torch.uint8, device="cuda")
    d_el = torch.empty((batch, n), dtype=torch.int16, device="cuda")
    d_out = torch.full((batch, sl * k), 0xAA, dtype=torch.uint8, device="cuda")

    def fill(seed):
        pay = np.stack([synth.payload(seed * 100 + b, plen) for b in range(batch)])
        cnt = thr if seed % 2 else k
        pres = np.stack([synth.present_mask(seed * 1000 + b, nv, cnt, n) for b in range(batch)])
        d_pay.copy_(torch.from_numpy(pay))
        d_pr.copy_(torch.from_numpy(pres))
        return pay, pres

    def step():
        if use_ws:
            E.encode_batch_ws(nv, d_pay, plen, plen, batch, d_sh, ss, ws)
            E.error_locator_ws(nv, d_pr, batch, d_el, ws)
            E.reconstruct_batch_ws(nv, d_sh, sl, ss, d_pr, d_el, batch, d_out, sl * k, ws)
        else:
            E.encode_batch(nv, d_pay, plen, plen, batch, d_sh, ss)
            E.error_locator(nv, d_pr, batch, d_el)
            E.reconstruct_batch(nv, d_sh, sl, ss, d_pr, d_el, batch, d_out, sl * k)

    fill(1)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()  # outside capture: kernel attributes, tables, fold, the stream's scratch
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        step()
    for seed in (2, 3):
        pay, pres = fill(seed)
        g.replay()
        torch.cuda.synchronize()
        sh = d_sh.cpu().numpy()
        out = d_out.cpu().numpy()
        for b in range(batch):
            ref = oracle.encode(nv, pay[b].tobytes())
            assert [sh[b, v, :sl].tobytes() for v in range(nv)] == ref, (nv, seed, b)
            keep = [ref[v] if pres[b, v] else None for v in range(nv)]
            assert out[b].tobytes() == oracle.reconstruct(nv, keep), (nv, seed, b)
            assert out[b, :plen].tobytes() == pay[b].tobytes()


def test_workspace_too_small_is_reported():
    """A *_ws call whose workspace is below the queried size (or misaligned)
    returns an error and launches nothing (the output stays untouched)."""
    import torch
    nv, plen, batch = 1024, 70_001, 3
    n, k, thr = E.code_params(nv)
    sl = E.shard_len(nv, plen)
    ss = (sl + 63) // 64 * 64
    _, wl, wr = E.workspace_bytes(nv, plen, batch)
    d_sh = torch.zeros((batch, nv, ss), dtype=torch.uint8, device="cuda")
    d_pr = torch.from_numpy(np.stack([synth.present_mask(b, nv, thr, n) for b in range(batch)])).cuda()
    d_el = torch.zeros((batch, n), dtype=torch.int16, device="cuda")
    d_out = torch.full((batch, sl * k), 0x5A, dtype=torch.uint8, device="cuda")
    small = torch.empty(wr - 256, dtype=torch.uint8, device="cuda")
    with pytest.raises(E.ECError) as e:
        E.reconstruct_batch_ws(nv, d_sh, sl, ss, d_pr, d_el, batch, d_out, sl * k, small)
    assert e.value.tag == E.Tag.UNKNOWN_RECONSTRUCTION and "workspace" in E.last_error()
    big = torch.empty(max(wl, wr) + 512, dtype=torch.uint8, device="cuda")
    with pytest.raises(E.ECError):  # misaligned
        E.reconstruct_batch_ws(nv, d_sh, sl, ss, d_pr, d_el, batch, d_out, sl * k, big[1:])
    assert wl == 0  # n <= 4096: the locator computes every row, no dedup scratch
    E.error_locator_ws(nv, d_pr, batch, d_el, big[1:])  # needs none, so any workspace will do
    torch.cuda.synchronize()
    assert bool((d_out == 0x5A).all())


# ------------------------------------------------------- runtime robustness
def test_scratch_failure_is_reported(oracle):
    """A shape whose per-device scratch cannot be had (here: capped below its
    need, as when hipMalloc fails) returns an error and launches nothing;
    with the cap lifted the same calls are bit-exact again."""
    import torch
    nv, plen = 4096, 30001  # the k = 1024 encode takes its tile counter from scratch (256 B)
    p = synth.payload(1, plen).tobytes()
    E.set_scratch_limit(128)
    try:
        with pytest.raises(E.ECError) as e:
            E.obtain_chunks(nv, p)
        assert e.value.tag == E.Tag.UNKNOWN_CODE_PARAM
        assert "scratch" in E.last_error()
        sl = E.shard_len(nv, plen)
        ss = (sl + 15) // 16 * 16
        d_pay = torch.from_numpy(np.frombuffer(p, np.uint8).copy()).cuda()
        d_sh = torch.zeros((1, nv, ss), dtype=torch.uint8, device="cuda")
        with pytest.raises(E.ECError):
            E.encode_batch(nv, d_pay, plen, plen, 1, d_sh, ss)
        # n = 65536 reconstruct runs the generic kernel with global scratch
        nv2 = 65536
        n2, k2, _ = E.code_params(nv2)
        sh2 = oracle.encode(nv2, synth.payload(2, 3 * k2 + 1).tobytes())
        with pytest.raises(E.ECError) as e2:
            E.reconstruct(nv2, [(i, sh2[i]) for i in range(k2, 2 * k2)])
        assert e2.value.tag == E.Tag.UNKNOWN_RECONSTRUCTION
    finally:
        E.set_scratch_limit(0)
    assert E.obtain_chunks(nv, p) == oracle.encode(nv, p)


def test_locator_and_scratch_after_thread_exit(oracle):
    """Locator-cache entries and the per-call scratch are used by short-lived
    threads, whose streams are destroyed at exit; later calls on other threads
    hit, evict and recycle those entries and lease the scratch again (round 5:
    an event recorded on a destroyed stream was synchronised on and HIP
    reported "operation not permitted on an event last recorded in a
    capturing stream")."""
    import threading
    nv, plen = 1024, 3000
    n, k, thr = E.code_params(nv)
    p = synth.payload(7, plen).tobytes()
    sh = E.obtain_chunks(nv, p)
    sets = [set(int(x) for x in synth.present_set(70_000 + j, nv, thr)) for j in range(72)]
    errs = []

    def run(js):
        try:
            for j in js:
                assert decode_subset(nv, sh, sets[j])[:plen] == p, j
        except Exception as e:  # reported by the main thread
            errs.append(e)

    for t0 in range(0, 24, 4):  # 6 threads x 4 patterns, each thread gone before the next
        t = threading.Thread(target=run, args=(range(t0, t0 + 4),))
        t.start()
        t.join()
    assert not errs, errs
    run([0, 5, 23])  # hits on entries created by exited threads
    run(range(24, 72))  # misses: recycle the least recent entries (the exited threads')
    run(range(0, 8))  # evicted by now: misses again
    assert not errs, errs
    keep = sets[3]
    assert decode_subset(nv, sh, keep) == oracle.reconstruct(nv, [sh[i] if i in keep else None for i in range(nv)])


def test_thread_exit_releases_contexts():
    """Each host thread's C-ABI context (stream, pinned and device staging) is
    released when the thread exits: many short-lived threads leave device
    memory where it was."""
    import threading
    import torch
    nv, plen = 1024, 1_000_000
    p = synth.payload(3, plen).tobytes()
    n, k, thr = E.code_params(nv)
    keep = set(int(x) for x in synth.present_set(5, nv, thr))

    def one():
        sh = E.obtain_chunks(nv, p)
        assert E.reconstruct(nv, [(i, sh[i]) for i in sorted(keep)])[:plen] == p

    t = threading.Thread(target=one)  # warm the per-device state
    t.start()
    t.join()
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info()[0]
    for _ in range(48):
        t = threading.Thread(target=one)
        t.start()
        t.join()
    torch.cuda.synchronize()
    free1 = torch.cuda.mem_get_info()[0]
    # each context holds >= 9 MB of device staging (4 MB shards in, 4 MB out, 1 MB payload)
    assert free0 - free1 < 64 << 20, (free0, free1)


FIRST_CALLS = r'''
import sys, threading
sys.path[:0] = [{pkg!r}, {orc!r}]
import ecc_amd as E, oracle, synth
o = oracle.Oracle()
cases = [(1024, 40001), (4096, 30001), (600, 20001), (1500, 20001), (2500, 20001), (100, 9999), (20, 999), (3070, 30001)]
want = {{}}
for nv, plen in cases:
    p = synth.payload(nv, plen).tobytes()
    want[nv] = (p, b"".join(o.encode(nv, p)))
go = threading.Barrier(len(cases))
bad = []
def worker(nv):
    p, ref = want[nv]
    go.wait()  # every thread makes its first library call at once
    sh = E.obtain_chunks(nv, p)
    if b"".join(sh) != ref:
        bad.append(("encode", nv))
        return
    n, k, thr = E.code_params(nv)
    keep = sorted(int(x) for x in synth.present_set(nv + 1, nv, thr))
    if E.reconstruct(nv, [(i, sh[i]) for i in keep])[:len(p)] != p:
        bad.append(("reconstruct", nv))
ts = [threading.Thread(target=worker, args=(nv,)) for nv, _ in cases]
[t.start() for t in ts]
[t.join(240) for t in ts]
print("BAD", bad)
sys.exit(1 if bad or any(t.is_alive() for t in ts) else 0)
'''


def test_fresh_process_concurrent_first_calls():
    """In a fresh process, threads make their FIRST library calls at the same
    moment, over shapes that use every specialised kernel (their per-device
    first-call setup races): all results equal the oracle's."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = FIRST_CALLS.format(pkg=os.path.join(root, "erasure-coding-crust_amd"),
                              orc=os.path.join(root, "oracle"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])


# ------------------------------------------- packed small-payload kernels (round 3)
@pytest.mark.parametrize("nv,plen,batch,layout", [
    (1024, 1, 37, "tight"), (1024, 15, 300, "tight"), (1024, 15, 64, "pad64"), (1024, 300, 129, "tight"),
    (1024, 511, 9, "odd"), (1024, 512, 33, "tight"), (1024, 513, 17, "pad16"), (1024, 3001, 21, "odd"),
    (1024, 5000, 40, "tight"), (1024, 5000, 24, "pad64"), (1024, 16385, 5, "odd"), (1024, 65535, 3, "tight"),
    (1024, 70001, 3, "odd"),                     # > 64 KB with odd pitches: packed tiles too
    (800, 300, 45, "tight"), (1000, 20000, 7, "pad16"), (766, 15, 80, "odd"),
    (1025, 300, 31, "tight"), (1500, 5000, 9, "odd")])  # n = 2048 encode (packed) / reconstruct_n4096
def test_packed_small_batches(oracle, nv, plen, batch, layout):
    """Small payloads (the benchmark/ sizes) and pitches the 16-B kernels cannot
    take run the packed encode_k256 / reconstruct_n1024 (flattened pieces /
    columns across payloads, any alignment): every shard byte and every output
    byte vs the oracle, shard rows and outputs prefilled with 0xAA (a write
    past a payload's pieces or columns shows up), absent rows overwritten with
    garbage.  tight: pitch = length; odd: odd payload base and pitch, shard
    pitch = shard_len + 2; padNN: pitches rounded to NN bytes."""
    import torch
    n, k, thr = E.code_params(nv)
    sl = E.shard_len(nv, plen)
    if layout == "tight":
        ps, ss, off = plen, sl, 0
    elif layout == "odd":
        ps, ss, off = plen + 3, sl + 2, 1
    else:
        pad = int(layout[3:])
        ps, ss, off = (plen + pad - 1) // pad * pad, (sl + pad - 1) // pad * pad, 0
    rng = np.random.default_rng(nv * 31 + plen)
    pay = np.stack([synth.payload(70_000 + 13 * b + plen, plen) for b in range(batch)])
    buf = np.zeros(off + batch * ps + 8, dtype=np.uint8)
    for b in range(batch):
        buf[off + b * ps: off + b * ps + plen] = pay[b]
    d_buf = torch.from_numpy(buf).cuda()
    d_pay = d_buf[off:]
    d_sh = _prefilled((batch * nv * ss,))
    E.encode_batch(nv, d_pay, plen, ps, batch, d_sh, ss)
    torch.cuda.synchronize()
    shv = d_sh.cpu().numpy().reshape(batch, nv, ss)
    refs = []
    for b in range(batch):
        ref = oracle.encode(nv, pay[b].tobytes())
        refs.append(ref)
        assert [shv[b, v, :sl].tobytes() for v in range(nv)] == ref, (b, "encode")
        assert (shv[b, :, sl:] == 0xAA).all(), (b, "shard pitch bytes written")
    cnts = [k, thr, nv]
    pres = np.stack([synth.present_mask(90_000 + b, nv, cnts[b % 3], n) for b in range(batch)])
    d_pr = torch.from_numpy(pres).cuda()
    for b in range(batch):  # absent rows: garbage that must never be read
        gone = np.where(pres[b][:nv] == 0)[0]
        if len(gone):
            d_sh.view(batch, nv, ss)[b, torch.from_numpy(gone).cuda()] = 0x5C
    d_el = torch.zeros((batch, n), dtype=torch.int16, device="cuda")
    d_out = _prefilled((batch, sl * k))
    E.error_locator(nv, d_pr, batch, d_el)
    E.reconstruct_batch(nv, d_sh, sl, ss, d_pr, d_el, batch, d_out, sl * k)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    for b in range(batch):
        keep = [refs[b][i] if pres[b][i] else None for i in range(nv)]
        assert out[b].tobytes() == oracle.reconstruct(nv, keep), (b, "reconstruct")
        assert out[b, :plen].tobytes() == pay[b].tobytes()


def test_locator_rows_every_pattern(oracle):
    """The wave-per-pattern error locator (64 <= n <= 4096) on a batch of
    distinct and repeated patterns, every row mod 65535 vs oracle.error_poly,
    for each n it covers; rows past the batch untouched."""
    import torch
    for nv in (33, 64, 100, 200, 300, 600, 1000, 1024, 1500, 2048, 3000, 4096):
        n, k, thr = E.code_params(nv)
        batch = 11
        pres = np.stack([synth.present_mask(5_000 + nv + (b % 7), nv, [k, thr, nv][b % 3], n)
                         for b in range(batch)])
        d_pr = torch.from_numpy(pres).cuda()
        d_el = torch.full((batch + 1, n), 0x1234, dtype=torch.int16, device="cuda")
        E.error_locator(nv, d_pr, batch, d_el)
        torch.cuda.synchronize()
        el = d_el.cpu().numpy().view(np.uint16)
        assert (el[batch] == 0x1234).all(), nv
        for b in range(batch):
            erased = (pres[b][:n] == 0).astype(np.uint8)
            ep = oracle.error_poly(erased, n)[:n].astype(np.int64) % 65535
            assert ((el[b].astype(np.int64) % 65535) == ep).all(), (nv, b)



@pytest.mark.parametrize("nv", [6, 16, 100, 1024])
def test_systematic_tiny_boundaries(oracle, nv):
    """the per-call decode from exactly the k systematic shards
    (systematic_tiny when k * shard_len <= 2048 B rides in the kernel
    arguments, else systematic_g) on each side of its size limit and of the
    64 / 512 B marks, through ECCR_reconstruct and
    ECCR_reconstruct_from_systematic, against the reference."""
    n, k, thr = E.code_params(nv)
    slens = set()
    for mark in (64, 512, 2048):
        s = max(2, mark // k // 2 * 2)
        slens.update(x for x in (s - 2, s, s + 2) if x >= 2)
    rng = np.random.default_rng(nv)
    for sl in sorted(slens):
        for plen in sorted({k * sl, max(1, k * (sl - 2) + 1)}):
            assert E.shard_len(nv, plen) == sl, (nv, plen, sl)
            p = rng.integers(0, 256, plen, dtype=np.uint8).tobytes()
            sh = E.obtain_chunks(nv, p)
            ref = oracle.reconstruct_from_systematic(nv, sh[:k])
            assert ref[:plen] == p
            assert E.reconstruct_from_systematic(nv, [(i, sh[i]) for i in range(k)]) == ref, (nv, plen)
            assert E.reconstruct(nv, [(i, sh[i]) for i in range(k)]) == ref, (nv, plen)


def test_encode_ws_without_counter(oracle):
    """a workspace below the queried size (here NULL / 0 bytes, as a
    caller that cached an older size would pass) runs the k = 256 / 512 / 1024
    encodes on their static tile schedule instead of failing; bit-exact."""
    import torch
    for nv, plen, B in ((1024, 70_000, 5), (600, 50_000, 3), (2500, 60_000, 3), (4096, 80_000, 3),
                         (300, 40_000, 2), (100, 40_000, 2)):
        n, k, thr = E.code_params(nv)
        assert E.workspace_bytes(nv, plen, B)[0] == 256, nv
        sl = E.shard_len(nv, plen)
        ss = (sl + 63) // 64 * 64
        pays = [synth.payload(nv * 7 + b, plen) for b in range(B)]
        d_pay = torch.from_numpy(np.stack(pays)).cuda()
        d_sh = torch.zeros((B, nv, ss), dtype=torch.uint8, device="cuda")
        E.encode_batch_ws(nv, d_pay, plen, plen, B, d_sh, ss, None)
        torch.cuda.synchronize()
        got = d_sh.cpu().numpy()
        for b in range(B):
            want = oracle.encode(nv, pays[b].tobytes())
            assert all(got[b, i, :sl].tobytes() == want[i] for i in range(nv)), (nv, b)


def test_stream_scratch_eviction_many_streams():
    """more streams than the 64 kept scratch buffers.  84 streams
    issue plain batch calls (the n = 1024 reconstruct keeps its gather order in
    its stream's scratch), so 20 are evicted and the evicted buffers are freed
    in one implicit drain (16 at a time); the first streams, evicted by then,
    run again (new buffers) and every round trip holds."""
    import ctypes
    import torch
    # distinct HIP streams (torch.cuda.Stream() hands out a pool of 32)
    hip = ctypes.CDLL("libamdhip64.so")
    raw = []
    for _ in range(84):
        h = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(h)) == 0
        raw.append(h)
    streams = [torch.cuda.ExternalStream(h.value) for h in raw]
    for j, s in enumerate(streams):
        with torch.cuda.stream(s):
            pay, pres, sh, el, out = _batch_case(1024, 20_001, 2, seed0=900 + j, pad=64)
        assert (out[:, :20_001] == pay).all(), j
    for j, s in enumerate(streams[:8]):  # evicted: allocated again
        with torch.cuda.stream(s):
            pay, pres, sh, el, out = _batch_case(1024, 30_001, 2, seed0=990 + j, pad=64)
        assert (out[:, :30_001] == pay).all(), j
    torch.cuda.synchronize()
    kept = sum(E.release_stream_scratch(s) for s in streams)
    assert kept == 64, kept  # the 64 most recent streams hold one each
    for h in raw:
        assert hip.hipStreamDestroy(h) == 0


def test_release_stream_scratch_while_leased():
    """ECCR_AMD_release_stream_scratch from one thread while another
    thread's plain calls lease that stream's scratch: a release waits for the
    lease holder to finish enqueueing, a buffer still held goes to the dead
    list, and every call's results stay exact."""
    import threading
    import time
    import torch
    s = torch.cuda.Stream()
    errs, done = [], threading.Event()

    def caller():
        try:
            for rep in range(12):
                with torch.cuda.stream(s):
                    pay, pres, sh, el, out = _batch_case(1024, 40_001 + 2 * rep, 2, seed0=70 + rep, pad=64)
                assert (out[:, :40_001 + 2 * rep] == pay).all(), rep
        except Exception as e:  # reported by the main thread
            errs.append(e)
        finally:
            done.set()

    t = threading.Thread(target=caller)
    t.start()
    releases = 0
    while not done.is_set():
        releases += E.release_stream_scratch(s)
        time.sleep(0.002)
    t.join(120)
    assert not t.is_alive() and not errs, errs
    torch.cuda.synchronize()
    E.release_stream_scratch(s)
