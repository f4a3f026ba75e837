"""CPU checks of the C-ABI library: it loads, exports every declared symbol,
and its host-side logic (parameters, validation, error mapping, skew table)
matches the reference (src/erasure_coding.rs, test/erasure_coding/reconstruct.cpp).
No compute call needs a GPU here; on a GPU-less machine the compute entry
points must fail loudly (there is no CPU fallback).
"""
import hashlib
import re
import subprocess

import pytest

import ecc_amd as E


def test_library_exports_every_declared_symbol():
    declared = set()
    for h in E.HEADERS:
        declared |= set(re.findall(r"\b(ECCR_\w+)\s*\(", open(h).read()))
    assert len(declared) >= 9 + 9
    out = subprocess.run(["nm", "-D", "--defined-only", E.build()], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (ECCR_\w+)", out))
    assert declared <= exported, declared - exported
    for name in declared:
        getattr(E.lib(), name)


def test_reference_nine_symbols():  # the cbindgen surface of src/erasure_coding.rs
    for name in ("ECCR_get_recovery_threshold", "ECCR_deallocate_data_block",
                 "ECCR_deallocate_chunk", "ECCR_deallocate_chunk_list", "ECCR_AFFT_Table",
                 "ECCR_Test_MeasurePerformance", "ECCR_obtain_chunks",
                 "ECCR_reconstruct_from_systematic", "ECCR_reconstruct"):
        getattr(E.lib(), name)


def test_struct_layout():
    import ctypes as C
    assert C.sizeof(E.DataBlock) == 16 and C.sizeof(E.Chunk) == 24
    assert C.sizeof(E.ChunksList) == 16 and C.sizeof(E.NPRSResult) == 24


@pytest.mark.parametrize("nv,thr", [(5, 2), (100, 34), (6, 2), (1024, 342), (65536, 21846)])
def test_recovery_threshold(nv, thr):  # reconstruct.cpp:293-313
    assert E.get_recovery_threshold(nv) == thr


@pytest.mark.parametrize("nv,tag", [(1, E.Tag.NOT_ENOUGH_VALIDATORS), (0, E.Tag.NOT_ENOUGH_VALIDATORS),
                                    (90000, E.Tag.TOO_MANY_VALIDATORS),
                                    (65537, E.Tag.TOO_MANY_VALIDATORS)])
def test_recovery_threshold_errors(nv, tag):  # reconstruct.cpp:282-325
    with pytest.raises(E.ECError) as e:
        E.get_recovery_threshold(nv)
    assert e.value.tag == tag


def test_afft_table_matches_reference(golden_tables):  # reconstruct.cpp:211-225
    sk = E.afft_table()
    assert hashlib.sha256(sk.tobytes()).hexdigest() == golden_tables["skews_sha256"]


@pytest.mark.parametrize("nv,n,k", [(2, 2, 1), (6, 8, 2), (1000, 1024, 256), (1024, 1024, 256),
                                    (4096, 4096, 1024), (65536, 65536, 16384)])
def test_code_params(oracle, nv, n, k):
    assert E.code_params(nv)[:2] == (n, k) == oracle.params(nv)


@pytest.mark.parametrize("nv,plen", [(6, 1), (6, 92), (1024, 1_000_000), (4096, 300), (3, 7)])
def test_shard_len(oracle, nv, plen):
    assert E.shard_len(nv, plen) == oracle.shard_len(oracle.params(nv)[1], plen)


@pytest.mark.parametrize("nv,tag", [(70000, E.Tag.TOO_MANY_VALIDATORS),
                                    (1, E.Tag.NOT_ENOUGH_VALIDATORS)])
def test_obtain_chunks_param_errors(nv, tag):  # reconstruct.cpp:335-344
    with pytest.raises(E.ECError) as e:
        E.obtain_chunks(nv, b"payload")
    assert e.value.tag == tag


def test_obtain_chunks_empty_payload():
    with pytest.raises(E.ECError) as e:
        E.obtain_chunks(6, b"")
    assert e.value.tag == E.Tag.BAD_PAYLOAD  # reference panics; documented divergence


def test_reconstruct_validation():  # src/erasure_coding.rs:363-400
    with pytest.raises(E.ECError) as e:
        E.reconstruct(6, [(0, b"ab"), (9, b"cd")])
    assert e.value.tag == E.Tag.CHUNK_INDEX_OUT_OF_BOUNDS and e.value.detail == (9, 6)
    with pytest.raises(E.ECError) as e:
        E.reconstruct(6, [(0, b"abc"), (1, b"abc")])
    assert e.value.tag == E.Tag.UNEVEN_LENGTH
    with pytest.raises(E.ECError) as e:
        E.reconstruct(6, [(0, b"ab"), (1, b"abcd")])
    assert e.value.tag == E.Tag.NON_UNIFORM_CHUNKS
    with pytest.raises(E.ECError) as e:  # ReconstructLess1_3 (reconstruct.cpp:403-420)
        E.reconstruct(6, [(0, b"ab"), (1, None), (2, b"")])
    assert e.value.tag == E.Tag.NOT_ENOUGH_CHUNKS
    # only the first n_validators entries are considered (src/erasure_coding.rs:363)
    with pytest.raises(E.ECError) as e:
        E.reconstruct(2, [(0, None), (1, None), (0, b"ab")])
    assert e.value.tag == E.Tag.NOT_ENOUGH_CHUNKS


def test_systematic_validation():  # src/erasure_coding.rs:291-312
    with pytest.raises(E.ECError) as e:
        E.reconstruct_from_systematic(6, [(1, b"ab"), (5, b"cd")])
    assert e.value.tag == E.Tag.NOT_ENOUGH_CHUNKS
    with pytest.raises(E.ECError) as e:
        E.reconstruct_from_systematic(6, [(0, b"ab"), (1, b"abcd")])
    assert e.value.tag == E.Tag.NON_UNIFORM_CHUNKS


def test_no_gpu_fails_loudly():
    if E.device_count() > 0:
        pytest.skip("a HIP device is present")
    with pytest.raises(E.ECError) as e:
        E.obtain_chunks(6, b"some payload")
    assert e.value.tag == E.Tag.UNKNOWN_CODE_PARAM
    assert "no HIP device" in E.last_error()


def test_host_batch_validation():  # host-batch errors are raised before any device work
    import numpy as np
    sh = np.zeros((2, 3, 8), dtype=np.uint8)
    out = np.zeros((2, 16), dtype=np.uint8)
    idx = np.array([[0, 1, 7], [0, 1, 2]], dtype=np.uint16)  # 7 >= n_validators 6
    with pytest.raises(E.ECError) as e:
        E.reconstruct_host_batch(6, sh, 8, 8, idx, 3, 2, out, 16)
    assert e.value.tag == E.Tag.CHUNK_INDEX_OUT_OF_BOUNDS and e.value.detail == (7, 6)
    dup = np.array([[3, 3, 3], [0, 1, 2]], dtype=np.uint16)  # one distinct shard < k = 2
    with pytest.raises(E.ECError) as e:
        E.reconstruct_host_batch(6, sh, 8, 8, dup, 3, 2, out, 16)
    assert e.value.tag == E.Tag.NOT_ENOUGH_CHUNKS
    with pytest.raises(E.ECError) as e:
        E.reconstruct_host_batch(6, sh, 7, 8, idx, 3, 2, out, 16)
    assert e.value.tag == E.Tag.UNEVEN_LENGTH
    with pytest.raises(E.ECError) as e:
        E.encode_host_batch(6, np.zeros(4, np.uint8), 0, 4, 1, np.zeros(8, np.uint8), 8)
    assert e.value.tag == E.Tag.BAD_PAYLOAD
