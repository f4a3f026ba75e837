"""ctypes mirror of the erasure_coding.h C ABI (+ the ec_amd.h device extension).

This is how Python callers (tests, bench.py) reach the HIP implementation in
lib/liberasure_coding_crust.so; names, argument meaning and error behaviour are
those of the reference's C ABI (src/erasure_coding.rs).  There is no CPU
fallback: compute calls on a machine without a HIP device return an error and
print why.

If torch is importable it is imported first, so that this library binds to the
same libamdhip64.so.7 instance torch uses (torch ships its own copy; one HIP
runtime per process) and device pointers from torch tensors are valid here.
"""
from __future__ import annotations

import ctypes as C
import enum
import os
import subprocess

try:  # one HIP runtime per process: let torch's copy be the one
    import torch  # noqa: F401
except Exception:  # pragma: no cover
    torch = None

HERE = os.path.dirname(os.path.abspath(__file__))
# ECC_AMD_LIB: an alternative build of the same library (A/B kernel experiments)
LIB_PATH = os.environ.get("ECC_AMD_LIB") or os.path.join(HERE, "lib", "liberasure_coding_crust.so")
HEADERS = [os.path.join(os.path.dirname(HERE), "include", "erasure_coding", h)
           for h in ("erasure_coding.h", "ec_amd.h")]


class Tag(enum.IntEnum):  # src/erasure_coding.rs:10-46
    OK = 0
    TOO_MANY_VALIDATORS = 1
    NOT_ENOUGH_VALIDATORS = 2
    WRONG_VALIDATOR_COUNT = 3
    NOT_ENOUGH_CHUNKS = 4
    TOO_MANY_CHUNKS = 5
    NON_UNIFORM_CHUNKS = 6
    UNEVEN_LENGTH = 7
    CHUNK_INDEX_OUT_OF_BOUNDS = 8
    BAD_PAYLOAD = 9
    INVALID_BRANCH_PROOF = 10
    BRANCH_OUT_OF_BOUNDS = 11
    UNKNOWN_RECONSTRUCTION = 12
    UNKNOWN_CODE_PARAM = 13


class DataBlock(C.Structure):
    _fields_ = [("array", C.POINTER(C.c_uint8)), ("length", C.c_ulong)]


class Chunk(C.Structure):
    _fields_ = [("data", DataBlock), ("index", C.c_ulong)]


class ChunksList(C.Structure):
    _fields_ = [("data", C.POINTER(Chunk)), ("count", C.c_ulong)]


class _OOB(C.Structure):
    _fields_ = [("chunk_index", C.c_ulong), ("n_validators", C.c_ulong)]


class _Body(C.Union):
    _fields_ = [("chunk_index_out_of_bounds", _OOB)]


class NPRSResult(C.Structure):
    _anonymous_ = ("u",)
    _fields_ = [("tag", C.c_int), ("u", _Body)]


class ECError(RuntimeError):
    def __init__(self, res: NPRSResult, where: str = ""):
        self.tag = Tag(res.tag)
        self.detail = None
        if self.tag == Tag.CHUNK_INDEX_OUT_OF_BOUNDS:
            b = res.chunk_index_out_of_bounds
            self.detail = (b.chunk_index, b.n_validators)
        super().__init__(f"{where}: {self.tag.name} {self.detail or ''}".strip())


def build(force: bool = False) -> str:
    """Compile the HIP library in-tree (hipcc --offload-arch=gfx950)."""
    args = ["make", "-s", "-C", HERE] + (["-B"] if force else [])
    subprocess.run(args, check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        ul, up, vp = C.c_ulong, C.POINTER(C.c_ulong), C.c_void_p
        sig = {
            "ECCR_get_recovery_threshold": (NPRSResult, [ul, up]),
            "ECCR_deallocate_data_block": (None, [C.POINTER(DataBlock)]),
            "ECCR_deallocate_chunk": (None, [C.POINTER(Chunk)]),
            "ECCR_deallocate_chunk_list": (None, [C.POINTER(ChunksList)]),
            "ECCR_AFFT_Table": (NPRSResult, [C.POINTER(C.c_uint16 * 65535)]),
            "ECCR_Test_MeasurePerformance": (NPRSResult, [C.POINTER(DataBlock), ul, up, up]),
            "ECCR_obtain_chunks": (NPRSResult, [ul, C.POINTER(DataBlock), C.POINTER(ChunksList)]),
            "ECCR_reconstruct_from_systematic": (NPRSResult, [ul, C.POINTER(ChunksList),
                                                              C.POINTER(DataBlock)]),
            "ECCR_reconstruct": (NPRSResult, [ul, C.POINTER(ChunksList), C.POINTER(DataBlock)]),
            "ECCR_AMD_code_params": (NPRSResult, [ul, up, up, up]),
            "ECCR_AMD_shard_len": (ul, [ul, ul]),
            "ECCR_AMD_device_count": (C.c_int, []),
            "ECCR_AMD_init_device": (NPRSResult, []),
            "ECCR_AMD_encode_batch": (NPRSResult, [ul, vp, ul, ul, ul, vp, ul, vp]),
            "ECCR_AMD_error_locator": (NPRSResult, [ul, vp, ul, vp, vp]),
            "ECCR_AMD_reconstruct_batch": (NPRSResult, [ul, vp, ul, ul, vp, vp, ul, vp, ul, vp]),
            "ECCR_AMD_systematic_batch": (NPRSResult, [ul, vp, ul, ul, ul, vp, ul, vp]),
            "ECCR_AMD_dedup_patterns": (NPRSResult, [ul, vp, ul, vp, vp]),
            "ECCR_AMD_error_locator_patterns": (NPRSResult, [ul, vp, vp, ul, vp, vp]),
            "ECCR_AMD_reconstruct_batch_patterns": (NPRSResult, [ul, vp, ul, ul, vp, vp, vp, ul, vp,
                                                                 ul, vp]),
            "ECCR_AMD_locator_cache_stats": (NPRSResult, [up, up]),
            "ECCR_AMD_encode_workspace_bytes": (ul, [ul, ul, ul]),
            "ECCR_AMD_error_locator_workspace_bytes": (ul, [ul, ul]),
            "ECCR_AMD_reconstruct_workspace_bytes": (ul, [ul, ul, ul]),
            "ECCR_AMD_encode_batch_ws": (NPRSResult, [ul, vp, ul, ul, ul, vp, ul, vp, ul, vp]),
            "ECCR_AMD_error_locator_ws": (NPRSResult, [ul, vp, ul, vp, vp, ul, vp]),
            "ECCR_AMD_reconstruct_batch_ws": (NPRSResult, [ul, vp, ul, ul, vp, vp, vp, ul, vp, ul,
                                                           vp, ul, vp]),
            "ECCR_AMD_host_alloc": (vp, [ul]),
            "ECCR_AMD_host_free": (None, [vp]),
            "ECCR_AMD_encode_host_batch": (NPRSResult, [ul, vp, ul, ul, ul, vp, ul, ul]),
            "ECCR_AMD_reconstruct_host_batch": (NPRSResult, [ul, vp, ul, ul, vp, ul, ul, vp, ul,
                                                             ul]),
            "ECCR_AMD_set_scratch_limit": (None, [ul]),
            "ECCR_AMD_release_stream_scratch": (C.c_int, [vp]),
            "ECCR_AMD_last_error": (C.c_char_p, []),
        }
        for name, (res, args) in sig.items():
            try:
                f = getattr(L, name)
            except AttributeError:
                if os.environ.get("ECC_AMD_LIB"):  # an older A/B build: newer symbols absent
                    continue
                raise
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _check(res: NPRSResult, where: str):
    if res.tag != Tag.OK:
        raise ECError(res, where)


# ------------------------------------------------------------------ host ABI


def get_recovery_threshold(nv: int) -> int:
    out = C.c_ulong()
    _check(lib().ECCR_get_recovery_threshold(nv, C.byref(out)), "get_recovery_threshold")
    return out.value


def afft_table():
    import numpy as np
    buf = (C.c_uint16 * 65535)()
    _check(lib().ECCR_AFFT_Table(C.byref(buf)), "AFFT_Table")
    return np.frombuffer(buf, dtype=np.uint16).copy()


def code_params(nv: int):
    n, k, t = C.c_ulong(), C.c_ulong(), C.c_ulong()
    _check(lib().ECCR_AMD_code_params(nv, C.byref(n), C.byref(k), C.byref(t)), "code_params")
    return n.value, k.value, t.value


def shard_len(nv: int, payload_len: int) -> int:
    return int(lib().ECCR_AMD_shard_len(nv, payload_len))


def device_count() -> int:
    return int(lib().ECCR_AMD_device_count())


def set_scratch_limit(nbytes: int) -> None:
    lib().ECCR_AMD_set_scratch_limit(nbytes)


def release_stream_scratch(stream=None) -> bool:
    """Free the batch calls' scratch kept for `stream` (default: torch's current stream)."""
    return bool(lib().ECCR_AMD_release_stream_scratch(_stream(stream)))


def last_error() -> str:
    return lib().ECCR_AMD_last_error().decode()


def obtain_chunks(nv: int, payload: bytes) -> list[bytes]:
    """ECCR_obtain_chunks -> list of shards (index = position)."""
    buf = (C.c_uint8 * max(len(payload), 1)).from_buffer_copy(bytes(payload) or b"\0")
    db = DataBlock(C.cast(buf, C.POINTER(C.c_uint8)), len(payload))
    out = ChunksList()
    _check(lib().ECCR_obtain_chunks(nv, C.byref(db), C.byref(out)), "obtain_chunks")
    try:
        shards = [None] * out.count
        for i in range(out.count):
            ch = out.data[i]
            shards[ch.index] = C.string_at(ch.data.array, ch.data.length)
        return shards
    finally:
        lib().ECCR_deallocate_chunk_list(C.byref(out))


def _chunks_list(chunks):
    """chunks: iterable of (index, bytes|None).  Keeps buffers alive via the return."""
    items = list(chunks)
    arr = (Chunk * max(len(items), 1))()
    keep = []
    for j, (idx, data) in enumerate(items):
        if data is None or len(data) == 0:
            arr[j] = Chunk(DataBlock(None, 0), idx)
        else:
            b = (C.c_uint8 * len(data)).from_buffer_copy(bytes(data))
            keep.append(b)
            arr[j] = Chunk(DataBlock(C.cast(b, C.POINTER(C.c_uint8)), len(data)), idx)
    return ChunksList(C.cast(arr, C.POINTER(Chunk)), len(items)), (arr, keep)


def _take_block(db: DataBlock) -> bytes:
    try:
        return C.string_at(db.array, db.length)
    finally:
        lib().ECCR_deallocate_data_block(C.byref(db))


def reconstruct(nv: int, chunks) -> bytes:
    """ECCR_reconstruct; chunks = [(index, bytes or None), ...]."""
    cl, _keep = _chunks_list(chunks)
    out = DataBlock()
    _check(lib().ECCR_reconstruct(nv, C.byref(cl), C.byref(out)), "reconstruct")
    return _take_block(out)


def reconstruct_from_systematic(nv: int, chunks) -> bytes:
    cl, _keep = _chunks_list(chunks)
    out = DataBlock()
    _check(lib().ECCR_reconstruct_from_systematic(nv, C.byref(cl), C.byref(out)),
           "reconstruct_from_systematic")
    return _take_block(out)


def measure_performance(nv: int, payload: bytes):
    buf = (C.c_uint8 * max(len(payload), 1)).from_buffer_copy(bytes(payload) or b"\0")
    db = DataBlock(C.cast(buf, C.POINTER(C.c_uint8)), len(payload))
    e, d = C.c_ulong(), C.c_ulong()
    _check(lib().ECCR_Test_MeasurePerformance(C.byref(db), nv, C.byref(e), C.byref(d)),
           "Test_MeasurePerformance")
    return e.value, d.value


# ------------------------------------------------------- device batch (ec_amd.h)


def _p(x):
    """pointer of a torch tensor, a numpy array or an int."""
    if isinstance(x, int):
        return C.c_void_p(x)
    if hasattr(x, "data_ptr"):
        return C.c_void_p(x.data_ptr())
    return C.c_void_p(x.ctypes.data)


def _stream(stream):
    if stream is None:
        return C.c_void_p(torch.cuda.current_stream().cuda_stream) if torch is not None else None
    return C.c_void_p(stream if isinstance(stream, int) else stream.cuda_stream)


def encode_batch(nv, d_payloads, payload_len, payload_stride, batch, d_shards, shard_stride,
                 stream=None):
    _check(lib().ECCR_AMD_encode_batch(nv, _p(d_payloads), payload_len, payload_stride, batch,
                                       _p(d_shards), shard_stride, _stream(stream)),
           "encode_batch")


def error_locator(nv, d_present, batch, d_err_log, stream=None):
    _check(lib().ECCR_AMD_error_locator(nv, _p(d_present), batch, _p(d_err_log), _stream(stream)),
           "error_locator")


def reconstruct_batch(nv, d_shards, shard_len_, shard_stride, d_present, d_err_log, batch, d_out,
                      out_stride, stream=None):
    _check(lib().ECCR_AMD_reconstruct_batch(nv, _p(d_shards), shard_len_, shard_stride,
                                            _p(d_present), _p(d_err_log), batch, _p(d_out),
                                            out_stride, _stream(stream)),
           "reconstruct_batch")


def dedup_patterns(nv, d_present, batch, d_pattern, stream=None):
    """d_pattern[b] (uint32) = a row with the same erasure pattern as b that is its own
    leader (d_pattern[l] == l), or b itself (ec_amd.h)."""
    _check(lib().ECCR_AMD_dedup_patterns(nv, _p(d_present), batch, _p(d_pattern), _stream(stream)),
           "dedup_patterns")


def error_locator_patterns(nv, d_present, d_pattern, batch, d_err_log, stream=None):
    _check(lib().ECCR_AMD_error_locator_patterns(nv, _p(d_present),
                                                 None if d_pattern is None else _p(d_pattern),
                                                 batch, _p(d_err_log), _stream(stream)),
           "error_locator_patterns")


def reconstruct_batch_patterns(nv, d_shards, shard_len_, shard_stride, d_present, d_err_log,
                               d_pattern, batch, d_out, out_stride, stream=None):
    """reconstruct_batch where payload b uses row d_pattern[b] of d_present / d_err_log."""
    _check(lib().ECCR_AMD_reconstruct_batch_patterns(
        nv, _p(d_shards), shard_len_, shard_stride, _p(d_present), _p(d_err_log),
        None if d_pattern is None else _p(d_pattern), batch, _p(d_out), out_stride,
        _stream(stream)), "reconstruct_batch_patterns")


def workspace_bytes(nv, payload_len, batch):
    """(encode, error_locator, reconstruct) device scratch bytes of a batch shape."""
    sl = shard_len(nv, payload_len)
    L = lib()
    return (int(L.ECCR_AMD_encode_workspace_bytes(nv, payload_len, batch)),
            int(L.ECCR_AMD_error_locator_workspace_bytes(nv, batch)),
            int(L.ECCR_AMD_reconstruct_workspace_bytes(nv, sl, batch)))


def _ws(ws):
    if ws is None:
        return None, 0
    return _p(ws), (ws.numel() * ws.element_size() if hasattr(ws, "numel") else ws.nbytes)


def encode_batch_ws(nv, d_payloads, payload_len, payload_stride, batch, d_shards, shard_stride,
                    ws, stream=None):
    """encode_batch on caller-owned scratch `ws` (graph-capture-safe after one warm call)."""
    wp, wb = _ws(ws)
    _check(lib().ECCR_AMD_encode_batch_ws(nv, _p(d_payloads), payload_len, payload_stride, batch,
                                          _p(d_shards), shard_stride, wp, wb, _stream(stream)),
           "encode_batch_ws")


def error_locator_ws(nv, d_present, batch, d_err_log, ws, stream=None):
    wp, wb = _ws(ws)
    _check(lib().ECCR_AMD_error_locator_ws(nv, _p(d_present), batch, _p(d_err_log), wp, wb,
                                           _stream(stream)), "error_locator_ws")


def reconstruct_batch_ws(nv, d_shards, shard_len_, shard_stride, d_present, d_err_log, batch,
                         d_out, out_stride, ws, d_pattern=None, stream=None):
    wp, wb = _ws(ws)
    _check(lib().ECCR_AMD_reconstruct_batch_ws(
        nv, _p(d_shards), shard_len_, shard_stride, _p(d_present), _p(d_err_log),
        None if d_pattern is None else _p(d_pattern), batch, _p(d_out), out_stride, wp, wb,
        _stream(stream)), "reconstruct_batch_ws")


def locator_cache_stats():
    h, m = C.c_ulong(), C.c_ulong()
    _check(lib().ECCR_AMD_locator_cache_stats(C.byref(h), C.byref(m)), "locator_cache_stats")
    return h.value, m.value


def systematic_batch(nv, d_shards, shard_len_, shard_stride, batch, d_out, out_stride, stream=None):
    _check(lib().ECCR_AMD_systematic_batch(nv, _p(d_shards), shard_len_, shard_stride, batch,
                                           _p(d_out), out_stride, _stream(stream)),
           "systematic_batch")


# --------------------------------------------------- host batches (ec_amd.h)


def encode_host_batch(nv, h_payloads, payload_len, payload_stride, batch, h_shards, shard_stride,
                      chunk=0):
    """payloads [batch][payload_stride] (host) -> shards [batch][nv][shard_stride] (host)."""
    _check(lib().ECCR_AMD_encode_host_batch(nv, _p(h_payloads), payload_len, payload_stride,
                                            batch, _p(h_shards), shard_stride, chunk),
           "encode_host_batch")


def reconstruct_host_batch(nv, h_shards, shard_len_, shard_stride, h_index, count, batch, h_out,
                           out_stride, chunk=0):
    """present shards compacted [batch][count][shard_stride] + uint16 indices
    [batch][count] (host) -> payload bytes [batch][out_stride] (host)."""
    _check(lib().ECCR_AMD_reconstruct_host_batch(nv, _p(h_shards), shard_len_, shard_stride,
                                                 _p(h_index), count, batch, _p(h_out), out_stride,
                                                 chunk),
           "reconstruct_host_batch")
