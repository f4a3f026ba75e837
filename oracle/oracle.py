"""ctypes front-end to the parity checkers (TEST INFRASTRUCTURE ONLY).

``Oracle``   -> oracle/liboracle.so     (C restatement, ec_oracle.c)
``RefEC``    -> oracle/_ref/libecref.so (the reference ec-cpp itself, built by
                oracle/Makefile from /root/reference; absent if never built)

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  The product library never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libecref.so")

_u8p = C.POINTER(C.c_uint8)
_u16p = C.POINTER(C.c_uint16)
_szp = C.POINTER(C.c_size_t)

# ec_cpp::Error order (include/ec-cpp/errors.hpp:13-24), +1 (0 = ok)
ERRORS = [
    "ok", "ArgsMustBePowOf2", "WantedShardCountTooLow", "WantedShardCountTooHigh",
    "WantedPayloadShardCountTooLow", "PayloadSizeIsZero", "TooManyValidators",
    "NotEnoughValidators", "NeedMoreShards", "InconsistentShardLengths", "EmptyShard",
]


class CodecError(RuntimeError):
    def __init__(self, code: int):
        self.code = code
        self.name = ERRORS[code] if 0 <= code < len(ERRORS) else str(code)
        super().__init__(self.name)


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def _ptr(a: np.ndarray, t=_u8p):
    return a.ctypes.data_as(t)


class _Lib:
    prefix = ""

    def __init__(self, path: str):
        self.lib = C.CDLL(path)

    def _fn(self, name):
        return getattr(self.lib, self.prefix + name)

    def params(self, nv: int):
        n, k = C.c_size_t(), C.c_size_t()
        e = self._fn("params")(C.c_size_t(nv), C.byref(n), C.byref(k))
        if e:
            raise CodecError(e)
        return n.value, k.value

    def threshold(self, nv: int) -> int:
        t = C.c_size_t()
        e = self._fn("recovery_threshold" if self.prefix == "eco_" else "threshold")(
            C.c_size_t(nv), C.byref(t))
        if e:
            raise CodecError(e)
        return t.value

    @staticmethod
    def shard_len(k: int, plen: int) -> int:
        return ((plen + 1) // 2 + k - 1) // k * 2

    def _shard_args(self, shards):
        nr = len(shards)
        keep = [None if s is None else np.ascontiguousarray(np.frombuffer(bytes(s), np.uint8))
                for s in shards]
        ptrs = (_u8p * max(nr, 1))()
        lens = (C.c_size_t * max(nr, 1))()
        for i, s in enumerate(keep):
            if s is not None and s.size:
                ptrs[i] = _ptr(s)
                lens[i] = s.size
            else:
                ptrs[i] = None
                lens[i] = 0
        return keep, ptrs, lens, nr

    def reconstruct(self, nv: int, shards) -> bytes:
        keep, ptrs, lens, nr = self._shard_args(shards)
        sl = max((int(l) for l in lens[:nr]), default=0)
        n, k = self.params(nv)
        out = np.zeros(max(sl // 2 * 2 * k, 1), np.uint8)
        olen = C.c_size_t()
        e = self._fn("reconstruct")(C.c_size_t(nv), ptrs, lens, C.c_size_t(nr), _ptr(out),
                                    C.c_size_t(out.size), C.byref(olen))
        if e:
            raise CodecError(e)
        return out[: olen.value].tobytes()

    def reconstruct_from_systematic(self, nv: int, chunks) -> bytes:
        keep, ptrs, lens, nr = self._shard_args(chunks)
        sl = max((int(l) for l in lens[:nr]), default=0)
        n, k = self.params(nv)
        out = np.zeros(max(sl // 2 * 2 * k, 1), np.uint8)
        olen = C.c_size_t()
        e = self._fn("reconstruct_from_systematic")(C.c_size_t(nv), ptrs, lens, C.c_size_t(nr),
                                                    _ptr(out), C.c_size_t(out.size), C.byref(olen))
        if e:
            raise CodecError(e)
        return out[: olen.value].tobytes()


class Oracle(_Lib):
    prefix = "eco_"

    def __init__(self, path: str = ORACLE_SO):
        if not os.path.exists(path):
            build()
        super().__init__(path)
        L = self.lib
        for nm in ("eco_log_table", "eco_exp_table", "eco_log_walsh_table", "eco_skews"):
            getattr(L, nm).restype = _u16p
        L.eco_mul.restype = C.c_uint16
        L.eco_mul.argtypes = [C.c_uint16, C.c_uint16]
        L.eco_shard_len.restype = C.c_size_t

    def table(self, name: str) -> np.ndarray:
        fn = {"log": "eco_log_table", "exp": "eco_exp_table",
              "log_walsh": "eco_log_walsh_table", "skews": "eco_skews"}[name]
        cnt = 65535 if name == "skews" else 65536
        p = getattr(self.lib, fn)()
        return np.ctypeslib.as_array(p, shape=(cnt,)).copy()

    def mul(self, x: int, logc: int) -> int:
        return int(self.lib.eco_mul(x, logc))

    def afft(self, data: np.ndarray, index: int) -> np.ndarray:
        d = np.ascontiguousarray(data, np.uint16).copy()
        self.lib.eco_afft(_ptr(d, _u16p), C.c_size_t(d.size), C.c_size_t(index))
        return d

    def inverse_afft(self, data: np.ndarray, index: int) -> np.ndarray:
        d = np.ascontiguousarray(data, np.uint16).copy()
        self.lib.eco_inverse_afft(_ptr(d, _u16p), C.c_size_t(d.size), C.c_size_t(index))
        return d

    def formal_derivative(self, data: np.ndarray) -> np.ndarray:
        d = np.ascontiguousarray(data, np.uint16).copy()
        self.lib.eco_formal_derivative(_ptr(d, _u16p), C.c_size_t(d.size))
        return d

    def walsh(self, data: np.ndarray) -> np.ndarray:
        d = np.ascontiguousarray(data, np.uint16).copy()
        self.lib.eco_walsh(_ptr(d, _u16p), C.c_size_t(d.size))
        return d

    def error_poly(self, erased: np.ndarray, n: int, folded: bool = False) -> np.ndarray:
        e = np.ascontiguousarray(erased, np.uint8)
        out = np.zeros(65536, np.uint16)
        fn = self.lib.eco_error_poly_folded if folded else self.lib.eco_error_poly
        fn(_ptr(e), C.c_size_t(e.size), C.c_size_t(n), _ptr(out, _u16p))
        return out[:n] if folded else out

    def encode(self, nv: int, payload: bytes) -> list[bytes]:
        n, k = self.params(nv)
        p = np.frombuffer(bytes(payload), np.uint8)
        sl = self.shard_len(k, len(payload))
        out = np.zeros(max(nv * sl, 1), np.uint8)
        pp = _ptr(np.ascontiguousarray(p)) if p.size else None
        e = self.lib.eco_encode(C.c_size_t(nv), pp, C.c_size_t(p.size), _ptr(out),
                                C.c_size_t(out.size))
        if e:
            raise CodecError(e)
        return [out[v * sl:(v + 1) * sl].tobytes() for v in range(nv)]


class RefEC(_Lib):
    """The reference ec-cpp (oracle/_ref/libecref.so)."""

    prefix = "ecref_"

    @staticmethod
    def available() -> bool:
        return os.path.exists(REF_SO)

    def __init__(self, path: str = REF_SO):
        super().__init__(path)

    def tables(self):
        log, exp, lw = (np.zeros(65536, np.uint16) for _ in range(3))
        self.lib.ecref_tables(_ptr(log, _u16p), _ptr(exp, _u16p), _ptr(lw, _u16p))
        return log, exp, lw

    def skews(self) -> np.ndarray:
        out = np.zeros(65535, np.uint16)
        self.lib.ecref_skews(_ptr(out, _u16p))
        return out

    def encode(self, nv: int, payload: bytes) -> list[bytes]:
        n, k = self.params(nv)
        p = np.frombuffer(bytes(payload), np.uint8)
        sl = self.shard_len(k, len(payload))
        out = np.zeros(max(nv * sl, 1), np.uint8)
        slen = C.c_size_t()
        pp = _ptr(np.ascontiguousarray(p)) if p.size else None
        e = self.lib.ecref_encode(C.c_size_t(nv), pp, C.c_size_t(p.size), _ptr(out),
                                  C.c_size_t(out.size), C.byref(slen))
        if e:
            raise CodecError(e)
        return [out[v * sl:(v + 1) * sl].tobytes() for v in range(nv)]

    def time(self, nv: int, payload: bytes, present: np.ndarray):
        p = np.ascontiguousarray(np.frombuffer(bytes(payload), np.uint8))
        pr = np.ascontiguousarray(present, np.uint8)
        te, td = C.c_double(), C.c_double()
        e = self.lib.ecref_time(C.c_size_t(nv), _ptr(p), C.c_size_t(p.size), _ptr(pr),
                                C.byref(te), C.byref(td))
        if e:
            raise CodecError(e)
        return te.value, td.value

    def time_mt(self, nv: int, payload: bytes, present: np.ndarray, threads: int, seconds: float):
        """All-core rate: `threads` threads each encoding + reconstructing the
        payload until `seconds` pass.  Returns (payloads done, wall s, encode s
        summed over threads, reconstruct s summed over threads)."""
        p = np.ascontiguousarray(np.frombuffer(bytes(payload), np.uint8))
        pr = np.ascontiguousarray(present, np.uint8)
        done, wall, te, td = C.c_uint64(), C.c_double(), C.c_double(), C.c_double()
        e = self.lib.ecref_time_mt(C.c_size_t(nv), _ptr(p), C.c_size_t(p.size), _ptr(pr),
                                   C.c_int(threads), C.c_double(seconds), C.byref(done),
                                   C.byref(wall), C.byref(te), C.byref(td))
        if e:
            raise CodecError(e)
        return done.value, wall.value, te.value, td.value


class Checker:
    """What the tests compare byte outputs with: the
    reference ec-cpp itself (RefEC) for encode / reconstruct /
    reconstruct_from_systematic when oracle/_ref/libecref.so was built, the C
    restatement otherwise; every internal the reference does not export
    (error_poly, afft, walsh, tables, ...) from the restatement.  `kind` says
    which one checked the bytes: "reference" or "restatement"."""

    BYTE_OUTPUTS = ("encode", "reconstruct", "reconstruct_from_systematic", "params", "threshold",
                    "shard_len")

    def __init__(self, restatement: "Oracle", ref: "RefEC | None" = None):
        self.restatement = restatement
        self.ref = ref
        self.kind = "reference" if ref is not None else "restatement"

    @classmethod
    def default(cls) -> "Checker":
        return cls(Oracle(), RefEC() if RefEC.available() else None)

    def __getattr__(self, name):
        src = self.ref if (self.ref is not None and name in self.BYTE_OUTPUTS) else self.restatement
        return getattr(src, name)
