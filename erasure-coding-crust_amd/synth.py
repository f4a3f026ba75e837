"""Seeded synthetic inputs shared by bench.py, tests and tests/golden.

Payload bytes: splitmix64 stream (seed = payload index), little-endian bytes
of successive outputs.  Erasure sets: Fisher-Yates over splitmix64 with seed
10**6 + payload index (BASELINE.md "Seeds and fill").  Also the reference's
own fills: ``(i+1) % 255`` (test/erasure_coding/reconstruct.cpp:507-512) and
``'a' + i % 24`` (benchmark/benchmark.cpp:42-44).
"""
from __future__ import annotations

import numpy as np

_M64 = (1 << 64) - 1
_GOLDEN = 0x9E3779B97F4A7C15


def splitmix64_words(seed: int, count: int) -> np.ndarray:
    """``count`` successive splitmix64 outputs for ``seed`` (vectorised)."""
    with np.errstate(over="ignore"):
        idx = np.arange(1, count + 1, dtype=np.uint64)
        z = np.uint64(seed & _M64) + idx * np.uint64(_GOLDEN)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def payload(seed: int, length: int) -> np.ndarray:
    words = splitmix64_words(seed, (length + 7) // 8)
    return words.view(np.uint8)[:length].copy()


def pattern_mod255(length: int) -> np.ndarray:
    return ((np.arange(length, dtype=np.int64) + 1) % 255).astype(np.uint8)


def pattern_alpha24(length: int) -> np.ndarray:
    return (97 + np.arange(length, dtype=np.int64) % 24).astype(np.uint8)


def present_set(seed: int, n_validators: int, count: int) -> np.ndarray:
    """Sorted indices of ``count`` shards kept out of ``n_validators`` (Fisher-Yates)."""
    perm = np.arange(n_validators, dtype=np.int64)
    r = splitmix64_words(seed, max(n_validators, 1))
    for i in range(n_validators - 1, 0, -1):
        j = int(r[i] % np.uint64(i + 1))
        perm[i], perm[j] = perm[j], perm[i]
    return np.sort(perm[:count])


def present_mask(seed: int, n_validators: int, count: int, n: int | None = None) -> np.ndarray:
    m = np.zeros(n if n is not None else n_validators, np.uint8)
    m[present_set(seed, n_validators, count)] = 1
    return m


def present_masks(seeds, n_validators: int, count: int, n: int | None = None) -> np.ndarray:
    """Vectorised erasure patterns for large batches (bench.py): for payload b keep
    the ``count`` shards with the smallest splitmix64(seeds[b]) keys.  Seeded and
    reproducible like ``present_set``; a different (faster) selection rule."""
    seeds = list(seeds)
    keys = np.stack([splitmix64_words(s, n_validators) for s in seeds])
    order = np.argsort(keys, axis=1, kind="stable")[:, :count]
    m = np.zeros((len(seeds), n if n is not None else n_validators), np.uint8)
    np.put_along_axis(m, order, 1, axis=1)
    return m


def payloads_torch(seeds, length: int, device="cuda"):
    """splitmix64 payloads generated on the device (bit-identical to ``payload``)."""
    import torch

    words = (length + 7) // 8
    seed = torch.tensor([s & _M64 for s in seeds], dtype=torch.uint64).view(torch.int64)
    seed = seed.to(device).view(-1, 1)
    idx = torch.arange(1, words + 1, dtype=torch.int64, device=device).view(1, -1)

    def lsr(x, s):
        return (x >> s) & ((1 << (64 - s)) - 1)

    g = _GOLDEN - (1 << 64)
    z = seed + idx * g
    z = (z ^ lsr(z, 30)) * (0xBF58476D1CE4E5B9 - (1 << 64))
    z = (z ^ lsr(z, 27)) * (0x94D049BB133111EB - (1 << 64))
    z = z ^ lsr(z, 31)
    out = z.view(torch.uint8).view(len(seeds), words * 8)
    # rows of exactly `length` bytes (pstride = length), not a strided view
    return out if length == words * 8 else out[:, :length].contiguous()
