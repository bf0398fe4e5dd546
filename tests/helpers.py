"""Shared test helpers (inputs, digests, fixture loading)."""
import hashlib
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def digest(b) -> str:
    return hashlib.sha256(bytes(b)).hexdigest()[:16]


def survey_input(k, shard_bytes=64):
    """SURVEY.md App. B parity input: input[s][j] = (131*s + 7*j + 11) & 255."""
    s = np.arange(k, dtype=np.int64)[:, None]
    j = np.arange(shard_bytes, dtype=np.int64)[None, :]
    return ((131 * s + 7 * j + 11) & 255).astype(np.uint8)


def iota_input(k, shard_bytes=64):
    """tests.zig:66-67 / 109-110: byte i = i % 256 over k*shard_bytes."""
    return (np.arange(k * shard_bytes) % 256).astype(np.uint8).reshape(k, shard_bytes)


def splitmix_bytes(seed: int, n: int) -> np.ndarray:
    """Counter-based splitmix64 byte stream, identical on CPU and GPU tests."""
    cnt = (np.arange((n + 7) // 8, dtype=np.uint64) + np.uint64(seed)) * np.uint64(0x9E3779B97F4A7C15)
    z = cnt
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.view(np.uint8)[:n].copy()
