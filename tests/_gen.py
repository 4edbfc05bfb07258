"""Deterministic test inputs (splitmix64 over numpy uint64; independent of numpy's RNG streams).

Used by tests/golden/make_golden.py and the parity tests, so committed fixtures can always be
regenerated bit for bit.
"""
import numpy as np

_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_G = np.uint64(0x9E3779B97F4A7C15)


def _mix(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = z ^ (z >> np.uint64(30))
        z = z * _M1
        z = z ^ (z >> np.uint64(27))
        z = z * _M2
        z = z ^ (z >> np.uint64(31))
    return z


def gen_bytes(seed: int, n: int) -> np.ndarray:
    """n pseudo-random bytes for `seed` (little-endian bytes of splitmix64(seed*G + i))."""
    words = (n + 7) // 8
    with np.errstate(over="ignore"):
        idx = np.arange(words, dtype=np.uint64) + np.uint64(seed & 0xFFFFFFFFFFFFFFFF) * _G
    return _mix(idx).view(np.uint8)[:n].copy()


def cluster_reader_bytes() -> bytes:
    """tests/cluster.rs:95-102 `default_reader`: 80 blocks of 256 bytes, byte = (x % 128) + i."""
    out = bytearray()
    for i in range(80):
        out += bytes(((x % 128) + i) & 0xFF for x in range(256))
    return bytes(out)
