"""ORACLE — test infrastructure only (see cec_oracle.c header).

ctypes wrapper over ``oracle/liboracle.so``, the CPU restatement of reed-solomon-erasure 4.0.2
(galois_8) and sha2 0.9.9 used by the reference's hot path.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg import this module; the
product library under ``chunky-bits_amd/`` never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import List, Optional, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

# Error codes (identical to include/chunky_ec.h / reed_solomon_erasure::Error order).
OK = 0
TOO_FEW_SHARDS = 1
TOO_MANY_SHARDS = 2
TOO_FEW_DATA_SHARDS = 3
TOO_MANY_DATA_SHARDS = 4
TOO_FEW_PARITY_SHARDS = 5
TOO_MANY_PARITY_SHARDS = 6
INCORRECT_SHARD_SIZE = 9
TOO_FEW_SHARDS_PRESENT = 10
EMPTY_SHARD = 11


def build() -> str:
    """Compile liboracle.so with the committed Makefile (gcc)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.or_gf_mul.argtypes = [ctypes.c_uint8, ctypes.c_uint8]
        L.or_gf_mul.restype = ctypes.c_uint8
        L.or_gf_div.argtypes = [ctypes.c_uint8, ctypes.c_uint8]
        L.or_gf_div.restype = ctypes.c_uint8
        L.or_gf_exp.argtypes = [ctypes.c_uint8, ctypes.c_size_t]
        L.or_gf_exp.restype = ctypes.c_uint8
        L.or_rs_matrix.argtypes = [ctypes.c_size_t, ctypes.c_size_t, u8p]
        L.or_gf_invert.argtypes = [u8p, ctypes.c_size_t, u8p]
        L.or_rs_encode_sep.argtypes = [
            ctypes.c_size_t, ctypes.c_size_t,
            ctypes.POINTER(u8p), ctypes.POINTER(ctypes.c_size_t), ctypes.c_size_t,
            ctypes.POINTER(u8p), ctypes.POINTER(ctypes.c_size_t), ctypes.c_size_t,
        ]
        L.or_rs_reconstruct.argtypes = [
            ctypes.c_size_t, ctypes.c_size_t, ctypes.POINTER(u8p),
            ctypes.POINTER(ctypes.c_size_t), u8p, ctypes.c_size_t, ctypes.c_int,
        ]
        L.or_sha256.argtypes = [u8p, ctypes.c_size_t, u8p]
        L.or_sha256.restype = None
        L.or_sha256_shani.argtypes = [u8p, ctypes.c_size_t, u8p]
        L.or_cpu_has_shani.restype = ctypes.c_int
        L.or_part_encode.argtypes = [
            ctypes.c_size_t, ctypes.c_size_t, u8p, ctypes.c_size_t, u8p, u8p,
            ctypes.POINTER(ctypes.c_size_t),
        ]
        L.or_baseline_encode_sha.argtypes = [
            ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t,
            ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
        ]
        L.or_encode_hash_parts.argtypes = [
            ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t, u8p,
            ctypes.c_size_t, u8p, ctypes.c_void_p, ctypes.c_int,
        ]
        _lib = L
    return _lib


def _u8p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def _as_u8(b) -> np.ndarray:
    if isinstance(b, np.ndarray):
        return np.ascontiguousarray(b, dtype=np.uint8)
    return np.frombuffer(bytes(b), dtype=np.uint8).copy()


def gf_mul(a: int, b: int) -> int:
    return lib().or_gf_mul(a, b)


def gf_div(a: int, b: int) -> int:
    return lib().or_gf_div(a, b)


def gf_exp(a: int, n: int) -> int:
    return lib().or_gf_exp(a, n)


def coding_matrix(d: int, p: int) -> np.ndarray:
    """ReedSolomon::new(d, p).matrix — (d+p) x d; raises ValueError(code) on crate errors."""
    out = np.zeros(((d + p) * max(d, 1),), dtype=np.uint8)
    st = lib().or_rs_matrix(d, p, _u8p(out))
    if st:
        raise ValueError(st)
    return out.reshape(d + p, d)


def gf_invert(m: np.ndarray) -> np.ndarray:
    m = np.ascontiguousarray(m, dtype=np.uint8)
    n = m.shape[0]
    out = np.zeros((n, n), dtype=np.uint8)
    st = lib().or_gf_invert(_u8p(m), n, _u8p(out))
    if st:
        raise ValueError(st)
    return out


def encode_sep(d: int, p: int, data: Sequence, parity_lens: Optional[Sequence[int]] = None
               ) -> Tuple[int, List[np.ndarray]]:
    """ReedSolomon::encode_sep — returns (status, parity list)."""
    arrs = [_as_u8(x) for x in data]
    if parity_lens is None:
        parity_lens = [len(arrs[0]) if arrs else 0] * p
    par = [np.zeros(max(n, 1), dtype=np.uint8) for n in parity_lens]
    u8p = ctypes.POINTER(ctypes.c_uint8)
    dp = (u8p * max(len(arrs), 1))(*[_u8p(a) for a in arrs])
    dl = (ctypes.c_size_t * max(len(arrs), 1))(*[len(a) for a in arrs])
    pp = (u8p * max(len(par), 1))(*[_u8p(a) for a in par])
    pl = (ctypes.c_size_t * max(len(par), 1))(*list(parity_lens))
    st = lib().or_rs_encode_sep(d, p, dp, dl, len(arrs), pp, pl, len(par))
    return st, [a[:n] for a, n in zip(par, parity_lens)]


def reconstruct(d: int, p: int, shards: Sequence[Optional[bytes]], data_only: bool = False
                ) -> Tuple[int, List[Optional[np.ndarray]]]:
    """ReedSolomon::reconstruct / reconstruct_data on Option<Vec<u8>> shards."""
    n = len(shards)
    present = np.array([s is not None for s in shards], dtype=np.uint8)
    slen = max((len(s) for s in shards if s is not None), default=0)
    bufs, lens = [], []
    for s in shards:
        if s is None:
            bufs.append(np.zeros(max(slen, 1), dtype=np.uint8))
            lens.append(0)
        else:
            a = _as_u8(s)
            bufs.append(a if len(a) else np.zeros(1, dtype=np.uint8))
            lens.append(len(a))
    u8p = ctypes.POINTER(ctypes.c_uint8)
    sp = (u8p * max(n, 1))(*[_u8p(a) for a in bufs])
    sl = (ctypes.c_size_t * max(n, 1))(*lens)
    st = lib().or_rs_reconstruct(d, p, sp, sl, _u8p(present), n, 1 if data_only else 0)
    out: List[Optional[np.ndarray]] = []
    for i in range(n):
        if present[i]:
            out.append(bufs[i][: (lens[i] or slen)].copy())
        else:
            out.append(None)
    return st, out


def sha256(buf) -> bytes:
    a = _as_u8(buf)
    out = np.zeros(32, dtype=np.uint8)
    lib().or_sha256(_u8p(a) if len(a) else _u8p(np.zeros(1, np.uint8)), len(a), _u8p(out))
    return out.tobytes()


def sha256_shani(buf) -> Optional[bytes]:
    a = _as_u8(buf)
    out = np.zeros(32, dtype=np.uint8)
    src = _u8p(a) if len(a) else _u8p(np.zeros(1, np.uint8))
    if lib().or_sha256_shani(src, len(a), _u8p(out)) != 0:
        return None
    return out.tobytes()


def has_shani() -> bool:
    return bool(lib().or_cpu_has_shani())


def part_encode(d: int, p: int, data_buf: np.ndarray, length: int):
    """FilePart::write_with_encoder compute: returns (chunksize, parity (p,L), digests (d+p,32))."""
    L = (length + d - 1) // d
    buf = np.zeros(d * L, dtype=np.uint8)
    buf[:length] = _as_u8(data_buf)[:length]
    par = np.zeros(max(p * L, 1), dtype=np.uint8)
    dig = np.zeros((d + p) * 32, dtype=np.uint8)
    cs = ctypes.c_size_t(0)
    st = lib().or_part_encode(d, p, _u8p(buf), length, _u8p(par), _u8p(dig), ctypes.byref(cs))
    if st:
        raise ValueError(st)
    return cs.value, par[: p * L].reshape(p, L), dig.reshape(d + p, 32)


def encode_hash_parts(d: int, p: int, parts: np.ndarray, threads: int,
                      check_parity: bool = False):
    """Digests [n][d+p][32] of the full parts in `parts` ([n][c][L] uint8, C-contiguous, c >= d:
    the first d chunks of each part are its data): encode_sep then SHA-256 of every chunk, as
    part_encode does, over `threads` workers.  With check_parity (c >= d+p) also returns
    parity_ok [n] (bool): chunks d..d+p-1 of the part equal the computed parity."""
    parts = np.ascontiguousarray(parts, dtype=np.uint8)
    n, c, L = parts.shape
    assert c >= d and (not check_parity or c >= d + p)
    out = np.zeros((n, d + p, 32), dtype=np.uint8)
    match = np.zeros(n, dtype=np.uint8) if check_parity else None
    st = lib().or_encode_hash_parts(d, p, L, n, _u8p(parts), c * L, _u8p(out),
                                    None if match is None else match.ctypes.data, threads)
    if st:
        raise ValueError(st)
    return (out, match.astype(bool)) if check_parity else out


def baseline_encode_sha(d: int, p: int, L: int, total_parts: int, pool: int, threads: int,
                        shani: bool = True, do_hash: bool = True) -> float:
    """Wall seconds for total_parts (encode_sep + sha256 of d+p chunks) on `threads` workers."""
    sec = ctypes.c_double(0.0)
    st = lib().or_baseline_encode_sha(d, p, L, total_parts, pool, threads, 1 if shani else 0,
                                      1 if do_hash else 0, ctypes.byref(sec))
    if st:
        raise ValueError(st)
    return sec.value
