"""chunky_ec — Python host binding of the MI355X erasure-coding + chunk-hashing engine.

Thin ctypes layer over ``libchunky_ec.so`` (C-ABI declared in ``include/chunky_ec.h``), shaped
like the Rust API the reference calls on its hot path so that tests read like the reference's:

* :class:`ReedSolomon` — ``reed_solomon_erasure::ReedSolomon<galois_8::Field>``
  (``new`` / ``encode_sep`` / ``reconstruct`` / ``reconstruct_data``; call sites
  src/file/file_part.rs:77,128,161-165,302-304).
* :class:`Sha256Hash` / :class:`AnyHash` — src/file/hash/{sha256,any}.rs (``from_buf``,
  ``verify``, ``sha256-<hex>`` display).
* :class:`Error` — ``reed_solomon_erasure::Error`` variants (wrapped by
  ``FileWriteError::Erasure`` / ``FileReadError::Erasure``, src/error.rs:44,55).
* :func:`part_encode` and the ``*_batch`` functions — the part layer's compute
  (``FilePart::write_with_encoder`` / ``read_with_context`` / ``resilver`` / ``verify``,
  src/file/file_part.rs:73-390), batched over parts resident in HBM.

Host loops built on these (submodules): :mod:`chunky_ec.readstream` (FileReadBuilder's part
loop over a ReadPipeline with read_with_context's retry rule), :mod:`chunky_ec.batchwriter` /
:mod:`chunky_ec.batchreader` (the batched FileWriteBuilder / FileReadBuilder loops over the
multi-GPU scheduler: twins of the Rust crate's ``batch`` module), :mod:`chunky_ec.sharding`
(part ranges and the bench's cross-rank helpers).

All computation runs in the HIP library on the GPU; there is no CPU fallback.  If the
library is missing this module raises on import.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import List, MutableSequence, Optional, Sequence

try:  # torch ships its own libamdhip64.so.7: load it first so one HIP runtime serves both.
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the host-buffer API
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
# CEC_LIBRARY points the A/B timing tools (tools/*_ab.py) at the attribution build
# (tools/ab/libchunky_ec.so, `make -C chunky-bits_amd/csrc ab`); everything else loads the product
# library next to this file.
LIB_PATH = os.environ.get("CEC_LIBRARY") or os.path.join(_HERE, "libchunky_ec.so")

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"chunky_ec: HIP library not built ({LIB_PATH}); run `make -C chunky-bits_amd/csrc` "
        "or __graft_entry__.build()")

_lib = ctypes.CDLL(LIB_PATH)

_u8p = ctypes.POINTER(ctypes.c_uint8)
_szp = ctypes.POINTER(ctypes.c_size_t)
_vp = ctypes.c_void_p


class PartBatchStruct(ctypes.Structure):
    _fields_ = [
        ("base", ctypes.c_void_p),
        ("part_stride", ctypes.c_size_t),
        ("chunk_stride", ctypes.c_size_t),
        ("n_parts", ctypes.c_size_t),
        ("chunk_len", ctypes.c_size_t),
    ]


def _sig(name, argtypes, restype=ctypes.c_int):
    fn = getattr(_lib, name)
    fn.argtypes = argtypes
    fn.restype = restype
    return fn


_sig("cec_abi_version", [])
# the include/chunky_ec.h this binding mirrors (2: CEC_PRESENT_VERIFIED = 0x80)
ABI_VERSION = 3
if _lib.cec_abi_version() != ABI_VERSION:
    raise ImportError(f"chunky_ec: {LIB_PATH} has ABI {_lib.cec_abi_version()}, this binding "
                      f"needs {ABI_VERSION}; rebuild with `make -C chunky-bits_amd/csrc`")
if not hasattr(_lib, "cec_build_id"):
    raise ImportError(f"chunky_ec: {LIB_PATH} predates cec_build_id; rebuild with "
                      "`make -C chunky-bits_amd/csrc`")
_sig("cec_build_id", [], ctypes.c_char_p)


def _shipped_source_hash() -> Optional[str]:
    """Hash of the library sources shipped beside this package (csrc/source_hash.py), or None
    when they are not (an installed copy)."""
    csrc = os.path.join(os.path.dirname(_HERE), "csrc")
    script = os.path.join(csrc, "source_hash.py")
    if not os.path.exists(script):
        return None
    import importlib.util
    spec = importlib.util.spec_from_file_location("_cec_source_hash", script)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.source_hash()


BUILD_ID = _lib.cec_build_id().decode()
SOURCE_HASH = _shipped_source_hash()
# Build provenance: a library built from other sources than the ones shipped with it (a stale
# build, or objects carried over from another tree) is refused, so what runs on a GPU box is what
# the tree says.  CEC_ALLOW_STALE_BUILD=1 lets a developer load it anyway.
BUILD_MATCHES_SOURCE = SOURCE_HASH is None or SOURCE_HASH == BUILD_ID
if not BUILD_MATCHES_SOURCE and os.environ.get("CEC_ALLOW_STALE_BUILD") != "1":
    raise ImportError(f"chunky_ec: {LIB_PATH} was built from sources {BUILD_ID}, the shipped "
                      f"sources hash to {SOURCE_HASH}; rebuild with `make -C chunky-bits_amd/csrc`")
_sig("cec_status_name", [ctypes.c_int], ctypes.c_char_p)
_sig("cec_last_error", [], ctypes.c_char_p)
_sig("cec_device_count", [])
_sig("cec_build_info", [], ctypes.c_char_p)
_sig("cec_reload_knobs", [], None)
_sig("cec_release_cached", [ctypes.c_int], ctypes.c_size_t)
_sig("cec_codec_cached_patterns", [_vp], ctypes.c_size_t)
_sig("cec_codec_new", [ctypes.c_size_t, ctypes.c_size_t, ctypes.POINTER(_vp)])
_sig("cec_codec_free", [_vp], None)
_sig("cec_codec_data_shards", [_vp], ctypes.c_size_t)
_sig("cec_codec_parity_shards", [_vp], ctypes.c_size_t)
_sig("cec_codec_total_shards", [_vp], ctypes.c_size_t)
_sig("cec_codec_matrix", [_vp, _u8p, ctypes.c_size_t])
_sig("cec_encode_sep", [_vp, ctypes.POINTER(_u8p), _szp, ctypes.c_size_t,
                        ctypes.POINTER(_u8p), _szp, ctypes.c_size_t])
_sig("cec_reconstruct", [_vp, ctypes.POINTER(_u8p), _szp, _u8p, ctypes.c_size_t])
_sig("cec_reconstruct_data", [_vp, ctypes.POINTER(_u8p), _szp, _u8p, ctypes.c_size_t])
_sig("cec_sha256", [_u8p, ctypes.c_size_t, _u8p])
_sig("cec_sha256_many", [ctypes.POINTER(_u8p), _szp, ctypes.c_size_t, _u8p])
_sig("cec_part_encode", [_vp, _u8p, ctypes.c_size_t, _u8p, _u8p, _szp])
_sig("cec_coalesce_stats", [ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)],
     None)
_sig("cec_encode_batch", [_vp, ctypes.POINTER(PartBatchStruct), _vp])
_sig("cec_encode_hash_batch", [_vp, ctypes.POINTER(PartBatchStruct), _vp, _vp])
_sig("cec_sha256_batch", [ctypes.POINTER(PartBatchStruct), ctypes.c_size_t, ctypes.c_size_t,
                          _vp, _vp])
_sig("cec_reconstruct_batch", [_vp, ctypes.POINTER(PartBatchStruct), _u8p, ctypes.c_int, _vp])
_sig("cec_fill_synthetic", [ctypes.POINTER(PartBatchStruct), ctypes.c_size_t, ctypes.c_uint64,
                            _vp])
_sig("cec_verify_batch", [ctypes.POINTER(PartBatchStruct), ctypes.c_size_t, ctypes.c_size_t,
                          _vp, _vp, _vp, _vp])
_sig("cec_read_batch", [_vp, ctypes.POINTER(PartBatchStruct), _u8p, _vp, _u8p,
                        ctypes.POINTER(ctypes.c_int), _vp])
_sig("cec_resilver_batch", [_vp, ctypes.POINTER(PartBatchStruct), _u8p, _vp, _u8p,
                            ctypes.POINTER(ctypes.c_int), _vp])
_sig("cec_pipeline_new", [_vp, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t,
                          ctypes.POINTER(_vp)])
_sig("cec_pipeline_free", [_vp], None)
_sig("cec_pipeline_depth", [_vp], ctypes.c_size_t)
_sig("cec_pipeline_acquire", [_vp, _szp, ctypes.POINTER(_u8p)])
_sig("cec_pipeline_submit", [_vp, ctypes.c_size_t, ctypes.c_size_t])
_sig("cec_pipeline_wait", [_vp, ctypes.c_size_t, ctypes.POINTER(_u8p), ctypes.POINTER(_u8p),
                           _szp])
_sig("cec_pipeline_drain", [_vp])
_sig("cec_pipeline_query", [_vp, ctypes.c_size_t])
_sig("cec_read_pipeline_query", [_vp, ctypes.c_size_t])
_sig("cec_pipeline_last_error", [], ctypes.c_char_p)
_sig("cec_read_pipeline_new", [_vp, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t,
                               ctypes.POINTER(_vp)])
_sig("cec_read_pipeline_free", [_vp], None)
_sig("cec_read_pipeline_depth", [_vp], ctypes.c_size_t)
_sig("cec_read_pipeline_acquire", [_vp, _szp, ctypes.POINTER(_u8p), ctypes.POINTER(_u8p),
                                   ctypes.POINTER(_u8p)])
_sig("cec_read_pipeline_submit", [_vp, ctypes.c_size_t, ctypes.c_size_t])
_sig("cec_read_pipeline_acquire_idle", [_vp, _szp, ctypes.POINTER(_u8p), ctypes.POINTER(_u8p),
                                        ctypes.POINTER(_u8p)])
_sig("cec_read_pipeline_wait", [_vp, ctypes.c_size_t, ctypes.POINTER(_u8p), ctypes.POINTER(_u8p),
                                ctypes.POINTER(ctypes.POINTER(ctypes.c_int)), _szp])
_sig("cec_read_pipeline_drain", [_vp])
_sig("cec_read_pipeline_new_ex", [_vp, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t,
                                  ctypes.c_uint, ctypes.POINTER(_vp)])
_sig("cec_read_pipeline_data_chunks", [_vp, ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p),
                                       ctypes.c_size_t])
_sig("cec_synth_byte", [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64],
     ctypes.c_uint8)
_sig("cec_current_device", [ctypes.POINTER(ctypes.c_int)])
_sig("cec_set_device", [ctypes.c_int])
_sig("cec_device_numa_node", [ctypes.c_int])
_sig("cec_host_alloc", [ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(_vp)])
_sig("cec_host_free", [_vp], None)
_sig("cec_host_is_pinned", [_vp, ctypes.c_size_t])
_sig("cec_host_numa_node", [_vp])
_sig("cec_bind_thread_to_device_node", [ctypes.c_int])
_sig("cec_pipeline_new_ex", [_vp, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_uint,
                             ctypes.POINTER(_vp)])
_sig("cec_pipeline_submit_from", [_vp, ctypes.c_size_t, _vp, ctypes.c_size_t, _vp, _vp])
_sig("cec_read_pipeline_submit_from", [_vp, ctypes.c_size_t, _vp, _vp, _vp, ctypes.c_size_t, _vp])
_sig("cec_read_pipeline_submit_packed", [_vp, ctypes.c_size_t, _vp, _vp, _vp, ctypes.c_size_t, _vp])
_sig("cec_read_pipeline_carry_ids", [_vp, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int32),
                                     ctypes.c_size_t])
_sig("cec_read_pipeline_submit_carried", [_vp, ctypes.c_size_t, ctypes.c_size_t,
                                          ctypes.POINTER(ctypes.c_int32)])
_sig("cec_read_pipeline_carry_release", [_vp, ctypes.c_int32])
_sig("cec_read_pipeline_carry_held", [_vp], ctypes.c_size_t)


class ReadSubmitStruct(ctypes.Structure):
    """cec_read_submit (include/chunky_ec.h)."""
    _fields_ = [("chunks", ctypes.c_void_p), ("present", ctypes.c_void_p),
                ("expected", ctypes.c_void_p), ("n_parts", ctypes.c_size_t),
                ("data_out", ctypes.c_void_p), ("carry_ids", ctypes.c_void_p),
                ("flags", ctypes.c_uint)]


class MultiStatsStruct(ctypes.Structure):
    """cec_multi_stats (include/chunky_ec.h)."""
    _fields_ = [("device", ctypes.c_int), ("numa_node", ctypes.c_int),
                ("parts", ctypes.c_uint64), ("pipelines_made", ctypes.c_uint64),
                ("chunks_uploaded", ctypes.c_uint64), ("chunks_carried", ctypes.c_uint64),
                ("carry_held", ctypes.c_uint64)]


_sig("cec_read_pipeline_submit_ex", [_vp, ctypes.c_size_t, ctypes.POINTER(ReadSubmitStruct)])
_sig("cec_pipelines_made", [], ctypes.c_uint64)
_sig("cec_multi_new_ex", [_vp, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t,
                          ctypes.POINTER(ctypes.c_int), ctypes.c_size_t, ctypes.c_uint,
                          ctypes.POINTER(_vp)])
_sig("cec_multi_read_carry", [_vp, _vp, _vp, _vp, ctypes.c_size_t, _vp, _vp,
                              ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_void_p),
                              ctypes.c_uint, ctypes.POINTER(ctypes.c_int32),
                              ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_uint64)])
_sig("cec_multi_carry_release", [_vp, ctypes.c_int32])
_sig("cec_multi_shard_stats", [_vp, ctypes.c_size_t, ctypes.POINTER(MultiStatsStruct)])
_sig("cec_multi_new", [_vp, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t,
                       ctypes.POINTER(ctypes.c_int), ctypes.c_size_t, ctypes.POINTER(_vp)])
_sig("cec_multi_free", [_vp], None)
_sig("cec_multi_shards", [_vp], ctypes.c_size_t)
_sig("cec_multi_shard_info", [_vp, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int),
                              ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_uint64)])
_sig("cec_multi_encode_hash", [_vp, _vp, ctypes.c_size_t, _vp, _vp,
                               ctypes.POINTER(ctypes.c_uint64)])
_sig("cec_multi_read", [_vp, _vp, _vp, _vp, ctypes.c_size_t, _vp, _vp,
                        ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint,
                        ctypes.POINTER(ctypes.c_uint64)])
_sig("cec_multi_resilver", [_vp, _vp, _vp, _vp, ctypes.c_size_t, _vp, _vp,
                            ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_void_p),
                            ctypes.POINTER(ctypes.c_uint64)])
_sig("cec_multi_verify", [_vp, _vp, _vp, _vp, ctypes.c_size_t, _vp,
                          ctypes.POINTER(ctypes.c_uint64)])
_sig("cec_multi_wait", [_vp, ctypes.c_uint64])
_sig("cec_multi_query", [_vp, ctypes.c_uint64])
_sig("cec_multi_last_error", [], ctypes.c_char_p)

# Status codes (include/chunky_ec.h).
OK = 0
TOO_FEW_SHARDS = 1
TOO_MANY_SHARDS = 2
TOO_FEW_DATA_SHARDS = 3
TOO_MANY_DATA_SHARDS = 4
TOO_FEW_PARITY_SHARDS = 5
TOO_MANY_PARITY_SHARDS = 6
TOO_FEW_BUFFER_SHARDS = 7
TOO_MANY_BUFFER_SHARDS = 8
INCORRECT_SHARD_SIZE = 9
TOO_FEW_SHARDS_PRESENT = 10
EMPTY_SHARD = 11
INVALID_SHARD_FLAGS = 12
INVALID_INDEX = 13
ERR_INVALID_ARGUMENT = 101
ERR_HIP = 102
ERR_NO_DEVICE = 103
ERR_OUT_OF_MEMORY = 104


class Error(Exception):
    """reed_solomon_erasure::Error (codes 1..13) or an engine error (>= 100)."""

    def __init__(self, code: int):
        self.code = code
        self.name = _lib.cec_status_name(code).decode()
        detail = _lib.cec_last_error().decode() if code >= 100 else ""
        super().__init__(f"{self.name}" + (f": {detail}" if detail else ""))


def _check(code: int) -> None:
    if code != OK:
        raise Error(code)


def abi_version() -> int:
    return _lib.cec_abi_version()


def device_count() -> int:
    return _lib.cec_device_count()


def build_info() -> str:
    return _lib.cec_build_info().decode()


def reload_knobs() -> None:
    """Re-read the CEC_* environment knobs (test-only: the library reads them once per
    process, cec_reload_knobs)."""
    _lib.cec_reload_knobs()


def release_cached(device: int = -1) -> int:
    """Free the idle per-call staging on `device` (every device when < 0); returns the device
    bytes released (cec_release_cached)."""
    return _lib.cec_release_cached(device)


def status_name(code: int) -> str:
    return _lib.cec_status_name(code).decode()


def _buf_ptr(b, keep: list) -> "ctypes._Pointer":
    """Pointer to the first byte of a bytes-like object (valid while `b` / `keep` live)."""
    if isinstance(b, bytes):
        return ctypes.cast(ctypes.c_char_p(b), _u8p)
    mv = memoryview(b)
    if mv.nbytes == 0:
        return _u8p()
    if mv.readonly or not mv.c_contiguous:
        tmp = mv.tobytes()
        keep.append(tmp)
        return ctypes.cast(ctypes.c_char_p(tmp), _u8p)
    return ctypes.cast((ctypes.c_char * mv.nbytes).from_buffer(mv.cast("B")), _u8p)


def _nbytes(b) -> int:
    return memoryview(b).nbytes


class ReedSolomon:
    """reed_solomon_erasure::ReedSolomon<galois_8::Field> backed by the gfx950 kernels."""

    def __init__(self, data_shards: int, parity_shards: int):
        h = _vp()
        _check(_lib.cec_codec_new(data_shards, parity_shards, ctypes.byref(h)))
        self._h = h

    def __del__(self, _free=_lib.cec_codec_free):
        h = getattr(self, "_h", None)
        if h:
            _free(h)
            self._h = None

    @property
    def handle(self):
        return self._h

    def data_shard_count(self) -> int:
        return _lib.cec_codec_data_shards(self._h)

    def parity_shard_count(self) -> int:
        return _lib.cec_codec_parity_shards(self._h)

    def total_shard_count(self) -> int:
        return _lib.cec_codec_total_shards(self._h)

    def cached_patterns(self) -> int:
        """Decode matrices cached in the codec (bounded LRU)."""
        return _lib.cec_codec_cached_patterns(self._h)

    def matrix(self) -> List[List[int]]:
        d, t = self.data_shard_count(), self.total_shard_count()
        out = (ctypes.c_uint8 * (d * t))()
        _check(_lib.cec_codec_matrix(self._h, out, d * t))
        return [list(out[r * d:(r + 1) * d]) for r in range(t)]

    def encode_sep(self, data: Sequence, parity: MutableSequence) -> None:
        """Overwrites each writable parity buffer with the parity of `data` (crate semantics)."""
        keep: list = []
        dp = (_u8p * max(len(data), 1))(*[_buf_ptr(x, keep) for x in data])
        dl = (ctypes.c_size_t * max(len(data), 1))(*[_nbytes(x) for x in data])
        pp = (_u8p * max(len(parity), 1))(*[_buf_ptr(x, keep) for x in parity])
        pl = (ctypes.c_size_t * max(len(parity), 1))(*[_nbytes(x) for x in parity])
        _check(_lib.cec_encode_sep(self._h, dp, dl, len(data), pp, pl, len(parity)))

    def _reconstruct(self, shards: MutableSequence[Optional[bytearray]], data_only: bool):
        n = len(shards)
        present = (ctypes.c_uint8 * max(n, 1))(*[0 if s is None else 1 for s in shards])
        slen = next((_nbytes(s) for s in shards if s is not None and _nbytes(s) > 0), 0)
        bufs = []
        for s in shards:
            bufs.append(bytearray(slen) if s is None else s)
        keep: list = []
        ptrs = (_u8p * max(n, 1))(*[_buf_ptr(b, keep) for b in bufs])
        lens = (ctypes.c_size_t * max(n, 1))(*[_nbytes(b) for b in bufs])
        code = (_lib.cec_reconstruct_data if data_only else _lib.cec_reconstruct)(
            self._h, ptrs, lens, present, n)
        _check(code)
        for i in range(n):
            if shards[i] is None and present[i]:
                shards[i] = bufs[i]

    def reconstruct(self, shards: MutableSequence[Optional[bytearray]]) -> None:
        """Fills every None slot (data and parity), like ReedSolomon::reconstruct."""
        self._reconstruct(shards, False)

    def reconstruct_data(self, shards: MutableSequence[Optional[bytearray]]) -> None:
        """Fills missing data slots only, like ReedSolomon::reconstruct_data."""
        self._reconstruct(shards, True)


class Sha256Hash:
    """src/file/hash/sha256.rs: Sha256Hash([u8; 32]) with hex display."""

    __slots__ = ("digest",)

    def __init__(self, digest: bytes):
        assert len(digest) == 32
        self.digest = bytes(digest)

    @classmethod
    def from_buf(cls, buf) -> "Sha256Hash":
        out = (ctypes.c_uint8 * 32)()
        keep: list = []
        _check(_lib.cec_sha256(_buf_ptr(buf, keep), _nbytes(buf), out))
        return cls(bytes(out))

    @classmethod
    def from_bufs(cls, bufs: Sequence) -> List["Sha256Hash"]:
        """Batched DataHasher::from_buf over many buffers (one launch)."""
        n = len(bufs)
        if n == 0:
            return []
        out = (ctypes.c_uint8 * (32 * n))()
        keep: list = []
        ptrs = (_u8p * n)(*[_buf_ptr(b, keep) for b in bufs])
        lens = (ctypes.c_size_t * n)(*[_nbytes(b) for b in bufs])
        _check(_lib.cec_sha256_many(ptrs, lens, n, out))
        raw = bytes(out)
        return [cls(raw[32 * i:32 * (i + 1)]) for i in range(n)]

    @classmethod
    def from_str(cls, s: str) -> "Sha256Hash":
        return cls(bytes.fromhex(s))

    def verify(self, buf) -> bool:
        return Sha256Hash.from_buf(buf) == self

    def __eq__(self, other) -> bool:
        return isinstance(other, Sha256Hash) and other.digest == self.digest

    def __hash__(self) -> int:
        return hash(self.digest)

    def __str__(self) -> str:
        return self.digest.hex()

    __repr__ = __str__


class AnyHash:
    """src/file/hash/any.rs: AnyHash::Sha256, displayed as ``sha256-<hex>``."""

    def __init__(self, h: Sha256Hash):
        self.sha256 = h

    def __str__(self) -> str:
        return f"sha256-{self.sha256}"

    @classmethod
    def from_str(cls, s: str) -> "AnyHash":
        kind, _, hexs = s.partition("-")
        if not _:
            raise ValueError("Invalid hash format")
        if kind != "sha256":
            raise ValueError(f"Unknown Hash Format: {kind}")
        return cls(Sha256Hash.from_str(hexs))

    def verify(self, buf) -> bool:
        return self.sha256.verify(buf)

    def __eq__(self, other) -> bool:
        return isinstance(other, AnyHash) and other.sha256 == self.sha256


@dataclass
class EncodedPart:
    """Compute result of FilePart::write_with_encoder: chunksize, parity chunks, digests."""

    chunksize: int
    parity: List[bytes]
    hashes: List[Sha256Hash]  # d data then p parity, in order


def part_encode(codec: ReedSolomon, data_buf, length: int) -> EncodedPart:
    """FilePart::write_with_encoder's compute (file_part.rs:150-185) for one part."""
    d, p = codec.data_shard_count(), codec.parity_shard_count()
    if length > _nbytes(data_buf):  # file_part.rs:150 asserts length <= data_buf.len()
        raise ValueError(f"length {length} > data_buf length {_nbytes(data_buf)}")
    L = (length + d - 1) // d if length else 0
    buf = bytearray(d * L)
    src = memoryview(data_buf)[:length]
    buf[:length] = src
    par = (ctypes.c_uint8 * max(p * L, 1))()
    dig = (ctypes.c_uint8 * (32 * (d + p)))()
    cs = ctypes.c_size_t(0)
    keep: list = []
    _check(_lib.cec_part_encode(codec.handle, _buf_ptr(buf, keep) if L else _u8p(), length, par,
                                dig, ctypes.byref(cs)))
    raw = bytes(par)
    draw = bytes(dig)
    return EncodedPart(
        chunksize=cs.value,
        parity=[raw[i * L:(i + 1) * L] for i in range(p)],
        hashes=[Sha256Hash(draw[32 * i:32 * (i + 1)]) for i in range(d + p)],
    )


# ---------------------------------------------------------------------------------------------
# Device-resident batches
# ---------------------------------------------------------------------------------------------


@dataclass
class PartBatch:
    """Part k's chunk i at base + k*part_stride + i*chunk_stride, chunk_len bytes (device)."""

    base: int
    part_stride: int
    chunk_stride: int
    n_parts: int
    chunk_len: int

    def struct(self) -> PartBatchStruct:
        return PartBatchStruct(self.base, self.part_stride, self.chunk_stride, self.n_parts,
                               self.chunk_len)

    @classmethod
    def from_tensor(cls, t, chunk_len: Optional[int] = None) -> "PartBatch":
        """t: contiguous uint8 device tensor shaped (n_parts, n_chunks, chunk_stride)."""
        assert t.dtype == torch.uint8 and t.dim() == 3 and t.is_contiguous()
        n_parts, n_chunks, cstride = t.shape
        return cls(t.data_ptr(), n_chunks * cstride, cstride, n_parts,
                   cstride if chunk_len is None else chunk_len)


def _stream_ptr(stream) -> int:
    if stream is None:
        if torch is not None and torch.cuda.is_available():
            return torch.cuda.current_stream().cuda_stream
        return 0
    if hasattr(stream, "cuda_stream"):
        return stream.cuda_stream
    return int(stream)


def encode_batch(codec: ReedSolomon, batch: PartBatch, stream=None) -> None:
    s = batch.struct()
    _check(_lib.cec_encode_batch(codec.handle, ctypes.byref(s), _stream_ptr(stream)))


def encode_hash_batch(codec: ReedSolomon, batch: PartBatch, digests_ptr: int,
                      stream=None) -> None:
    s = batch.struct()
    _check(_lib.cec_encode_hash_batch(codec.handle, ctypes.byref(s), digests_ptr,
                                      _stream_ptr(stream)))


def sha256_batch(batch: PartBatch, first_chunk: int, n_chunks: int, digests_ptr: int,
                 stream=None) -> None:
    s = batch.struct()
    _check(_lib.cec_sha256_batch(ctypes.byref(s), first_chunk, n_chunks, digests_ptr,
                                 _stream_ptr(stream)))


def reconstruct_batch(codec: ReedSolomon, batch: PartBatch, present, data_only: bool,
                      stream=None) -> None:
    """present: host bytes-like of n_parts*(d+p) flags (part-major)."""
    s = batch.struct()
    pres = bytes(present)
    _check(_lib.cec_reconstruct_batch(codec.handle, ctypes.byref(s),
                                      ctypes.cast(ctypes.c_char_p(pres), _u8p),
                                      1 if data_only else 0, _stream_ptr(stream)))


def verify_batch(batch: PartBatch, first_chunk: int, n_chunks: int, expected_ptr: int,
                 ok_ptr: int, present_ptr: int = 0, stream=None) -> None:
    """DataVerifier::verify over a batch (device pointers; present_ptr 0 = all present)."""
    s = batch.struct()
    _check(_lib.cec_verify_batch(ctypes.byref(s), first_chunk, n_chunks, present_ptr or None,
                                 expected_ptr, ok_ptr, _stream_ptr(stream)))


def _verify_rebuild(fn, codec, batch, present, expected_ptr, stream):
    t = codec.total_shard_count()
    n = batch.n_parts * t
    pres = bytes(present)
    assert len(pres) == n
    verified = (ctypes.c_uint8 * max(n, 1))()
    status = (ctypes.c_int * max(batch.n_parts, 1))()
    s = batch.struct()
    _check(fn(codec.handle, ctypes.byref(s), ctypes.cast(ctypes.c_char_p(pres), _u8p),
              expected_ptr, verified, status, _stream_ptr(stream)))
    return bytes(verified)[:n], list(status)[:batch.n_parts]


def read_batch(codec: ReedSolomon, batch: PartBatch, present, expected_ptr: int, stream=None):
    """FilePart::read_with_context compute: verify loaded chunks, reconstruct_data.
    Returns (verified flags, per-part status)."""
    return _verify_rebuild(_lib.cec_read_batch, codec, batch, present, expected_ptr, stream)


def resilver_batch(codec: ReedSolomon, batch: PartBatch, present, expected_ptr: int,
                   stream=None):
    """FilePart::resilver compute: verify all chunks, rebuild missing data and parity."""
    return _verify_rebuild(_lib.cec_resilver_batch, codec, batch, present, expected_ptr, stream)


def fill_synthetic(batch: PartBatch, n_chunks: int, seed: int, stream=None) -> None:
    s = batch.struct()
    _check(_lib.cec_fill_synthetic(ctypes.byref(s), n_chunks, seed, _stream_ptr(stream)))


def coalesce_stats():
    """(calls, launches) made through the per-call coalescing path (cec_coalesce_stats)."""
    calls, launches = ctypes.c_uint64(0), ctypes.c_uint64(0)
    _lib.cec_coalesce_stats(ctypes.byref(calls), ctypes.byref(launches))
    return calls.value, launches.value


def synth_byte(seed: int, part: int, chunk: int, offset: int) -> int:
    return _lib.cec_synth_byte(seed, part, chunk, offset)


# ---------------------------------------------------------------------------------------------
# Host-staged write pipeline (FileWriteBuilder::write's part loop, batched)
# ---------------------------------------------------------------------------------------------


class Pipeline:
    """cec_pipeline: pinned host slots -> H2D -> fused encode+hash -> D2H, `depth` in flight.

    Usage per batch: ``slot, data = pl.acquire()`` (a writable numpy view of the pinned
    [parts][d][L] buffer), fill it, ``pl.submit(slot, n_parts)``, later
    ``parity, digests = pl.wait(slot)`` (numpy views valid until the slot is re-acquired).
    """

    def __init__(self, codec: ReedSolomon, chunk_len: int, parts_per_batch: int, depth: int = 4,
                 flags: int = 0):
        h = _vp()
        code = _lib.cec_pipeline_new_ex(codec.handle, chunk_len, parts_per_batch, depth, flags,
                                        ctypes.byref(h))
        if code != OK:
            raise Error(code)
        self._h = h
        self.codec = codec  # keep the codec alive
        self.d, self.p = codec.data_shard_count(), codec.parity_shard_count()
        self.L = chunk_len
        self.parts = parts_per_batch
        self.depth = depth

    def __del__(self, _free=_lib.cec_pipeline_free):
        h = getattr(self, "_h", None)
        if h:
            _free(h)
            self._h = None

    def acquire(self):
        import numpy as np
        slot = ctypes.c_size_t(0)
        ptr = _u8p()
        _check(_lib.cec_pipeline_acquire(self._h, ctypes.byref(slot), ctypes.byref(ptr)))
        if not ptr:  # PIPE_EXTERNAL: no slot buffer, batches come through submit_from
            return slot.value, None
        n = self.parts * self.d * self.L
        arr = np.ctypeslib.as_array(ptr, shape=(n,)).reshape(self.parts, self.d, self.L)
        return slot.value, arr

    def submit(self, slot: int, n_parts: int) -> None:
        _check(_lib.cec_pipeline_submit(self._h, slot, n_parts))

    def submit_from(self, slot: int, data, n_parts: int, parity=None, digests=None) -> None:
        """Batch from the caller's buffers (page-locked ones are DMA'd directly)."""
        _check(_lib.cec_pipeline_submit_from(self._h, slot, _addr(data), n_parts,
                                             _addr(parity) if parity is not None else None,
                                             _addr(digests) if digests is not None else None))

    def wait(self, slot: int):
        import numpy as np
        par, dig = _u8p(), _u8p()
        n = ctypes.c_size_t(0)
        _check(_lib.cec_pipeline_wait(self._h, slot, ctypes.byref(par), ctypes.byref(dig),
                                      ctypes.byref(n)))
        k = n.value
        parity = np.ctypeslib.as_array(par, shape=(max(k * self.p * self.L, 1),))[
            : k * self.p * self.L].reshape(k, self.p, self.L)
        digests = np.ctypeslib.as_array(dig, shape=(max(k * (self.d + self.p) * 32, 1),))[
            : k * (self.d + self.p) * 32].reshape(k, self.d + self.p, 32)
        return parity, digests

    def query(self, slot: int) -> bool:
        """True when the slot's batch is complete (never blocks)."""
        r = _lib.cec_pipeline_query(self._h, slot)
        if r < 0 or r > 1:
            raise Error(r)
        return bool(r)

    def drain(self) -> None:
        _check(_lib.cec_pipeline_drain(self._h))


class ReadPipeline:
    """cec_read_pipeline: FileReadBuilder's part loop batched over pinned slots.

    ``slot, chunks, present, expected = rp.acquire()`` gives writable numpy views of the pinned
    [parts][d+p][L] chunk buffer, [parts][d+p] loaded flags and [parts][d+p][32] metadata
    digests; fill them, ``rp.submit(slot, n_parts)``; later
    ``data, verified, status = rp.wait(slot)`` -> [parts][d][L] part bytes (read_with_context's
    output), [parts][d+p] verification flags, [parts] status codes (views valid until the slot
    is re-acquired).
    """

    REBUILT_ONLY = 1  # CEC_READ_REBUILT_ONLY
    CARRY = 16  # CEC_READ_CARRY: retries' verified chunks kept on the device
    SUBMIT_PACKED = 32  # CEC_SUBMIT_PACKED (submit_ex)

    def __init__(self, codec: ReedSolomon, chunk_len: int, parts_per_batch: int, depth: int = 4,
                 flags: int = 0):
        h = _vp()
        code = _lib.cec_read_pipeline_new_ex(codec.handle, chunk_len, parts_per_batch, depth,
                                             flags, ctypes.byref(h))
        if code != OK:
            raise Error(code)
        self._h = h
        self.codec = codec
        self.d, self.p = codec.data_shard_count(), codec.parity_shard_count()
        self.t = self.d + self.p
        self.L = chunk_len
        self.parts = parts_per_batch
        self.depth = depth
        self.carry = bool(flags & self.CARRY)

    def __del__(self, _free=_lib.cec_read_pipeline_free):
        h = getattr(self, "_h", None)
        if h:
            _free(h)
            self._h = None

    def acquire(self):
        import numpy as np
        slot = ctypes.c_size_t(0)
        ch, pr, ex = _u8p(), _u8p(), _u8p()
        _check(_lib.cec_read_pipeline_acquire(self._h, ctypes.byref(slot), ctypes.byref(ch),
                                              ctypes.byref(pr), ctypes.byref(ex)))
        P, t, L = self.parts, self.t, self.L
        chunks = (np.ctypeslib.as_array(ch, shape=(P * t * L,)).reshape(P, t, L) if ch
                  else None)  # PIPE_EXTERNAL: chunks come through submit_from
        present = np.ctypeslib.as_array(pr, shape=(P * t,)).reshape(P, t)
        expected = np.ctypeslib.as_array(ex, shape=(P * t * 32,)).reshape(P, t, 32)
        return slot.value, chunks, present, expected

    def submit(self, slot: int, n_parts: int) -> None:
        _check(_lib.cec_read_pipeline_submit(self._h, slot, n_parts))

    def carry_ids(self, slot: int, n_parts: int):
        """[n_parts] int32: each part's carry entry after wait (-1: none; CARRY pipelines); the
        caller now holds the entries (submit them with a retry, or carry_release them)."""
        import numpy as np
        ids = np.full(self.parts, -1, np.int32)  # room for the largest batch a slot can hold
        _check(_lib.cec_read_pipeline_carry_ids(
            self._h, slot, ids.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), len(ids)))
        return ids[:n_parts]

    def carry_held(self) -> int:
        """Carry entries the caller holds (taken with carry_ids, not yet used or released)."""
        return _lib.cec_read_pipeline_carry_held(self._h)

    def submit_ex(self, slot: int, n_parts: int, chunks=None, present=None, expected=None,
                  data=None, carry_ids=None, mode: int = 0, packed: bool = False) -> None:
        """cec_read_pipeline_submit_ex: any mode (0 read, REBUILT_ONLY, READ_RESILVER,
        READ_VERIFY_ONLY) on this pipeline, the caller's or the slot's buffers (None), carry ids
        (CARRY pipelines) and a packed upload."""
        import numpy as np
        ids = None
        if carry_ids is not None:
            ids = np.ascontiguousarray(carry_ids, dtype=np.int32)
            assert len(ids) >= n_parts
        a = ReadSubmitStruct(
            _addr(chunks) if chunks is not None else None,
            _addr(present) if present is not None else None,
            _addr(expected) if expected is not None else None, n_parts,
            _addr(data) if data is not None else None,
            ids.ctypes.data if ids is not None else None,
            mode | (self.SUBMIT_PACKED if packed else 0))
        code = _lib.cec_read_pipeline_submit_ex(self._h, slot, ctypes.byref(a))
        if code != OK:
            raise Error(code)

    def submit_carried(self, slot: int, n_parts: int, carry_ids) -> None:
        """submit, with carry_ids[n_parts] (-1 = none): those parts' CEC_PRESENT_VERIFIED chunks
        come from the carry pool (the slot need not hold them)."""
        import numpy as np
        ids = np.ascontiguousarray(carry_ids, dtype=np.int32)
        assert len(ids) >= n_parts
        code = _lib.cec_read_pipeline_submit_carried(
            self._h, slot, n_parts, ids.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
        if code != OK:
            raise Error(code)

    def carry_release(self, carry_id: int) -> None:
        _check(_lib.cec_read_pipeline_carry_release(self._h, int(carry_id)))

    def submit_from(self, slot: int, chunks, present, expected, n_parts: int, data=None) -> None:
        """Batch from the caller's buffers (page-locked ones are DMA'd directly)."""
        _check(_lib.cec_read_pipeline_submit_from(
            self._h, slot, _addr(chunks), _addr(present), _addr(expected), n_parts,
            _addr(data) if data is not None else None))

    def submit_packed(self, slot: int, chunks, present, expected, n_parts: int,
                      data=None) -> None:
        """Batch whose loaded chunks are packed back to back in (part, chunk index) order
        (cec_read_pipeline_submit_packed): one upload per batch."""
        _check(_lib.cec_read_pipeline_submit_packed(
            self._h, slot, _addr(chunks), _addr(present), _addr(expected), n_parts,
            _addr(data) if data is not None else None))

    def wait(self, slot: int):
        import numpy as np
        data, ok = _u8p(), _u8p()
        status = ctypes.POINTER(ctypes.c_int)()
        n = ctypes.c_size_t(0)
        _check(_lib.cec_read_pipeline_wait(self._h, slot, ctypes.byref(data), ctypes.byref(ok),
                                           ctypes.byref(status), ctypes.byref(n)))
        k, t, d, L = n.value, self.t, self.d, self.L
        out = None  # a verify batch of a pipeline without its own output has none
        if data:
            out = np.ctypeslib.as_array(data, shape=(max(k * d * L, 1),))[: k * d * L].reshape(k, d, L)
        ver = np.ctypeslib.as_array(ok, shape=(max(k * t, 1),))[: k * t].reshape(k, t)
        st = np.ctypeslib.as_array(status, shape=(max(k, 1),))[:k]
        return out, ver, st

    def data_chunks(self, slot: int, n_parts: int, out_chunks: Optional[int] = None):
        """[n_parts][out] addresses of the output chunks (cec_read_pipeline_data_chunks; out = d,
        or d+p after a resilver batch)."""
        import numpy as np
        w = out_chunks or self.d
        ptrs = (ctypes.c_void_p * (self.parts * self.t))()  # room for any batch of the slot
        _check(_lib.cec_read_pipeline_data_chunks(self._h, slot, ptrs, len(ptrs)))
        return np.array([p or 0 for p in ptrs[: n_parts * w]],
                        dtype=np.uint64).reshape(n_parts, w)

    def part_bytes(self, slot: int, n_parts: int, k: int) -> bytes:
        """Part k's d data chunks concatenated (read_with_context's output), via data_chunks."""
        return b"".join(ctypes.string_at(int(a), self.L) for a in self.data_chunks(slot, n_parts)[k])

    def query(self, slot: int) -> bool:
        """True when the slot's batch is complete (never blocks)."""
        r = _lib.cec_read_pipeline_query(self._h, slot)
        if r < 0 or r > 1:
            raise Error(r)
        return bool(r)

    def drain(self) -> None:
        _check(_lib.cec_read_pipeline_drain(self._h))


# ---------------------------------------------------------------------------------------------
# Page-locked host memory (cec_host_alloc): buffers the engine DMAs directly
# ---------------------------------------------------------------------------------------------


def _addr(buf) -> int:
    """Address of a host buffer: a HostBuffer, a numpy array, or any writable bytes-like."""
    if isinstance(buf, HostBuffer):
        return buf.ptr
    if hasattr(buf, "__array_interface__"):
        return buf.__array_interface__["data"][0]
    mv = memoryview(buf)
    return ctypes.addressof((ctypes.c_char * mv.nbytes).from_buffer(mv.cast("B")))


class HostBuffer:
    """Page-locked, portable host memory from cec_host_alloc (pages on `device`'s NUMA node).
    ``.array`` is a writable numpy uint8 view.  Every view holds a reference to the HostBuffer
    (through its base buffer), so the memory is freed only once the object AND all views of it
    are gone: ``HostBuffer(n).view(a, b)`` is safe to keep."""

    def __init__(self, nbytes: int, device: int = -1):
        h = _vp()
        _check(_lib.cec_host_alloc(nbytes, device, ctypes.byref(h)))
        self.ptr = h.value
        self.nbytes = nbytes

    @property
    def array(self):
        import numpy as np
        if not self.ptr:
            raise ValueError("HostBuffer already freed")
        raw = (ctypes.c_uint8 * self.nbytes).from_address(self.ptr)
        raw._owner = self  # the numpy view's base is `raw`: it keeps this buffer alive
        return np.frombuffer(raw, dtype=np.uint8)

    def view(self, *shape):
        return self.array.reshape(*shape)

    def __del__(self, _free=_lib.cec_host_free):
        p = getattr(self, "ptr", None)
        if p:
            _free(p)
            self.ptr = None


def host_is_pinned(buf, nbytes: Optional[int] = None) -> bool:
    n = nbytes if nbytes is not None else (buf.nbytes if hasattr(buf, "nbytes") else _nbytes(buf))
    return bool(_lib.cec_host_is_pinned(_addr(buf), n))


def host_numa_node(buf) -> int:
    return _lib.cec_host_numa_node(_addr(buf))


def device_numa_node(device: int) -> int:
    return _lib.cec_device_numa_node(device)


def bind_thread_to_device_node(device: int) -> bool:
    """Restrict the calling thread to the CPUs of the device's NUMA node (False if impossible)."""
    return bool(_lib.cec_bind_thread_to_device_node(device))


def current_device() -> int:
    d = ctypes.c_int(0)
    _check(_lib.cec_current_device(ctypes.byref(d)))
    return d.value


def set_device(device: int) -> None:
    _check(_lib.cec_set_device(device))


# ---------------------------------------------------------------------------------------------
# Multi-GPU part scheduler (cec_multi_*): one process, contiguous part ranges per shard
# ---------------------------------------------------------------------------------------------

PIPE_EXTERNAL = 2  # CEC_PIPE_EXTERNAL
PRESENT_VERIFIED = 0x80  # CEC_PRESENT_VERIFIED: read-retry flag (loaded, verified by an earlier pass)
MULTI_AHEAD = 64  # CEC_MULTI_AHEAD: a read job queued ahead of the jobs not yet started
READ_RESILVER = 4  # CEC_READ_RESILVER: read-pipeline flag, FilePart::resilver's compute
READ_VERIFY_ONLY = 8  # CEC_READ_VERIFY_ONLY: read-pipeline flag, FilePart::verify's compute
READ_CARRY = 16  # CEC_READ_CARRY: read-pipeline flag, retries' verified chunks kept on the device


class MultiError(Error):
    def __init__(self, code: int):
        Exception.__init__(self, f"{_lib.cec_status_name(code).decode()}: "
                                 f"{_lib.cec_multi_last_error().decode()}")
        self.code = code
        self.name = _lib.cec_status_name(code).decode()


class Multi:
    """cec_multi: FileWriteBuilder::write / FileReadBuilder over several GPUs in one process.

    ``devices`` lists one device ordinal per shard (repeats allowed).  ``encode_hash`` /
    ``read`` take host buffers (numpy arrays or HostBuffer views; page-locked ones are DMA'd
    directly) and return a job id for ``wait``; the blocking forms ``encode_hash_sync`` /
    ``read_sync`` do both.  Shard g owns parts [g*n/G, (g+1)*n/G) of every job."""

    WRITE = 1  # CEC_MULTI_WRITE
    READ = 2  # CEC_MULTI_READ

    def __init__(self, codec: ReedSolomon, chunk_len: int, parts_per_batch: int, depth: int,
                 devices: Sequence[int], kinds: int = WRITE | READ):
        """``kinds``: the job kinds (WRITE, READ) whose pipelines every shard makes here, once."""
        h = _vp()
        devs = (ctypes.c_int * max(len(devices), 1))(*devices)
        code = _lib.cec_multi_new_ex(codec.handle, chunk_len, parts_per_batch, depth, devs,
                                     len(devices), kinds, ctypes.byref(h))
        if code != OK:
            raise MultiError(code)
        self._h = h
        self.codec = codec
        self.d, self.p = codec.data_shard_count(), codec.parity_shard_count()
        self.t = self.d + self.p
        self.L = chunk_len
        self._keep = {}

    def __del__(self, _free=_lib.cec_multi_free):
        h = getattr(self, "_h", None)
        if h:
            _free(h)
            self._h = None

    def shards(self) -> int:
        return _lib.cec_multi_shards(self._h)

    def shard_info(self, g: int):
        dev, numa, parts = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_uint64(0)
        _check(_lib.cec_multi_shard_info(self._h, g, ctypes.byref(dev), ctypes.byref(numa),
                                         ctypes.byref(parts)))
        return dev.value, numa.value, parts.value

    def stats(self, g: int) -> dict:
        """Shard g's counters (cec_multi_shard_stats)."""
        st = MultiStatsStruct()
        _check(_lib.cec_multi_shard_stats(self._h, g, ctypes.byref(st)))
        return {name: getattr(st, name) for name, _ in MultiStatsStruct._fields_}

    def carry_release(self, carry_id: int) -> None:
        """Gives back a carry id this caller will not use (cec_multi_carry_release)."""
        code = _lib.cec_multi_carry_release(self._h, int(carry_id))
        if code != OK:
            raise MultiError(code)

    def encode_hash(self, data, n_parts: int, parity, digests) -> int:
        job = ctypes.c_uint64(0)
        code = _lib.cec_multi_encode_hash(self._h, _addr(data), n_parts, _addr(parity),
                                          _addr(digests), ctypes.byref(job))
        if code != OK:
            raise MultiError(code)
        self._keep[job.value] = (data, parity, digests)
        return job.value

    def read(self, chunks, present, expected, n_parts: int, data, verified, status,
             rebuilt_only: bool = False, carry_in=None, carry_out=None, ahead: bool = False):
        """Returns (job, data_ptrs) where data_ptrs ([n*d] c_void_p) is filled at wait().
        carry_out ([n] int32 numpy, nullable) receives, at wait(), a carry id for each part
        reported TOO_FEW_SHARDS_PRESENT whose verified chunks stay on its GPU (-1: none);
        carry_in ([n] int32, nullable) hands such ids to a retry: those parts' PRESENT_VERIFIED
        chunks are taken from the GPU, not from `chunks` (cec_multi_read_carry).  ahead
        (CEC_MULTI_AHEAD): the job goes ahead of the queued jobs not yet started (a reader's retry
        round, which the window being emitted waits for)."""
        import numpy as np
        job = ctypes.c_uint64(0)
        ptrs = (ctypes.c_void_p * max(n_parts * self.d, 1))()
        i32 = ctypes.POINTER(ctypes.c_int32)
        cin = None
        if carry_in is not None:
            cin = np.ascontiguousarray(carry_in, dtype=np.int32)
            assert len(cin) >= n_parts
        if carry_out is not None:
            assert carry_out.dtype == np.int32 and carry_out.flags.c_contiguous
            assert len(carry_out) >= n_parts
        code = _lib.cec_multi_read_carry(
            self._h, _addr(chunks), _addr(present), _addr(expected), n_parts, _addr(data),
            _addr(verified), ctypes.cast(_addr(status), ctypes.POINTER(ctypes.c_int)), ptrs,
            (1 if rebuilt_only else 0) | (MULTI_AHEAD if ahead else 0),
            cin.ctypes.data_as(i32) if cin is not None else None,
            carry_out.ctypes.data_as(i32) if carry_out is not None else None, ctypes.byref(job))
        if code != OK:
            raise MultiError(code)
        self._keep[job.value] = (chunks, present, expected, data, verified, status, ptrs, cin,
                                 carry_out)
        return job.value, ptrs

    def resilver(self, chunks, present, expected, n_parts: int, rebuilt, verified, status):
        """FilePart::resilver's compute; returns (job, chunk_ptrs [n*(d+p)] filled at wait())."""
        job = ctypes.c_uint64(0)
        ptrs = (ctypes.c_void_p * max(n_parts * self.t, 1))()
        code = _lib.cec_multi_resilver(self._h, _addr(chunks), _addr(present), _addr(expected),
                                       n_parts, _addr(rebuilt), _addr(verified),
                                       ctypes.cast(_addr(status), ctypes.POINTER(ctypes.c_int)),
                                       ptrs, ctypes.byref(job))
        if code != OK:
            raise MultiError(code)
        self._keep[job.value] = (chunks, present, expected, rebuilt, verified, status, ptrs)
        return job.value, ptrs

    def resilver_sync(self, chunks, present, expected, n_parts: int, rebuilt, verified, status):
        job, ptrs = self.resilver(chunks, present, expected, n_parts, rebuilt, verified, status)
        keep = self._keep[job]
        self.wait(job)
        del keep
        return [p or 0 for p in ptrs[: n_parts * self.t]]

    def verify(self, chunks, present, expected, n_parts: int, verified) -> int:
        """FilePart::verify's compute: verified[n][d+p] for every loaded chunk; returns the job."""
        job = ctypes.c_uint64(0)
        code = _lib.cec_multi_verify(self._h, _addr(chunks), _addr(present), _addr(expected),
                                     n_parts, _addr(verified), ctypes.byref(job))
        if code != OK:
            raise MultiError(code)
        self._keep[job.value] = (chunks, present, expected, verified)
        return job.value

    def verify_sync(self, chunks, present, expected, n_parts: int, verified) -> None:
        self.wait(self.verify(chunks, present, expected, n_parts, verified))

    def wait(self, job: int) -> None:
        code = _lib.cec_multi_wait(self._h, job)
        self._keep.pop(job, None)
        if code != OK:
            raise MultiError(code)

    def query(self, job: int) -> bool:
        """True when the job is done (wait() then returns at once); never blocks
        (cec_multi_query)."""
        code = _lib.cec_multi_query(self._h, job)
        if code not in (0, 1):
            raise MultiError(code)
        return code == 1

    def encode_hash_sync(self, data, n_parts: int, parity, digests) -> None:
        self.wait(self.encode_hash(data, n_parts, parity, digests))

    def read_sync(self, chunks, present, expected, n_parts: int, data, verified, status,
                  rebuilt_only: bool = False):
        job, ptrs = self.read(chunks, present, expected, n_parts, data, verified, status,
                              rebuilt_only)
        keep = self._keep[job]
        self.wait(job)
        del keep
        return [p or 0 for p in ptrs[: n_parts * self.d]]
