"""FileReadBuilder's reader batched over the multi-GPU scheduler, with read_with_context's retry
rule, parts handed out in file order: the Python twin of the Rust crate's
``chunky_ec_sys::batch::BatchReader`` / ``read_part`` / ``FileReader``
(chunky-bits_amd/rust/chunky-ec-sys/src/batch.rs) and of the C++ ``FileReference::read_run`` /
``retry_start`` / ``retry_collect`` (include/chunky_ec.hpp), step for step, so the loop the Rust side would run is executed
and tested on the GPU (tests/test_gpu_batchreader.py).

The reference reads a part by drawing chunks until d of them verify (src/file/file_part.rs:
86-107): for each drawn chunk it walks the chunk's locations in order and keeps the first copy
whose SHA-256 matches the metadata, and only when none does it draws another chunk.  It then
rebuilds the missing data chunks (:123-129), and FileReadBuilder yields the parts in file order
(src/file/reader.rs:40-75).

``fetch(part, chunk, start)`` is that walk's step: it reads the chunk's locations from index
``start`` on and returns ``(location index, bytes)`` of the first one that reads, or None when no
location is left (``Location::read_with_context`` over ``chunk.locations[start..]``).  A copy
that fails verification is followed by the same chunk's next location (``start`` = its index + 1)
before another chunk is drawn, so a chunk listed ``[bad, good]`` -- what resilver leaves behind
when it appends a rebuilt copy's location (file_part.rs:346) -- reads like in the reference.

:class:`BatchReader` loads a window of ``parts_per_batch * len(devices)`` parts of one shape at a
time -- for each part the first d chunks that fetch returns a copy of (data chunks first, so an
intact part needs no rebuild) -- into a page-locked buffer and submits the window as one scheduler
job (verify every loaded chunk, rebuild the data chunks; parts split over the GPUs in contiguous
ranges) while it loads the next window.  A part whose loaded chunks do not all verify is
resubmitted with the chunks that verified flagged ``CEC_PRESENT_VERIFIED`` (used, not hashed
again; kept on the GPU under the part's carry id), the failed chunks' next copies, then untried
chunks, up to d, until it decodes; a part that runs out of copies fails the read with
TooFewShardsPresent, as the reference's does.  depth + 1 window buffers (at most 8): a window is
checked (its job waited for, its failed parts' first retry round queued, ahead of the windows
queued after it: CEC_MULTI_AHEAD) as soon as its job is done (Multi.query), and each next round
as soon as the last one is, so retries run on the GPUs while the next windows load.  Only the
rebuilt data chunks come down (REBUILT_ONLY): a loaded one reaches the sink from the window's
chunk buffer it went up from.
:func:`read_part` is the same rule for one part through the per-call API, and :class:`FileReader`
splits a file into runs of one shape (chunk size, d, p: the short last part has its own chunk size,
file_part.rs:152) and keeps one BatchReader per shape.
"""
from __future__ import annotations

import time
from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

from . import (ERR_INVALID_ARGUMENT, OK, PRESENT_VERIFIED, TOO_FEW_SHARDS_PRESENT, Error, HostBuffer,
               Multi, ReedSolomon, Sha256Hash)

Fetch = Callable[[int, int, int], Optional[Tuple[int, bytes]]]


def next_copy(fetch: Fetch, part: int, chunk: int, start: int, size: int):
    """The chunk's next copy from location ``start`` on: ``(next start, bytes)``, or None when its
    locations are exhausted.  A copy that is not ``size`` bytes cannot hash to the metadata digest
    (the reference hashes it and moves on), so it is passed over here."""
    while True:
        got = fetch(part, chunk, start)
        if got is None:
            return None
        loc, b = got
        start = loc + 1
        if len(b) == size:
            return start, b


def draw_order(good, tried, exhausted):
    """Chunk indices to load next for a part that is short of d verified chunks: the chunks whose
    copy failed verification first (their next location: file_part.rs:100-107 walks a chunk's
    locations before drawing another chunk), then the untried ones."""
    t = len(good)
    again = [i for i in range(t) if tried[i] and not good[i] and not exhausted[i]]
    fresh = [i for i in range(t) if not tried[i] and not exhausted[i]]
    return again + fresh


@dataclass
class _Retry:
    """The retry of a window's failed parts (file_part.rs:92-107), one round in flight at a time."""
    failed: List[int]                     # window rows of the failed parts
    tried: dict
    good: dict
    cursor: dict
    exhausted: dict
    keep: dict                            # bytes of every chunk loaded so far
    cid: dict                             # carry id of the part's verified chunks (-1: none)
    open_: List[int]
    job: int = 0
    in_flight: bool = False


@dataclass
class _Window:
    slot: int
    job: int
    first: int
    n: int
    checked: bool = False                 # its read job waited for (and its retry started)
    retry: Optional[_Retry] = None
    ptrs: object = None                   # [n*d] where each data chunk is (filled at wait)
    redone: set = field(default_factory=set)  # parts whose data the retries put in `out`


class BatchReader:

    def __init__(self, data: int, parity: int, chunk_size: int, parts_per_batch: int, depth: int,
                 devices: List[int], carry: bool = True):
        """carry=False: retries send their verified chunks again instead of leaving them on the
        GPU (the comparison tests/test_gpu_batchreader.py makes)."""
        self.codec = ReedSolomon(data, parity)  # file_part.rs:77
        self.multi = Multi(self.codec, chunk_size, parts_per_batch, depth, devices,
                           kinds=Multi.READ)
        self.use_carry = carry
        self.d, self.p, self.t, self.L = data, parity, data + parity, chunk_size
        self.window = parts_per_batch * max(len(devices), 1)
        dev0 = devices[0] if devices else -1
        # window buffers: up to depth windows' read jobs in flight, one being emitted
        self.R = R = min(max(depth, 2), 7) + 1
        W, t, L = self.window, self.t, chunk_size
        self.chunks = [HostBuffer(W * t * L, dev0) for _ in range(R)]
        self.out = [HostBuffer(W * data * L, dev0) for _ in range(R)]
        self.present = [np.zeros((W, t), np.uint8) for _ in range(R)]
        self.expected = [np.zeros((W, t, 32), np.uint8) for _ in range(R)]
        self.verified = [np.zeros((W, t), np.uint8) for _ in range(R)]
        self.status = [np.zeros(W, np.int32) for _ in range(R)]
        # per chunk of the window: the next location to read, and whether none is left
        self.cursor = [np.zeros((W, t), np.int64) for _ in range(R)]
        self.exhausted = [np.zeros((W, t), bool) for _ in range(R)]
        # per part of the window: the scheduler's carry id of its verified chunks (-1: none)
        self.carry = [np.full(W, -1, np.int32) for _ in range(R)]
        self.retries = 0  # part resubmissions (a part retried twice counts twice)
        self.carried_parts = 0  # retried parts whose verified chunks stayed on the GPU
        self.dev0 = dev0
        # per window: retry buffers (page-locked chunks / data, kept copies; grown only)
        self._scr_parts = [0] * R
        self._scr = [None] * R

    def read(self, n_parts: int, fetch: Fetch, digests: Callable[[int], np.ndarray],
             sink: Callable[[int, List[memoryview]], None]):
        """Parts 0..n_parts-1 (all of this reader's shape): ``fetch(part, chunk, start)`` as the
        module describes, ``digests(part)`` the part's metadata digests [d+p][32]; ``sink(part,
        data_chunks)`` gets the d data chunks of every part, in file order.  Every window is
        checked (its job waited for, the first round of its failed parts' retry queued) as soon as
        its job is done, and its retry's next round queued as soon as the last one is
        (Multi.query never blocks), so retries run on the GPUs while windows load and while the
        loop waits for the window it emits (a retry round costs one SHA-256 chain, ~33 ms for
        1 MiB chunks, whatever its size)."""
        R = self.R
        live: List[Optional[_Window]] = [None] * R
        at = i = 0
        try:
            while True:
                # windows are emitted in submission order: live[i % R] went out R steps ago
                self._poll(live, i + 1, None, at >= n_parts, fetch)
                s = i % R
                if live[s] is not None:
                    self._finish(live[s], live, i, at >= n_parts, fetch, sink)
                    live[s] = None
                if at < n_parts:
                    cnt = min(self.window, n_parts - at)
                    self._load(s, at, cnt, fetch, digests)
                    job, ptrs = self._submit(s, cnt)
                    live[s] = _Window(s, job, at, cnt, ptrs=ptrs)
                    at += cnt
                elif all(x is None for x in live):
                    return
                i += 1
        except BaseException:
            self._drain(live)
            raise

    def _load(self, slot, first, cnt, fetch, digests):
        """The first d chunks of each part that fetch returns a copy of (file_part.rs:86-107 loads
        d), with every chunk's metadata digest."""
        d, t, L = self.d, self.t, self.L
        ch = self.chunks[slot].view(self.window, t, L)
        pres, exp = self.present[slot], self.expected[slot]
        cur, ex = self.cursor[slot], self.exhausted[slot]
        pres[:cnt] = 0
        cur[:cnt] = 0
        ex[:cnt] = False
        self.carry[slot][:cnt] = -1
        for q in range(cnt):
            exp[q] = digests(first + q)
            loaded = 0
            for i in range(t):
                if loaded == d:
                    break
                c = next_copy(fetch, first + q, i, 0, L)
                if c is None:
                    ex[q, i] = True
                    continue
                cur[q, i], b = c
                ch[q, i] = np.frombuffer(b, np.uint8)
                pres[q, i] = 1
                loaded += 1

    def _submit(self, slot, cnt):
        """REBUILT_ONLY: only the rebuilt data chunks come down; a loaded one is handed to the sink
        from the window's chunk buffer it went up from.  Returns (job, data pointers)."""
        return self.multi.read(self.chunks[slot], self.present[slot], self.expected[slot], cnt,
                               self.out[slot], self.verified[slot], self.status[slot],
                               rebuilt_only=True,
                               carry_out=self.carry[slot] if self.use_carry else None)

    def _check(self, w: _Window, fetch):
        """Waits for the window's read job; its failed parts' first retry round goes out."""
        w.checked = True
        self.multi.wait(w.job)
        st = self.status[w.slot]
        failed = [q for q in range(w.n) if st[q] != OK]
        if failed:
            self._retry_start(w, failed, fetch)

    def _poll(self, live, first, skip, everything, fetch):
        """Every live window but `skip`: checked if its job is done, its retry's next round
        queued if the last one is done; everything: checked whatever its state (nothing is left
        to load: the last retries run together)."""
        R = self.R
        for a in range(R):
            x = live[(first + a) % R]
            if x is None or x is skip:
                continue
            if not x.checked:
                if everything or self.multi.query(x.job):
                    self._check(x, fetch)
            elif x.retry is not None and x.retry.in_flight and self.multi.query(x.retry.job):
                self._retry_collect(x, fetch)

    def _finish(self, w: _Window, live, i, everything, fetch, sink):
        """w's job, then its retry rounds (polling the other windows meanwhile), then its parts
        to the sink."""
        while True:
            if not w.checked and self.multi.query(w.job):
                self._check(w, fetch)
            rt = w.retry
            if w.checked and rt is not None and rt.in_flight and self.multi.query(rt.job):
                self._retry_collect(w, fetch)
            if w.checked and (w.retry is None or not w.retry.in_flight):
                break
            self._poll(live, i + 1, w, everything, fetch)
            time.sleep(100e-6)
        w.retry = None
        d, L = self.d, self.L
        chb, outb = self.chunks[w.slot], self.out[w.slot]
        ch, out = memoryview(chb.array), memoryview(outb.array)

        def chunk(q, j):
            if q in w.redone:
                return out[(q * d + j) * L:(q * d + j + 1) * L]
            p = w.ptrs[q * d + j] or 0
            for base, n, view in ((chb.ptr, chb.nbytes, ch), (outb.ptr, outb.nbytes, out)):
                if base <= p and p + L <= base + n:
                    return view[p - base:p - base + L]
            raise Error(ERR_INVALID_ARGUMENT)  # a data pointer outside the window's buffers
        for q in range(w.n):
            sink(w.first + q, [chunk(q, j) for j in range(d)])

    def _retry_start(self, w: _Window, failed, fetch):
        """file_part.rs:92-107: the failed parts go again with the chunks that verified
        (PRESENT_VERIFIED) plus, up to d, the failed chunks' next copies and then untried chunks,
        until each decodes or runs out of copies.  The verified chunks stay on the GPU where the
        scheduler kept them (the part's carry id: only the new chunks are sent), or, when it kept
        none, are sent again from the window's buffer (the bytes that verified).  This queues the
        first round; _retry_collect takes each round's results and queues the next round."""
        t, L = self.t, self.L
        ch = self.chunks[w.slot].view(self.window, t, L)
        pres, ver = self.present[w.slot], self.verified[w.slot]
        _, _, kbuf = self._retry_buffers(w.slot, len(failed))
        keep = {}
        for r, q in enumerate(failed):
            kbuf[r] = ch[q]
            keep[q] = kbuf[r]
        cid = {}
        for q in failed:  # the retry holds the ids now
            cid[q] = int(self.carry[w.slot][q]) if self.use_carry else -1
            self.carry[w.slot][q] = -1
        w.retry = _Retry(failed, {q: pres[q] != 0 for q in failed}, {q: ver[q] != 0 for q in failed},
                         {q: self.cursor[w.slot][q].copy() for q in failed},
                         {q: self.exhausted[w.slot][q].copy() for q in failed}, keep, cid,
                         list(failed))
        self._retry_round(w, fetch)

    def _retry_buffers(self, slot, f):
        """The window's retry buffers, kept between retries (fresh zeroed ones cost ~200 ms of page
        faults per retry of a dozen RS(10,4) 1 MiB parts); rc / ro page-locked, so a single-shard
        retry goes up without staging.  Returns rc [f][t][L], ro [f][d][L], kept copies."""
        d, t, L = self.d, self.t, self.L
        if self._scr_parts[slot] < f:
            self._scr[slot] = None  # the old buffers go before the new ones are pinned
            n = max(f, 2 * self._scr_parts[slot])
            self._scr[slot] = (HostBuffer(n * t * L, self.dev0), HostBuffer(n * d * L, self.dev0),
                               np.empty((n, t, L), np.uint8))
            self._scr_parts[slot] = n
        rc_b, ro_b, kbuf = self._scr[slot]
        return (rc_b.array[:f * t * L].reshape(f, t, L), ro_b.array[:f * d * L].reshape(f, d, L),
                kbuf[:f])

    def _retry_round(self, w: _Window, fetch):
        """Builds and queues one round over the still-open failed parts."""
        d, t, L = self.d, self.t, self.L
        rt = w.retry
        f = len(rt.failed)
        rc, ro, _ = self._retry_buffers(w.slot, f)
        g = len(rt.open_)
        rt.r_pres = np.zeros((g, t), np.uint8)
        rt.r_exp = np.zeros((g, t, 32), np.uint8)
        rt.r_ver = np.zeros((g, t), np.uint8)
        rt.r_st = np.zeros(g, np.int32)
        rt.r_cin = np.full(g, -1, np.int32)
        rt.r_cout = np.full(g, -1, np.int32)
        for s, q in enumerate(rt.open_):
            rt.r_exp[s] = self.expected[w.slot][q]
            rt.r_cin[s] = rt.cid[q]
            have = int(rt.good[q].sum())
            for i in range(t):
                if rt.good[q][i]:
                    if rt.cid[q] < 0:  # not kept on the GPU: send the bytes that verified
                        rc[s, i] = rt.keep[q][i]
                    rt.r_pres[s, i] = PRESENT_VERIFIED
            added = 0
            for i in draw_order(rt.good[q], rt.tried[q], rt.exhausted[q]):
                if not have + added < d:
                    break
                rt.tried[q][i] = True
                c = next_copy(fetch, w.first + q, i, int(rt.cursor[q][i]), L)
                if c is None:
                    rt.exhausted[q][i] = True
                    continue
                rt.cursor[q][i], b = c
                rt.keep[q][i] = np.frombuffer(b, np.uint8)
                rc[s, i] = rt.keep[q][i]
                rt.r_pres[s, i] = 1
                added += 1
            if added == 0:
                raise Error(TOO_FEW_SHARDS_PRESENT)
        rt.job, _ = self.multi.read(rc[:g], rt.r_pres, rt.r_exp, g, ro[:g], rt.r_ver, rt.r_st,
                                    carry_in=rt.r_cin,
                                    carry_out=rt.r_cout if self.use_carry else None, ahead=True)
        for q in rt.open_:  # submitted: the ids are the job's now
            self.carried_parts += 1 if rt.cid[q] >= 0 else 0
            rt.cid[q] = -1
        rt.in_flight = True

    def _retry_collect(self, w: _Window, fetch):
        """Waits for the round in flight: the parts that decoded go to the window's output, the
        others go again in the next round, queued here (until every part decodes or one runs out
        of copies)."""
        d = self.d
        rt = w.retry
        out = self.out[w.slot].view(self.window, d, self.L)
        _, ro, _ = self._retry_buffers(w.slot, len(rt.failed))
        if rt.in_flight:
            rt.in_flight = False
            self.multi.wait(rt.job)
            self.retries += len(rt.open_)
            still = []
            for s, q in enumerate(rt.open_):
                rt.good[q] = rt.r_ver[s] != 0
                if rt.r_st[s] == OK:
                    out[q] = ro[s]
                    w.redone.add(q)
                else:
                    rt.cid[q] = int(rt.r_cout[s])
                    still.append(q)
            rt.open_ = still
            if still:
                self._retry_round(w, fetch)

    def _drain(self, live) -> None:
        """Error path: no job may still write into the windows; carry ids nobody will use go back
        to their GPUs."""
        for w in live:
            if w is None:
                continue
            ids = []
            try:
                if not w.checked:
                    self.multi.wait(w.job)
                rt = w.retry
                if rt is not None and rt.in_flight:
                    self.multi.wait(rt.job)
                    # the round's ids for its parts still short of d: nobody collects them now
                    ids += [int(c) for c in rt.r_cout[:len(rt.open_)] if c >= 0]
            except Exception:  # noqa: BLE001 (the error being raised is the caller's)
                pass
            ids += [int(c) for c in self.carry[w.slot][:w.n] if c >= 0]
            if w.retry is not None:
                ids += [c for c in w.retry.cid.values() if c >= 0]
            for c in ids:
                try:
                    self.multi.carry_release(c)
                except Exception:  # noqa: BLE001
                    pass


def read_part(codec: ReedSolomon, chunksize: int, digests: np.ndarray, fetch: Fetch,
              part: int) -> bytes:
    """read_with_context (file_part.rs:73-135) for one part through the per-call API, with the
    batched loop's rule: d chunks drawn (data first), each kept at its first copy that verifies,
    failed chunks' next copies and then untried chunks until d verify (TooFewShardsPresent when
    the copies run out), missing data rebuilt.  The path for a part whose shape no BatchReader of
    the file has (the short last part, chunk size ceil(len / d))."""
    d = codec.data_shard_count()
    t = codec.total_shard_count()
    good, tried, exhausted = [False] * t, [False] * t, [False] * t
    cursor = [0] * t
    shards: List[Optional[bytearray]] = [None] * t
    while sum(good) < d:
        batch = []
        for i in draw_order(good, tried, exhausted):
            if sum(good) + len(batch) >= d:
                break
            tried[i] = True
            c = next_copy(fetch, part, i, cursor[i], chunksize)
            if c is None:
                exhausted[i] = True
                continue
            cursor[i], b = c
            batch.append((i, b))
        if not batch:
            raise Error(TOO_FEW_SHARDS_PRESENT)
        hashes = Sha256Hash.from_bufs([b for _, b in batch])  # one launch per round
        for (i, b), h in zip(batch, hashes):
            if h.digest == bytes(digests[i]):
                good[i] = True
                shards[i] = bytearray(b)
    if not all(s is not None for s in shards[:d]):
        codec.reconstruct_data(shards)
    return b"".join(bytes(s) for s in shards[:d])


Shape = Tuple[int, int, int]  # (d, p, chunksize) of a part


class FileReader:
    """FileReadBuilder's reader over a whole file (reader.rs:32-74): consecutive parts of one
    shape (d, p, chunk size) form a run; a run of two or more parts goes through a BatchReader of
    that shape -- kept (the ``keep`` most recently used shapes) for the next file, since its
    windows pin memory (~0.35 s per GiB) -- and a lone part (the short last part) through
    :func:`read_part`.  Parts reach ``sink(part, data_chunks)`` in file order."""

    def __init__(self, parts_per_batch: int, depth: int, devices: List[int], keep: int = 2):
        self.ppb, self.depth, self.devices, self.keep = parts_per_batch, depth, list(devices), keep
        self.readers: "OrderedDict[Shape, BatchReader]" = OrderedDict()
        self.codecs: "OrderedDict[Tuple[int, int], ReedSolomon]" = OrderedDict()

    def reader(self, shape: Shape) -> BatchReader:
        r = self.readers.pop(shape, None)
        if r is None:
            while len(self.readers) >= self.keep:  # free the least recently used first
                self.readers.popitem(last=False)
            d, p, L = shape
            r = BatchReader(d, p, L, self.ppb, self.depth, self.devices)
        self.readers[shape] = r
        return r

    def _codec(self, d: int, p: int) -> ReedSolomon:
        c = self.codecs.pop((d, p), None) or ReedSolomon(d, p)
        self.codecs[(d, p)] = c
        while len(self.codecs) > self.keep:
            self.codecs.popitem(last=False)
        return c

    def read(self, shapes: Sequence[Shape], fetch: Fetch, digests: Callable[[int], np.ndarray],
             sink: Callable[[int, List], None], first: int = 0, end: Optional[int] = None) -> None:
        """Parts [first, end) (default: every part) to ``sink(part, data_chunks)`` in order."""
        end = len(shapes) if end is None else min(end, len(shapes))
        k = first
        while k < end:
            run = 1
            while k + run < end and shapes[k + run] == shapes[k]:
                run += 1
            d, p, L = shapes[k]
            if run < 2:
                data = read_part(self._codec(d, p), L, digests(k), fetch, k)
                sink(k, [memoryview(data)[j * L:(j + 1) * L] for j in range(d)])
            else:
                k0 = k
                self.reader(shapes[k]).read(
                    run, lambda q, i, s: fetch(k0 + q, i, s), lambda q: digests(k0 + q),
                    lambda q, data: sink(k0 + q, data))
            k += run

    def read_range(self, shapes: Sequence[Shape], length: int, seek: int, take: int, fetch: Fetch,
                   digests: Callable[[int], np.ndarray], sink: Callable[[int, List], None]) -> int:
        """FileReadBuilder::seek / take (reader.rs:22-173): the file's bytes [seek, seek +
        range_len) -- ``length`` is FileReference::len_bytes -- from the parts that hold them,
        ``sink(part, pieces)`` getting each part's bytes inside the range as memoryviews.  Parts
        wholly before the range are not read and the first part's leading bytes are dropped, as
        the reference does (reader.rs:44-65); parts wholly past it are not read either (the
        reference reads them and empties their bytes, reader.rs:67-75: an undecodable part past
        the range fails its read, not this one).  Returns the bytes handed out."""
        want = range_len(length, seek, take)
        if want == 0:
            return 0
        part_len = [d * L for d, _, L in shapes]
        k, skip = 0, seek
        while k < len(shapes) and skip >= part_len[k]:
            skip -= part_len[k]
            k += 1
        end, covered = k, 0
        while end < len(shapes) and covered < skip + want:
            covered += part_len[end]
            end += 1
        state = {"skip": skip, "left": want}

        def trim(q, data):
            pieces = []
            for c in data:
                c = memoryview(c)
                s = min(len(c), state["skip"])
                state["skip"] -= s
                c = c[s:]
                m = min(len(c), state["left"])
                state["left"] -= m
                if m:
                    pieces.append(c[:m])
            sink(q, pieces)

        self.read(shapes, fetch, digests, trim, k, end)
        return want - state["left"]


def range_len(length: int, seek: int, take: int) -> int:
    """FileReadBuilder::len_bytes (reader.rs:129-138): the bytes a read from ``seek`` taking
    ``take`` (0: to the end) gives of a ``length``-byte file; 0 for a seek past the end (where the
    reference's u64 subtraction would underflow)."""
    if seek >= length:
        return 0
    return length - seek if take == 0 else min(take, length - seek)
