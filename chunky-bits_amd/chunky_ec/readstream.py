"""FileReadBuilder's part loop over a ReadPipeline, with read_with_context's retry rule.

The reference reads a part by sampling chunks at random until d of them verify
(src/file/file_part.rs:86-107: each of the d futures draws an untried chunk, reads it and keeps
it only if its sha256 matches the metadata; a chunk that fails is dropped and another is drawn),
then rebuilds the missing data chunks (file_part.rs:123-129).  FileReadBuilder streams the parts
in file order (src/file/reader.rs:40-75).

:class:`ReadRepairStream` runs that loop batched over a :class:`chunky_ec.ReadPipeline` (pinned
slots, `depth` batches in flight):

* a new part loads d chunks drawn at random from its d+p;
* a part the pipeline reports ``TooFewShardsPresent`` (one of its loaded chunks failed the
  hash) is queued for a retry: its verified chunks are loaded again flagged
  ``CEC_PRESENT_VERIFIED`` (used, not hashed again) plus as many untried chunks, drawn at random,
  as it is short of d; the next batch carries the queued retries ahead of its new parts;
* a part with fewer than d chunks left to try is undecodable (the reference's read fails with
  ``TooFewShardsPresent`` there; the stream counts it and goes on);
* on a pipeline made with ``ReadPipeline.CARRY`` the verified chunks of a part to retry stay on
  the device (the reference keeps them in memory, file_part.rs:102-104): its retry takes them
  from the carry pool, so only the new chunks are fetched and uploaded.

The caller supplies the storage side: ``fetch(chunks, rows)`` copies the chunk bytes into the
slot's pinned [parts][d+p][L] array for every (row, part id, flags) in ``rows``, for each chunk
whose flag is nonzero.  A chunk flagged 1 is a fresh read (it may come back corrupted: that is
what the retries are for); one flagged ``CEC_PRESENT_VERIFIED`` must be the bytes that verified
before (the reference keeps a verified chunk in memory, file_part.rs:102-104).
``digests(part_ids)`` returns the metadata digests [n][d+p][32].  Host bookkeeping only; all
hashing and decoding runs in the pipeline's HIP kernels.
"""
from __future__ import annotations

import time
from collections import deque
from dataclasses import dataclass, field
from typing import Callable, Deque, List, Optional, Sequence, Tuple

import numpy as np

from . import OK, PRESENT_VERIFIED, TOO_FEW_SHARDS_PRESENT, Error


@dataclass
class _Part:
    part: int                 # part id (file order)
    tried: np.ndarray         # [t] bool: chunks loaded by any pass so far
    good: np.ndarray          # [t] bool: chunks that verified
    attempts: int = 1         # submissions of this part so far
    carry: int = -1           # CARRY pipelines: the carry entry holding its verified chunks


@dataclass
class ReadRepairStats:
    parts: int = 0              # parts read back (decoded) successfully
    batches: int = 0            # batches submitted (new + retry)
    retry_batches: int = 0      # batches made of retried parts only (after the last new part)
    mixed_batches: int = 0      # batches carrying retried parts ahead of new ones
    retried_parts: int = 0      # part resubmissions (a part retried twice counts twice)
    rejected_chunks: int = 0    # loaded chunks whose sha256 did not match the metadata
    undecodable_parts: int = 0  # parts left with fewer than d chunks to try
    chunks_loaded: int = 0      # chunk loads (first loads, retry loads and re-sent verified ones)
    carried_chunks: int = 0     # verified chunks a retry took from the device carry pool
    undecodable: List[int] = field(default_factory=list)  # their part ids (first 64)
    # where the loop's time went (seconds): filling slots (fetch), waiting for the oldest batch,
    # the rest (batch building, digests, bookkeeping)
    fetch_s: float = 0.0
    wait_s: float = 0.0
    loop_s: float = 0.0

    def as_dict(self) -> dict:
        out = dict(self.__dict__)
        out["undecodable"] = list(self.undecodable)
        for k in ("fetch_s", "wait_s", "loop_s"):
            out[k] = round(out[k], 3)
        return out


class ReadRepairStream:
    """Batched read_with_context with retries over `rp` (a ReadPipeline or anything with its
    acquire / submit / wait / drain and `parts`, `d`, `t` attributes)."""

    def __init__(self, rp, fetch: Callable[[np.ndarray, Sequence[Tuple[int, int, np.ndarray]]], None],
                 digests: Callable[[np.ndarray], np.ndarray], seed: int = 0,
                 on_part: Optional[Callable[[int, int, int, int, int], None]] = None):
        self.rp = rp
        self.fetch = fetch
        self.digests = digests
        self.rng = np.random.default_rng(seed)
        # on_part(slot, n_parts_in_batch, row, part id, attempts): called for every part that
        # decoded, while its output is valid (before the slot is acquired again)
        self.on_part = on_part
        self.P, self.d, self.t = rp.parts, rp.d, rp.t
        self.depth = rp.depth
        self.carry = bool(getattr(rp, "carry", False))
        self.stats = ReadRepairStats()
        self._retry: Deque[_Part] = deque()
        self._inflight: Deque[Tuple[int, List[_Part], np.ndarray]] = deque()

    # -- batch building -------------------------------------------------------------------------

    def _new_parts(self, first: int, n: int) -> Tuple[List[_Part], np.ndarray]:
        """Parts [first, first + n): d chunks each, drawn uniformly without replacement."""
        t, d = self.t, self.d
        pick = np.argsort(self.rng.random((n, t)), axis=1)[:, :d]
        present = np.zeros((n, t), np.uint8)
        np.put_along_axis(present, pick, 1, axis=1)
        parts = [_Part(first + k, present[k] != 0, np.zeros(t, bool)) for k in range(n)]
        return parts, present

    def _retry_parts(self) -> Tuple[List[_Part], np.ndarray]:
        """Up to P queued retries: verified chunks re-sent as PRESENT_VERIFIED plus untried ones
        drawn at random up to d; parts that cannot reach d are counted undecodable."""
        t, d = self.t, self.d
        parts, rows = [], []
        while self._retry and len(parts) < self.P:
            e = self._retry.popleft()
            need = d - int(e.good.sum())
            untried = np.flatnonzero(~e.tried)
            if need <= 0 or len(untried) < need:
                # need <= 0 cannot come back from the pipeline (d verified chunks decode); fewer
                # untried chunks than needed: the reference's read runs out of chunks here
                self.stats.undecodable_parts += 1
                if len(self.stats.undecodable) < 64:
                    self.stats.undecodable.append(e.part)
                if e.carry >= 0:  # its kept chunks will not be used
                    self.rp.carry_release(e.carry)
                    e.carry = -1
                continue
            new = self.rng.choice(untried, need, replace=False)
            row = np.where(e.good, PRESENT_VERIFIED, 0).astype(np.uint8)
            row[new] = 1
            e.tried[new] = True
            parts.append(e)
            rows.append(row)
        present = np.stack(rows) if rows else np.zeros((0, t), np.uint8)
        return parts, present

    def _submit(self, parts: List[_Part], present: np.ndarray) -> None:
        n = len(parts)
        slot, chunks, pres, expected = self.rp.acquire()
        pres[:n] = present
        ids = np.fromiter((e.part for e in parts), dtype=np.int64, count=n)
        expected[:n] = self.digests(ids)
        carry = np.fromiter((e.carry for e in parts), dtype=np.int32, count=n)
        # a carried part's verified chunks are on the device already: fetch only its new ones
        fetch_rows = present.copy()
        fetch_rows[(carry >= 0)[:, None] & (present == PRESENT_VERIFIED)] = 0
        t0 = time.perf_counter()
        self.fetch(chunks, [(k, int(ids[k]), fetch_rows[k]) for k in range(n)])
        self.stats.fetch_s += time.perf_counter() - t0
        if (carry >= 0).any():
            self.rp.submit_carried(slot, n, carry)
            for e in parts:
                e.carry = -1  # an entry is used once
        else:
            self.rp.submit(slot, n)
        self.stats.batches += 1
        self.stats.chunks_loaded += int(np.count_nonzero(fetch_rows))
        self.stats.carried_chunks += int(np.count_nonzero(present) - np.count_nonzero(fetch_rows))
        self._inflight.append((slot, parts, present))

    # -- results --------------------------------------------------------------------------------

    def _collect(self) -> None:
        slot, parts, present = self._inflight.popleft()
        t0 = time.perf_counter()
        _, ver, status = self.rp.wait(slot)
        self.stats.wait_s += time.perf_counter() - t0
        n = len(parts)
        carry = self.rp.carry_ids(slot, n) if self.carry else None
        for k in range(n):
            st = int(status[k])
            e = parts[k]
            if st == OK:
                self.stats.parts += 1
                if self.on_part is not None:
                    self.on_part(slot, n, k, e.part, e.attempts)
                continue
            if st != TOO_FEW_SHARDS_PRESENT:
                raise Error(st)
            loaded = present[k] != 0
            ok = ver[k] != 0
            self.stats.rejected_chunks += int(np.count_nonzero(loaded & ~ok))
            e.good = ok.copy()
            e.carry = int(carry[k]) if carry is not None else -1
            e.attempts += 1
            self.stats.retried_parts += 1
            self._retry.append(e)

    # -- driver ---------------------------------------------------------------------------------

    def run(self, first: int, n_parts: int) -> ReadRepairStats:
        """Read parts [first, first + n_parts) to the end, retries included; returns the stats.

        Every batch takes the queued retries first and fills the rest with new parts, so a retried
        part goes out in the next batch and batches stay full (a batch costs about one SHA-256
        chain of time whatever its size).  After the last new part, retries wait until every
        batch in flight is in and then go out together: one batch (one SHA-256 chain, ~40 ms for
        1 MiB chunks) for the retries of the last `depth` batches instead of one batch each,
        which ran one after another (profiles/r6/c5r_sizes: the stream's fixed cost)."""
        nxt, end = first, first + n_parts
        t_run = time.perf_counter()
        while nxt < end or self._retry or self._inflight:
            # a slot is reused round-robin: collect the oldest batch before its slot is acquired
            if len(self._inflight) == self.depth:
                self._collect()
            if nxt < end or (self._retry and not self._inflight):
                parts, present = self._retry_parts()
                room = self.P - len(parts)
                if nxt < end and room > 0:
                    n = min(room, end - nxt)
                    new, new_present = self._new_parts(nxt, n)
                    nxt += n
                    if parts:
                        self.stats.mixed_batches += 1
                    parts, present = parts + new, np.concatenate([present, new_present])
                elif parts:
                    self.stats.retry_batches += 1
                if parts:
                    self._submit(parts, present)
                continue
            if self._inflight:
                self._collect()
        self.rp.drain()
        self.stats.loop_s = time.perf_counter() - t_run - self.stats.fetch_s - self.stats.wait_s
        return self.stats
