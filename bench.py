#!/usr/bin/env python3
"""Benchmark of the Chunky Bits hot path on MI355X (BASELINE.json metric).

A "step" is one pass of the hot path over one batch: for every part, RS(10,4) encode_sep of
the parity chunks plus SHA-256 of all d+p chunks (FilePart::write_with_encoder's compute,
reference src/file/file_part.rs:150-185), over BASELINE.json configs[1]'s shape: 4096 parts x
10 data chunks x 1 MiB on each GPU, inputs already resident in HBM.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4]

For N > 1 one rank runs per GPU under torch.distributed.run: the driver's launcher, or, when
`--gpus N` is given with no WORLD_SIZE in the environment, this script starts it itself as a child
process (launch_ranks; a world size other than --gpus is an error, exit 2).  Each rank owns its
own 4096 parts (parts are independent: weak scaling, no collective on the data path); the
process group carries only the barrier, the max-over-ranks step time and the per-rank rows, whose
`check_vs_oracle` (each rank's own sampled parts vs the oracle) is ANDed into the line's.

Rank 0 prints ONE JSON line.  `roofline` describes the dominant kernel, timed with HIP events
on the stream its launches go to; `cpu_baseline` times the CPU restatement of the reference
crates (oracle/, the same scalar galois_8 table path + SHA-256 with SHA-NI like sha2 0.9.9's
cpufeatures dispatch) on this host's cores over a bounded sample of the same workload.

The default (c2) line also carries: `north_star` (RS(10,4) encode and 2-erasure reconstruct_data
on the headline's buffer, fractions of 8 TB/s), `baseline_configs` (BASELINE configs[2] C3 and
configs[3] C4 per GPU), `end_to_end` (host-produced write stream, read + repair stream with
damaged fetches retried, the PCIe link alone, the one-process scheduler path), and at N = 1
`check_vs_oracle` (every part of the C2 and C4 buffers and of the end-to-end write stream
against the oracle, plus whole sampled parts of each block).  At N > 1: `ranks` (each rank's own
figures) and `node` (configs[3] and C3 at node level).  `--config c5` / `c5r` run BASELINE
configs[4]: a `--stream-gib` (1 TiB) stream fed per batch from pageable rings, written, or read
back with `--corrupt` of the fetched chunks damaged.

The oracle (oracle/) is only the checker and the CPU baseline: it is imported only in the
host-side leg that runs after every timed region (the `cpu_baseline` leg: `check_vs_oracle`, the
`--check` comparisons of any config, and the timed CPU baseline), never inside a timed region
and never on the product path.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "chunky-bits_amd"))

import torch  # noqa: E402  (import before chunky_ec: one HIP runtime)
import torch.distributed as dist  # noqa: E402

import chunky_ec as ce  # noqa: E402
from chunky_ec.readstream import ReadRepairStream  # noqa: E402
from chunky_ec.sharding import (all_ranks_ok, barrier, cpu_quota, dist_env,  # noqa: E402
                                gather_rows, max_over_ranks, multi_copy_threads, part_range,
                                quota_share, rank_seed, rank_threads)

METRIC = "RS(10,4) encode+sha256 GB/s per node at 1/2/4/8 GPUs; % of HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md).  The encode kernel streams
# 6.37 TB/s (0.796 of it), at the guide's measured 6.29 TB/s copy ceiling
MiB = 1 << 20
# slots in flight of the stream configs' pipelines (4 measured best of 2-8)
STREAM_DEPTH = 4

# VALU roofline of SHA-256 (the bound of every hashed config).  Per 64-byte block one lane issues
# 1406 VALU instructions (gfx950 ISA of the SHA loop: 576 v_alignbit, 241 v_add3, 16 v_perm
# half-rate; 352 v_bitop3, 121 v_add, 96 v_lshrrev full-rate).  Measured SIMD cost per wave64
# instruction with the SIMD saturated (tools/ubench_valu.hip): half-rate 4.45
# cycles, full-rate 2.34.  Peak = 1024 SIMDs x 2.4 GHz / (mix-weighted cycles per instruction).
SHA_VALU_PER_BLOCK = 1406
SHA_HALF, SHA_FULL = 833, 573
SHA_SIMD_CYCLES = (SHA_HALF * 4.45 + SHA_FULL * 2.34) / SHA_VALU_PER_BLOCK
MI355X_SIMDS, MI355X_CLOCK_GHZ = 1024, 2.4

CONFIGS = {
    # BASELINE.json configs[1]: the metric's workload.
    "c2": dict(d=10, p=4, chunk=1 * MiB, parts=4096, op="encode_hash",
               workload="C2: batched RS(10,4) encode_sep + SHA-256 of all 14 chunks per part, "
                        "{parts} parts x {chunk} chunks per GPU"),
    # configs[2]: reconstruct, 1-4 random erasures per part (data + parity rebuilt).
    "c3": dict(d=10, p=4, chunk=1 * MiB, parts=4096, op="reconstruct",
               workload="C3: RS(10,4) reconstruct, 1-4 random erasures per part, "
                        "{parts} parts x {chunk} chunks per GPU"),
    # north_star's reconstruct target: exactly 2 random erasures per part (of the 14), the read
    # path's reconstruct_data (file_part.rs:128) as the step, resilver's reconstruct
    # (file_part.rs:304) timed beside it.
    "c3e2": dict(d=10, p=4, chunk=1 * MiB, parts=4096, op="reconstruct_e2",
                 workload="C3 2-erasure: RS(10,4) reconstruct_data with exactly 2 random erasures "
                          "per part (reconstruct of the same parts timed beside it), {parts} parts "
                          "x {chunk} chunks per GPU"),
    # configs[3]: wide stripe with fused per-chunk hashing.
    "c4": dict(d=20, p=8, chunk=256 * 1024, parts=4096, op="encode_hash",
               workload="C4: RS(20,8) encode_sep + SHA-256 of all 28 chunks per part, "
                        "{parts} parts x {chunk} chunks per GPU"),
    # configs[4]: a host-produced stream through pinned double-buffered slots (PCIe-bound);
    # --stream-gib sets the stream size (default 1 TiB split across the ranks: strong scaling).
    "c5": dict(d=10, p=4, chunk=1 * MiB, parts=256, op="stream",
               workload="C5: {stream} synthetic object stream, RS(10,4) encode + SHA-256, {chunk} "
                        "chunks, every part copied from a pageable source ring into pinned-host "
                        "staged batches of {parts} parts inside the timed region, 4 slots in "
                        "flight"),
    # configs[4], verify/repair side: the same stream read back through FileReadBuilder /
    # read_with_context batched with its retry rule: d random chunks fetched per part from a
    # pageable ring of stored chunks, a seeded fraction of them damaged, SHA-256 verify, data
    # rebuilt, parts with a rejected chunk retried with another one (file_part.rs:92-107).
    "c5r": dict(d=10, p=4, chunk=1 * MiB, parts=256, op="read_stream",
                workload="C5 verify/repair: {stream} synthetic object stream read back, RS(10,4), "
                         "d random chunks per part fetched from a pageable ring of stored chunks "
                         "into pinned-host staged batches of {parts} parts inside the timed "
                         "region, damaged chunks rejected by SHA-256 verify and retried, "
                         "reconstruct_data, 4 slots in flight"),
    # configs[2], device-resident read: FilePart::read_with_context batched -- d random chunks
    # loaded per part (file_part.rs:86-122), SHA-256 verify + reconstruct_data of the missing data
    # chunks (the decode runs speculatively beside the verification).
    "c3r": dict(d=10, p=4, chunk=1 * MiB, parts=4096, op="read",
                workload="C3 read: RS(10,4) read_with_context batched, d random chunks loaded per "
                         "part, SHA-256 verify + reconstruct_data, {parts} parts x {chunk} chunks "
                         "per GPU"),
    # encode only (HBM roofline of the GF kernel alone).
    "c2enc": dict(d=10, p=4, chunk=1 * MiB, parts=4096, op="encode",
                  workload="RS(10,4) encode_sep only, {parts} parts x {chunk} chunks per GPU"),
    # the reference's example clusters' shape (RS(3,2), examples/*.yaml) as a device batch.
    "c1enc": dict(d=3, p=2, chunk=1 * MiB, parts=8192, op="encode",
                  workload="RS(3,2) encode_sep only, {parts} parts x {chunk} chunks per GPU"),
    # the C4 shape's encode alone (RS(20,8), 256 KiB chunks).
    "c4enc": dict(d=20, p=8, chunk=256 * 1024, parts=4096, op="encode",
                  workload="RS(20,8) encode_sep only, {parts} parts x {chunk} chunks per GPU"),
}


def size_label(nbytes: float) -> str:
    for unit, k in (("TiB", 1 << 40), ("GiB", 1 << 30), ("MiB", 1 << 20), ("KiB", 1 << 10)):
        if nbytes >= k:
            v = nbytes / k
            return f"{v:g} {unit}" if v == int(v) else f"{v:.3g} {unit}"
    return f"{int(nbytes)} B"


def workload(cfg, args, stream_bytes=None, shards=None) -> str:
    """The config's workload text with the sizes this run actually used."""
    text = cfg["workload"].format(parts=cfg["parts"], chunk=size_label(cfg["chunk"]),
                                  stream=size_label(stream_bytes or 0))
    if shards:
        text += f"; one process, {shards} shard(s) over devices {args.devices}"
    return text


# bench kernel name -> rocprofv3 symbol(s); a step of concurrent kernels sums their traffic
KERNEL_SYMBOL = {"sha256_kernel": "sha256_lane_kernel", "rs_apply_kernel": "rs_apply_kernel",
                 "rs_encode_bs_kernel": "rs_encode_bs_kernel",
                 "rs_apply_kernel(reconstruct)": "rs_apply_var_kernel",
                 "rs_apply_kernel(reconstruct_data)": "rs_apply_var_kernel",
                 "encode_hash_kernel": "encode_hash_kernel",
                 "read_batch(verify+decode)": ("sha256_lane_kernel", "rs_apply_var_kernel")}


# Shapes with a compiled bit-sliced encoder (rs_kernels.hip with_bs_shape / launch_rs_encode).
BS_SHAPES = {(3, 2), (10, 4), (20, 8)}


def encode_kernel(d: int, p: int) -> str:
    """The kernel cec_encode_batch launches for RS(d, p) at a 16-byte aligned layout."""
    bs = (d, p) in BS_SHAPES and os.environ.get("CEC_APPLY_BS", "1")[:1] != "0"
    return "rs_encode_bs_kernel" if bs else "rs_apply_kernel"


def measured_traffic(config: str, kernel: str, full_size: bool, with_source: bool = False):
    """HBM bytes per launch of `kernel` from the committed PMC runs (profiles/traffic.json,
    written by profiles/summarize.py from separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes
    with the gfx950 x2 FETCH_SIZE correction), or None when this workload was not profiled.
    with_source: (bytes, "the summary file it comes from") -- a committed measurement of the
    same kernel and workload, not a measurement of this run."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    none = (None, None) if with_source else None
    if not full_size or not os.path.exists(path):
        return none
    table = json.load(open(path)).get(config, {})
    syms = KERNEL_SYMBOL.get(kernel, kernel)
    entries = [table.get(k) for k in ((syms,) if isinstance(syms, str) else syms)]
    if not all(entries):
        return none
    total = sum(e["bytes_per_launch"] for e in entries)
    if not with_source:
        return total
    return total, "committed PMC run (not this run): " + ", ".join(
        sorted({e.get("source", "profiles/traffic.json") for e in entries}))


def host_info():
    """The host the run is on (diagnoses host-bound end-to-end figures and stragglers)."""
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    nodes = [n for n in os.listdir("/sys/devices/system/node") if n.startswith("node")] \
        if os.path.isdir("/sys/devices/system/node") else []
    mem = None
    try:
        for line in open("/proc/meminfo"):
            if line.startswith("MemTotal"):
                mem = round(int(line.split()[1]) / (1 << 20), 1)
    except OSError:
        pass
    aff, quota = cpu_quota()
    return {"cpu": model, "logical_cpus": os.cpu_count(), "affinity_cpus": aff,
            "cgroup_cpu_quota": quota, "numa_nodes": len(nodes), "mem_gib": mem,
            # provenance: the loaded library's source hash and whether it equals the hash of the
            # sources shipped with this tree (chunky_ec refuses a mismatch on import)
            "build_id": ce.BUILD_ID, "build_matches_source": ce.BUILD_MATCHES_SOURCE}


def measured_valu(config: str, kernel: str, full_size: bool):
    """VALU issue of `kernel` from the committed SQ counter runs (profiles/valu.json, written by
    profiles/summarize_shapes.py): SIMD-cycles per VALU wave-instruction and the busy fraction
    (4 x SQ_INSTS_VALU / SIMD-cycles, 4 cycles = one VALU issue of a lone wave), or None when this
    workload was not profiled."""
    path = os.path.join(ROOT, "profiles", "valu.json")
    if not full_size or not os.path.exists(path):
        return None
    e = json.load(open(path)).get(config, {}).get(KERNEL_SYMBOL.get(kernel, kernel)
                                                  if isinstance(KERNEL_SYMBOL.get(kernel, kernel), str)
                                                  else kernel)
    if not e:
        return None
    return {"simd_cycles_per_valu": e["simd_cycles_per_valu"], "valu_busy": e["valu_busy"],
            "unit": "SIMD-cycles per wave64 VALU instruction; busy = 4 x SQ_INSTS_VALU / "
                    "((GRBM_GUI_ACTIVE / 8) x 1024)",
            "source": "committed rocprofv3 SQ pass (not this run): " + e["source"]}


def cpu_baseline(cfg, threads: int, cores_total: int, cores_avail: int, quota):
    """Oracle restatement of the crate path timed on this host (rank 0, N=1 only), with the
    process's full CPU affinity (the caller restores it: the bench binds its main thread to
    GPU0's NUMA node, and the baseline's threads would inherit that mask)."""
    import oracle
    d, p, L = cfg["d"], cfg["p"], cfg["chunk"]
    hashed = cfg["op"] != "encode"
    # calibrate on a few parts, then size the sample for ~1.5 s wall on `threads` cores
    # (~10-25 s of CPU work)
    probe = max(threads, 4)
    sec = oracle.baseline_encode_sha(d, p, L, probe, 1, threads, True, hashed)
    per_part = sec / probe
    total = max(threads, int(1.5 / max(per_part, 1e-6)))
    total = min(total, 4096)
    sec = oracle.baseline_encode_sha(d, p, L, total, 2, threads, True, hashed)
    gbs = total * d * L / sec / 1e9
    # one core (SURVEY.md §8d asks for it beside the all-cores figure): ~1.5 s of work
    n1 = max(2, int(1.5 / max(per_part * threads, 1e-6)))
    sec1 = oracle.baseline_encode_sha(d, p, L, n1, 2, 1, True, hashed)
    return {
        "value": round(gbs, 3),
        "unit": "GB/s",
        "cores": threads,
        "threads": threads,
        "cores_used": min(threads, cores_avail, int(quota) if quota else cores_avail),
        "cores_avail": cores_avail,
        "cores_total": cores_total,
        "cgroup_cpu_quota": quota,
        "kind": "port",
        "sample": f"{total} parts of RS({d},{p}) x {L // 1024} KiB "
                  f"({'encode_sep + sha256 of all chunks' if hashed else 'encode_sep'}), "
                  f"{threads} threads on {cores_avail} CPUs of the process's affinity "
                  f"({cores_total} logical CPUs on the host"
                  f"{f', cgroup quota {quota} CPUs' if quota else ''}), one part per task; "
                  f"{sec:.2f} s wall; "
                  f"SHA-NI={'yes' if oracle.has_shani() else 'no'}",
        "single_core": {"value": round(n1 * d * L / sec1 / 1e9, 3), "unit": "GB/s",
                        "sample": f"{n1} parts on 1 thread; {sec1:.2f} s"},
    }


class HostCopier:
    """`threads` host threads working on part ranges (numpy releases the GIL for the copies):
    the caller's reader filling its part buffers (writer.rs:170-197 reads each part's
    d*chunk_size bytes into `data_buf`; read_with_context loads a part's chunks,
    file_part.rs:86-107)."""

    def __init__(self, threads: int):
        from concurrent.futures import ThreadPoolExecutor
        self.threads = threads
        self.pool = ThreadPoolExecutor(threads)

    def map(self, fn, n: int) -> None:
        """fn(a, b) over [0, n) split into `threads` contiguous ranges, run in parallel."""
        T = self.threads
        futs = [self.pool.submit(fn, n * i // T, n * (i + 1) // T) for i in range(T)
                if n * i // T < n * (i + 1) // T]
        for f in futs:
            f.result()

    def copy(self, dst, src) -> None:
        """dst[k] = src[k] for the leading (part) axis, split over the threads."""
        def job(a, b):
            dst[a:b] = src[a:b]
        self.map(job, len(src))

    def close(self) -> None:
        self.pool.shutdown()


def source_ring(n_parts, d, L, seed, copier):
    """A pageable [n_parts][d][L] source of distinct parts (the file the reader reads): a
    random 64 MiB block tiled with `copier`'s threads (first touch in parallel), then each
    part's first 8 bytes set to its ring index.  Not timed."""
    import numpy as np
    ring = np.empty((n_parts, d, L), np.uint8)
    blk = np.random.default_rng(seed).integers(0, 256, size=(max(1, (64 << 20) // (d * L)), d, L),
                                                dtype=np.uint8)
    for k in range(0, n_parts, len(blk)):
        m = min(len(blk), n_parts - k)
        copier.copy(ring[k:k + m], blk[:m])
    ring[:, 0, :8] = np.arange(n_parts, dtype=np.uint64).view(np.uint8).reshape(n_parts, 8)
    return ring


def part_stamps(first: int, n: int):
    """[n][8] bytes: the global part numbers [first, first + n) as little-endian u64."""
    import numpy as np
    return np.arange(first, first + n, dtype=np.uint64).view(np.uint8).reshape(n, 8)


def ring_reader(ring, copier):
    """fill(data, part, n): the reader producing parts [part, part + n) into a pinned slot --
    each part's bytes copied by `copier`'s threads from the pageable ring (part k is ring part
    k mod len(ring)), its first 8 bytes then set to its global part number, so every part of
    the stream differs."""
    R = len(ring)

    def fill(data, part, n):
        r = part % R
        m = min(n, R - r)
        copier.copy(data[:m], ring[r:r + m])
        if m < n:
            copier.copy(data[m:n], ring[:n - m])
        data[:n, 0, :8] = part_stamps(part, n)
    return fill


def ring_part_digests(ring, part: int):
    """SHA-256 of the d data chunks of stream part `part` as ring_reader produced it."""
    import hashlib
    src = ring[part % len(ring)].copy()
    src[0, :8] = part_stamps(part, 1)[0]
    return [hashlib.sha256(c.tobytes()).digest() for c in src]


def timed_write(pl, fill, first: int, n_parts: int, world: int, collect=None):
    """FileWriteBuilder::write's part loop through `pl` (cec_pipeline): parts [first, first +
    n_parts) produced by fill() into each acquired slot, then H2D, encode + SHA-256, D2H.  One
    untimed warmup batch per slot, barrier, the timed stream, drain, barrier.  With `collect`
    ([n_parts][d+p][32]) every batch's digests are copied out of its slot when the slot comes
    round again (as the reference's writer takes each part's digests for its FileReference).
    Returns (local seconds, the slot of the last batch, its part count)."""
    P, depth = pl.parts, pl.depth
    for _ in range(depth):
        slot, data = pl.acquire()
        fill(data, first, P)
        pl.submit(slot, P)
    pl.drain()
    barrier(world)
    held = {}

    def take(slot):
        if collect is not None and slot in held:
            k, m = held.pop(slot)
            collect[k - first:k - first + m] = pl.wait(slot)[1]

    t0 = time.perf_counter()
    part, end, last = first, first + n_parts, (0, 0)
    while part < end:
        slot, data = pl.acquire()
        take(slot)
        n = min(P, end - part)
        fill(data, part, n)
        pl.submit(slot, n)
        held[slot] = (part, n)
        part += n
        last = (slot, n)
    pl.drain()
    for slot in list(held):
        take(slot)
    barrier(world)
    return (time.perf_counter() - t0,) + last


def stream_check(ring, digests, d, p, threads):
    """cpu_baseline leg: every part of a ring-fed write stream that started at part 0 (part k =
    ring part k mod R with its first 8 bytes set to k, ring_reader) against the oracle's encode +
    SHA-256, lap by lap over the ring, stamped in place (the stream is over).  Returns the
    mismatched parts."""
    import numpy as np
    import oracle
    R, n = len(ring), len(digests)
    bad = []
    for k in range(0, n, R):
        m = min(R, n - k)
        ring[:m, 0, :8] = part_stamps(k, m)
        want = oracle.encode_hash_parts(d, p, ring[:m], threads)
        bad.extend(int(k + i) for i in np.nonzero((want != digests[k:k + m]).any(axis=(1, 2)))[0])
    return bad


def write_check(pl, ring, slot: int, n: int, last_part: int):
    """The size-independent check of a ring-fed write stream: the digests of every data chunk of
    the first and last part of the last batch equal SHA-256 of the bytes the reader produced."""
    _, dg = pl.wait(slot)
    ok = True
    for k in (0, n - 1):
        want = ring_part_digests(ring, last_part - (n - 1) + k)
        ok = ok and all(dg[k, j].tobytes() == want[j] for j in range(len(want)))
    return bool(ok)


def encoded_ring(codec, d, p, L, n_parts, seed, device, P=256):
    """The stored chunks the read streams fetch from: a pageable [n_parts][d+p][L] ring of
    encoded parts and their metadata digests [n_parts][d+p][32], made on the GPU P parts at a
    time (synthetic data, fused encode + SHA-256) and copied down.  Not timed."""
    import numpy as np
    t = d + p
    ring = np.empty((n_parts, t, L), np.uint8)
    dig = np.empty((n_parts, t, 32), np.uint8)
    blk = torch.empty((P, t, L), dtype=torch.uint8, device=device)
    dg = torch.empty((P, t, 32), dtype=torch.uint8, device=device)
    batch = ce.PartBatch.from_tensor(blk, L)
    for b0 in range(0, n_parts, P):
        m = min(P, n_parts - b0)
        ce.fill_synthetic(batch, d, seed + b0)
        ce.encode_hash_batch(codec, batch, dg.data_ptr())
        torch.cuda.synchronize(device)
        torch.from_numpy(ring[b0:b0 + m]).copy_(blk[:m])
        torch.from_numpy(dig[b0:b0 + m]).copy_(dg[:m])
    del blk, dg
    return ring, dig


def bench_carry():
    """CEC_READ_CARRY in the read-repair streams: a retried part's verified chunks stay on the
    device (not fetched or uploaded again); CEC_BENCH_CARRY=0 turns it off for A/B runs
    (DESIGN §4.5b)."""
    return os.environ.get("CEC_BENCH_CARRY", "1") != "0"


def read_repair_flags():
    return ce.ReadPipeline.REBUILT_ONLY | (ce.ReadPipeline.CARRY if bench_carry() else 0)


def timed_read_repair(codec, ring, ring_dig, L, P, depth, first, n_parts, world, corrupt,
                      copier, seed, n_samples=3, rp=None):
    """FileReadBuilder over parts [first, first + n_parts) with read_with_context's retries
    (chunky_ec.readstream over cec_read_pipeline, REBUILT_ONLY): each part loads d random
    chunks of its d+p, copied by `copier`'s threads from the pageable ring of stored chunks
    (stream part k is ring part k mod len(ring)) into the pinned slot; a seeded `corrupt`
    fraction of the fresh loads comes back with a flipped byte (the location served bad bytes);
    the GPU verifies every fresh chunk against the metadata digest, decodes the missing data
    chunks, and a part whose load failed verification is retried with one more chunk
    (file_part.rs:92-107), its verified chunks kept on the device (CEC_READ_CARRY: only the new
    chunk is fetched and uploaded; CEC_BENCH_CARRY=0 sends them again flagged
    CEC_PRESENT_VERIFIED).  One untimed warmup pass of `depth` batches, then the timed stream.
    Returns (local seconds, stats dict, sampled output checks)."""
    import numpy as np
    d = codec.data_shard_count()
    R = len(ring)
    if rp is None:
        rp = ce.ReadPipeline(codec, L, P, depth, read_repair_flags())
    crng = np.random.default_rng(seed)
    damaged = [0]

    def fetch(chunks, rows):
        def job(a, b):
            for k, part, flags in rows[a:b]:
                r = part % R
                for j in np.flatnonzero(flags):
                    chunks[k, j] = ring[r, j]
        copier.map(job, len(rows))
        if corrupt > 0 and rows:  # fresh reads only: a re-sent verified chunk verified already
            ks = np.fromiter((k for k, _, _ in rows), np.int64, len(rows))
            kk, jj = np.nonzero(np.stack([f for _, _, f in rows]) == 1)
            hit = crng.random(len(kk)) < corrupt
            kk, jj = ks[kk[hit]], jj[hit]
            chunks[kk, jj, crng.integers(L, size=len(kk))] ^= 0xA5
            damaged[0] += len(kk)

    checks = []
    sample_at = {first, first + n_parts // 2, first + n_parts - 1}
    retried_checked = [0]

    def on_part(slot, nb, k, part, attempts):
        # the part's d data chunks (loaded ones where they were read, rebuilt ones from the
        # D2H) must equal the stored data chunks: sampled parts plus the first retried ones
        if part in sample_at or (attempts > 1 and retried_checked[0] < n_samples):
            retried_checked[0] += attempts > 1
            checks.append({"part": int(part), "attempts": int(attempts),
                           "ok": rp.part_bytes(slot, nb, k) == ring[part % R, :d].tobytes()})

    warm = ReadRepairStream(rp, fetch, lambda ids: ring_dig[ids % R], seed=seed + 1)
    warm.run(first, min(n_parts, depth * P))
    damaged[0] = 0
    barrier(world)
    t0 = time.perf_counter()
    st = ReadRepairStream(rp, fetch, lambda ids: ring_dig[ids % R], seed=seed + 2,
                          on_part=on_part).run(first, n_parts)
    barrier(world)
    el = time.perf_counter() - t0
    del rp
    stats = st.as_dict()
    stats["damaged_loads"] = damaged[0]
    return el, stats, checks


def _stream_line(args, cfg, world, n_batches, warm, el, total, extra_config, data_text, **extra):
    d, p, L, P = cfg["d"], cfg["p"], cfg["chunk"], cfg["parts"]
    line = {
        "metric": f"{METRIC} [{args.config}]",
        "value": round(total / el / 1e9, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": n_batches,
        "warmup": warm,
        "ms_per_step": round(el / max(n_batches, 1) * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u8",
        "data": data_text,
        "config": dict({"workload": workload(cfg, args, total, extra_config.pop("shards", None)),
                        "d": d, "p": p, "chunk_bytes": L, "parts_per_batch": P,
                        "stream_bytes": total}, **extra_config),
        "seconds": round(el, 3),
    }
    line.update(extra)
    return line


def run_stream(args, cfg, codec, world, rank, device, reduce_dev):
    """C5 (BASELINE configs[4], write side): a `--stream-gib` object stream, split into
    contiguous part ranges over the ranks (strong scaling), each rank's parts produced inside
    the timed region by host threads copying from a pageable source ring into the pinned slots
    (ring_reader), then H2D -> fused encode + SHA-256 -> D2H of parity + digests (cec_pipeline,
    `depth` slots).  Time = first submit to last result, max over ranks."""
    d, p, L, P = cfg["d"], cfg["p"], cfg["chunk"], cfg["parts"]
    depth = STREAM_DEPTH
    total_parts = int(args.stream_gib * (1 << 30)) // (d * L)
    lo, hi = part_range(total_parts, rank, world)
    if args.devices:
        return run_stream_multi(args, cfg, codec, total_parts)
    threads = rank_threads(world)
    copier = HostCopier(threads)
    ring_parts = 2 * depth * P if world == 1 else 2 * P
    ring = source_ring(ring_parts, d, L, 0xC5 + rank, copier)
    pl = ce.Pipeline(codec, L, P, depth)
    # --check at N = 1: every part's digests kept (47 MB per TiB) and, after the timed region,
    # every part re-derived from the ring through the oracle (stream_check; ~100 s per TiB on 16
    # CPU workers)
    import numpy as np
    collect = np.empty((hi - lo, d + p, 32), np.uint8) if args.check and world == 1 else None
    loc, slot, n = timed_write(pl, ring_reader(ring, copier), lo, hi - lo, world, collect)
    ok = write_check(pl, ring, slot, n, hi - 1) if hi > lo else True
    ok = all_ranks_ok(ok, world, reduce_dev)
    el = max_over_ranks(loc, world, reduce_dev)
    del pl
    copier.close()
    whole = None
    if collect is not None:
        t0 = time.perf_counter()
        bad = stream_check(ring, collect, d, p, min(16, len(os.sched_getaffinity(0))))
        whole = {"parts": len(collect), "digests": int(collect.size // 32),
                 "mismatched": bad[:8], "ok": not bad,
                 "seconds": round(time.perf_counter() - t0, 1)}
    if rank == 0:
        total = total_parts * d * L
        print(json.dumps(_stream_line(
            args, cfg, world, (hi - lo + P - 1) // P, depth, el, total,
            {"slots": depth, "host_threads": threads,
             "parallelism": f"part-range-sharded x{world}, no collective"},
            f"synthetic host stream: every part copied inside the timed region by {threads} host "
            f"threads from a pageable source ring ({ring_parts} distinct parts, "
            f"{size_label(ring.nbytes)}) into the pinned slot, global part number stamped",
            check_digests_vs_source=ok,
            **({"check_all_parts_vs_oracle": whole} if whole is not None else {}))),
            flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


def run_read_stream(args, cfg, codec, world, rank, device, reduce_dev):
    """C5 (BASELINE configs[4], verify/repair side): the stream read back through
    FileReadBuilder / read_with_context batched with retries (timed_read_repair): d random
    chunks per part fetched inside the timed region from a pageable ring of stored chunks, a
    seeded --corrupt fraction of the fetched chunks damaged, every fetched chunk SHA-256-verified
    on the GPU, missing data rebuilt, failed parts retried with another chunk.  Contiguous part
    ranges over the ranks (strong scaling); value = part data bytes delivered / s, max over
    ranks."""
    d, p, L, P = cfg["d"], cfg["p"], cfg["chunk"], cfg["parts"]
    depth = STREAM_DEPTH
    total_parts = int(args.stream_gib * (1 << 30)) // (d * L)
    lo, hi = part_range(total_parts, rank, world)
    threads = rank_threads(world)
    copier = HostCopier(threads)
    ring, ring_dig = encoded_ring(codec, d, p, L, 2 * P, rank_seed(0xC5C5, rank), device, P)
    loc, stats, checks = timed_read_repair(codec, ring, ring_dig, L, P, depth, lo, hi - lo,
                                           world, args.corrupt, copier, 0x5EED + rank)
    ok = all(c["ok"] for c in checks) and stats["undecodable_parts"] == 0
    ok = all_ranks_ok(ok, world, reduce_dev)
    el = max_over_ranks(loc, world, reduce_dev)
    copier.close()
    if rank == 0:
        total = total_parts * d * L
        print(json.dumps(_stream_line(
            args, cfg, world, stats["batches"], depth, el, total,
            {"slots": depth, "host_threads": threads, "corrupt_frac": args.corrupt,
             "parallelism": f"part-range-sharded x{world}, no collective"},
            f"synthetic stored chunks: a pageable ring of {len(ring)} GPU-encoded parts "
            f"({size_label(ring.nbytes)}); d random chunks per part copied inside the timed "
            f"region by {threads} host threads into the pinned slot, {args.corrupt:g} of the "
            "fetched chunks damaged (seeded), failed parts retried"
            + (" (their verified chunks kept on the device, CEC_READ_CARRY)"
               if bench_carry() else ""),
            read_repair=stats, check_vs_stored=ok, checks=checks)), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


def end_to_end(codec, d, p, L, gib, world, rank, reduce_dev, host_threads, device_ordinal,
               device, corrupt, full_check=False):
    """North-star's PCIe-bound end-to-end figures beside the device-resident headline: the same
    RS(10,4) encode + SHA-256 with the parts produced in host memory, parity + digests landing
    back in it, `gib` GiB per rank (weak scaling like the headline), max over ranks.  Not
    `value` (that is HBM-resident).  Each form is timed on its own:

    value (`reader_to_pinned`): every batch's part bytes are copied, inside the timed region, by
      `host_threads` threads from a pageable source ring (2x the slots' bytes, so every copy
      reads DRAM) into the pinned slot -- the reference's reader filling `data_buf`
      (writer.rs:170-197) when `data_buf` is the engine's page-locked slot -- then H2D, the
      fused kernel (or, for these 256-part batches, encode + split SHA), D2H (cec_pipeline,
      256-part batches, 4 slots in flight);
    `read_repair`: the read side of the same stream (timed_read_repair): d random chunks per
      part fetched from a pageable ring of stored chunks, `corrupt` of them damaged, verified on
      the GPU, missing data rebuilt, failed parts retried with another chunk;
    `scheduler_pageable`: the `cp` path of a single process -- the same pageable ring handed to
      the multi-GPU scheduler (cec_multi, one shard on this rank's GPU), whose own NUMA-local
      copy threads stage it;
    `pcie_link`: the slots filled once and re-sent (8 bytes per part stamped): the link alone,
      no host production (round 2's figure)."""
    P, depth = CONFIGS["c5"]["parts"], 4
    n_parts = max(depth * P, int(gib * (1 << 30)) // (d * L))
    # 2x the slots' part count at N = 1 (20 GiB); at N > 1 every rank of the node holds its own
    # ring, slots and scheduler staging at once, so the ring shrinks to 2 batches (5 GiB, still
    # 20x a socket's L3: every copy reads DRAM) to keep the node's host memory near 20 GiB per GPU
    ring_parts = 2 * depth * P if world == 1 else 2 * P
    # ~14 GiB page-locked slots + the pageable ring per rank: if any rank cannot get them,
    # every rank skips the figure together (no rank may be left waiting in a barrier) and the
    # headline still prints
    copier = HostCopier(host_threads)
    try:
        pl, err = ce.Pipeline(codec, L, P, depth), None
        ring = source_ring(ring_parts, d, L, 0xE2E + rank, copier)
    except Exception as e:  # noqa: BLE001 (reported in the line)
        pl, ring, err = None, None, f"{type(e).__name__}: {e}"
    if not all_ranks_ok(pl is not None, world, reduce_dev):
        del pl, ring
        copier.close()
        return {"value": None, "unit": "GB/s", "bound": "pcie",
                "skipped": err or "another rank could not allocate its slots / source ring"}

    def stamp_only(data, part, n):
        data[:n, 0, :8] = part_stamps(part, n)

    import numpy as np
    collect = np.empty((n_parts, d + p, 32), np.uint8) if full_check else None
    loc_ring, slot, n = timed_write(pl, ring_reader(ring, copier), 0, n_parts, world, collect)
    el_ring = max_over_ranks(loc_ring, world, reduce_dev)
    # the ring-fed batches are checked for the property that holds at any size: the digests of
    # the data chunks equal SHA-256 of the bytes the reader produced (sampled)
    ring_ok = write_check(pl, ring, slot, n, n_parts - 1)
    loc_link = timed_write(pl, stamp_only, 0, n_parts, world)[0]
    el_link = max_over_ranks(loc_link, world, reduce_dev)
    del pl
    total = n_parts * d * L * world
    mine = n_parts * d * L
    res = {
        # this rank's own rates (the N > 1 line's `ranks` array; removed before printing)
        "_local": (mine / loc_ring / 1e9, mine / loc_link / 1e9),
        "value": round(total / el_ring / 1e9, 2), "unit": "GB/s", "bound": "pcie + host copy",
        "form": "reader_to_pinned",
        "stream_bytes": total, "seconds": round(el_ring, 3),
        "host_threads": host_threads,
        "host_copy_GBs": round(total / el_ring / 1e9, 2),
        # host DRAM traffic of the form: the copy reads the ring and writes the slot, the H2D
        # reads the slot, the D2H writes parity (p/d of the data) + 32-B digests per chunk
        "host_dram_GBs": round(total * (3 + p / d) / el_ring / 1e9, 1),
        "sampled_digest_matches_source": ring_ok,
        "path": f"pageable source ring ({ring_parts} distinct parts, {size_label(ring.nbytes)}) "
                f"-> {host_threads} host threads copy each batch into a page-locked slot -> H2D "
                f"-> encode + SHA-256 -> D2H parity + digests (cec_pipeline, {P}-part batches, "
                f"{depth} slots), {gib:g} GiB per GPU",
        "pcie_link": {
            "value": round(total / el_link / 1e9, 2), "unit": "GB/s", "seconds": round(el_link, 3),
            "path": "the same pipeline with its slots filled ONCE and re-sent (8 bytes per part "
                    "stamped): the PCIe link with no host production"},
    }
    # the scheduler's pageable path (what `cp` through the C++ FileWriteBuilder batch takes)
    res["scheduler_pageable"] = scheduler_pageable(codec, d, p, L, ring, n_parts, world,
                                                   reduce_dev, device_ordinal)
    if collect is not None:  # every part's digests, checked in the cpu_baseline leg
        res["_stream"] = (ring, collect)
    del ring
    res["read_repair"] = read_repair_form(codec, d, p, L, n_parts, world, rank, reduce_dev,
                                          copier, device, corrupt)
    copier.close()
    return res


def read_repair_form(codec, d, p, L, n_parts, world, rank, reduce_dev, copier, device, corrupt):
    """end_to_end's read side: n_parts per rank through timed_read_repair (2 batches of stored
    parts in the ring: 7 GiB, every fetch reads DRAM)."""
    P, depth = CONFIGS["c5r"]["parts"], 4
    # allocations first (the ring of stored parts, ~24 GiB of page-locked slots): if any rank
    # cannot get them every rank skips the form together, before any barrier of the stream
    try:
        ring, ring_dig = encoded_ring(codec, d, p, L, 2 * P, rank_seed(0xE2ED, rank), device, P)
        rp, err = ce.ReadPipeline(codec, L, P, depth, read_repair_flags()), None
    except Exception as e:  # noqa: BLE001 (reported in the line)
        ring, rp, err = None, None, f"{type(e).__name__}: {e}"
    if not all_ranks_ok(err is None, world, reduce_dev):
        return {"value": None, "unit": "GB/s",
                "skipped": err or "another rank could not allocate its read stream"}
    loc, stats, checks = timed_read_repair(codec, ring, ring_dig, L, P, depth, 0, n_parts, world,
                                           corrupt, copier, 0xE2E5 + rank, rp=rp)
    del rp
    el = max_over_ranks(loc, world, reduce_dev)
    total = n_parts * d * L * world
    ok = all(c["ok"] for c in checks) and stats["undecodable_parts"] == 0
    return {"value": round(total / el / 1e9, 2), "unit": "GB/s of part data delivered",
            "_local": n_parts * d * L / loc / 1e9,
            "seconds": round(el, 3), "stream_bytes": total, "corrupt_frac": corrupt,
            "retries": stats["retried_parts"], "retry_batches": stats["retry_batches"],
            "mixed_batches": stats["mixed_batches"],
            "rejected_chunks": stats["rejected_chunks"], "damaged_loads": stats["damaged_loads"],
            "undecodable_parts": stats["undecodable_parts"], "batches": stats["batches"],
            "chunks_loaded": stats["chunks_loaded"],
            "sampled_parts_equal_stored": ok, "checks": checks,
            "path": f"pageable ring of {len(ring)} stored parts ({size_label(ring.nbytes)}) -> "
                    f"{copier.threads} host threads copy d random chunks per part into a "
                    "page-locked slot, a seeded fraction of them damaged -> H2D -> SHA-256 "
                    "verify + reconstruct_data -> D2H of the rebuilt data chunks; parts with a "
                    "rejected chunk resubmitted in the next batch, ahead of its new parts, with "
                    + ("their verified chunks kept on the device (CEC_READ_CARRY) "
                       if bench_carry() else "their verified chunks (CEC_PRESENT_VERIFIED) ")
                    + f"and one more (cec_read_pipeline, {P}-part batches, {depth} slots)",
            "carried_chunks": stats["carried_chunks"],
            "loop_seconds": {"fetch": stats["fetch_s"], "wait": stats["wait_s"],
                             "rest": stats["loop_s"]}}


def scheduler_pageable(codec, d, p, L, ring, n_parts, world, reduce_dev, device_ordinal):
    """cec_multi with one shard on this rank's GPU, fed the pageable ring (two 512-part jobs in
    flight; the scheduler's own copy threads stage the bytes), page-locked parity / digest
    outputs.  Every rank streams its own n_parts."""
    P, depth = CONFIGS["c5"]["parts"], 4
    t = d + p
    ring_parts = len(ring)
    S, J = 2 * P, 2
    # every rank must reach the barriers below, or none: a rank that cannot build its scheduler
    # makes every rank skip this form together
    try:
        m, err = ce.Multi(codec, L, P, depth, [device_ordinal], kinds=ce.Multi.WRITE), None
        outs = [(ce.HostBuffer(S * p * L, device_ordinal),
                 ce.HostBuffer(S * t * 32, device_ordinal)) for _ in range(J)]
    except Exception as e:  # noqa: BLE001 (reported in the line)
        m, outs, err = None, None, f"{type(e).__name__}: {e}"
    if not all_ranks_ok(err is None, world, reduce_dev):
        del m, outs
        return {"value": None, "unit": "GB/s",
                "skipped": err or "another rank could not build its scheduler"}

    def submit(i, first):
        par, dig = outs[i % J]
        n = min(S, n_parts - first)
        r = first % ring_parts
        n = min(n, ring_parts - r)  # a job never wraps the ring
        return m.encode_hash(ring[r:r + n], n, par, dig), n

    for i in range(J):  # warmup: pins the shard's staging on its first pageable job
        m.wait(submit(i, i * S)[0])
    barrier(world)
    t0 = time.perf_counter()
    jobs, first, i = [], 0, 0
    while first < n_parts:
        if len(jobs) == J:
            m.wait(jobs.pop(0))
        job, n = submit(i, first)
        jobs.append(job)
        first += n
        i += 1
    for job in jobs:
        m.wait(job)
    barrier(world)
    el = max_over_ranks(time.perf_counter() - t0, world, reduce_dev)
    total = n_parts * d * L * world
    copy_threads = int(os.environ.get("CEC_MULTI_COPY_THREADS", "4"))
    del m, outs
    return {"value": round(total / el / 1e9, 2), "unit": "GB/s", "seconds": round(el, 3),
            "copy_threads": copy_threads,
            "path": f"pageable source ring -> cec_multi (1 shard on device {device_ordinal}, its "
                    f"{copy_threads} NUMA-local copy threads stage into page-locked slots) -> "
                    f"H2D -> encode + SHA-256 -> D2H into page-locked outputs; {S}-part jobs, "
                    f"{J} in flight"}


def snapshot_parts(buf, digests, parts):
    """Host copies of whole parts (every chunk) of a device batch, and their digests: the
    default line's full-size buffers, checked against the oracle after the timed work."""
    return [(int(k), buf[k].cpu().numpy(), None if digests is None else digests[k].cpu().numpy())
            for k in parts]


def batch_vs_oracle(dev, digests, d, p, threads, slab=256):
    """cpu_baseline leg: every part of a device batch ([n][d+p][L], torch tensor; copied down
    slab by slab) against the oracle: encode_sep of its data chunks must equal its parity chunks,
    and SHA-256 of all d+p chunks must equal `digests` ([n][d+p][32], host).  Returns the
    mismatched parts."""
    import numpy as np
    import oracle
    bad = []
    for k in range(0, dev.shape[0], slab):
        host = dev[k:k + slab].cpu().numpy()
        want, par_ok = oracle.encode_hash_parts(d, p, host, threads, check_parity=True)
        diff = (want != digests[k:k + slab]).any(axis=(1, 2)) | ~par_ok
        bad.extend(int(k + i) for i in np.nonzero(diff)[0])
    return bad


def check_vs_oracle(snap, d, p, threads=16):
    """cpu_baseline leg: the sampled parts of the default line's own buffers against the CPU
    restatement of the reference crates (oracle.encode_sep, the galois_8 table path) and
    hashlib SHA-256:
      headline        -- the fused encode_hash_kernel's parity and all d+p digests (C2);
      north_star      -- the parity the north_star encode (bit-sliced kernel) rewrote;
      c3_reconstruct  -- every chunk after C3's 1-4 erasures were rebuilt (data + parity);
      c4_encode_hash  -- RS(20,8) parity + 28 digests of the fused kernel (C4's buffer);
      c4_round_trip   -- the same C4 parts after 8 erasures and reconstruct;
      c2_all_parts    -- every part of the C2 buffer as the device-resident blocks left it
                         (the fused encode, north_star's re-encode and 2-erasure rebuild, C3's
                         re-encode and 1-4-erasure rebuild of data + parity): its parity equals
                         the oracle's encode_sep of its data, and SHA-256 of its 14 chunks the
                         digests the fused kernel produced (oracle.encode_hash_parts, `threads`
                         CPU workers, streamed down slab by slab: batch_vs_oracle);
      c4_all_parts    -- the same for C4's RS(20,8) buffer after its fused encode and 8-erasure
                         round trip."""
    import hashlib

    import numpy as np
    import oracle
    res = {}

    def parity_ok(part, dd, pp):
        st, par = oracle.encode_sep(dd, pp, [part[j] for j in range(dd)])
        return st == 0 and all(np.array_equal(par[i], part[dd + i]) for i in range(pp))

    def digests_ok(part, dg):
        return all(hashlib.sha256(part[i].tobytes()).digest() == dg[i].tobytes()
                   for i in range(len(part)))

    head = {k: part for k, part, _ in snap["headline"]}
    res["headline"] = all(parity_ok(part, d, p) and digests_ok(part, dg)
                          for _, part, dg in snap["headline"])
    if "north_star_encode" in snap:
        res["north_star_encode"] = all(np.array_equal(part[d:], head[k][d:]) and
                                       parity_ok(part, d, p)
                                       for k, part, _ in snap["north_star_encode"])
    if "c3_reconstruct" in snap:
        res["c3_reconstruct"] = all(np.array_equal(part, head[k]) and parity_ok(part, d, p)
                                    for k, part, _ in snap["c3_reconstruct"])
    if "c4_encode_hash" in snap:
        c4 = CONFIGS["c4"]
        d4, p4 = c4["d"], c4["p"]
        first = {k: part for k, part, _ in snap["c4_encode_hash"]}
        res["c4_encode_hash"] = all(parity_ok(part, d4, p4) and digests_ok(part, dg)
                                    for _, part, dg in snap["c4_encode_hash"])
        if "c4_round_trip" in snap:
            res["c4_round_trip"] = all(np.array_equal(part, first[k])
                                       for k, part, _ in snap["c4_round_trip"])
    extra = {}

    def whole_batch(key, dd, pp, dev, digests):
        bad = batch_vs_oracle(dev, digests, dd, pp, threads)
        res[f"{key}_all_parts"] = not bad
        extra[f"{key}_all_parts_checked"] = {"parts": int(digests.shape[0]),
                                             "digests": int(digests.shape[0] * digests.shape[1])}
        extra[f"{key}_all_parts_mismatched"] = bad[:8]

    if "c2_dev" in snap:
        whole_batch("c2", d, p, snap["c2_dev"], snap["c2_digests"])
    if "c4_dev" in snap:
        c4 = CONFIGS["c4"]
        whole_batch("c4", c4["d"], c4["p"], snap["c4_dev"], snap["c4_digests"])
    return {"ok": all(res.values()), "checks": res, "parts": list(snap["parts"]), **extra,
            "erased_in_c3": {str(k): v for k, v in snap.get("c3_erased", {}).items()},
            "basis": "whole parts (all chunks) copied from the buffers that produced value, "
                     "north_star and baseline_configs, compared with oracle.encode_sep (CPU "
                     "restatement of reed-solomon-erasure 4.0.2 galois_8) and hashlib SHA-256"}


def two_erasures(n_parts: int, t: int, rank: int):
    """north_star's reconstruct case: exactly 2 erasures per part, uniform over the t chunks
    (seeded, the c3e2 config's sets).  Returns the present mask as a uint8 [n][t] tensor."""
    g = torch.Generator().manual_seed(2222 + rank)
    pres = torch.ones((n_parts, t), dtype=torch.uint8)
    for i in range(n_parts):
        pres[i, torch.randperm(t, generator=g)[:2]] = 0
    return pres


def reconstruct_data_bytes(pres, d: int, L: int) -> int:
    """Algorithmic bytes of reconstruct_data over `pres`: parts with a missing data chunk read d
    chunks and write the missing data ones; parts missing only parity are skipped (the crate
    returns early)."""
    miss = d - pres[:, :d].sum(1)
    return int((miss > 0).sum().item()) * d * L + int(miss.sum().item()) * L


def north_star_block(codec, batch, buf, digests, stream, device, rank, d, p, L, steps,
                     snap=None):
    """north_star's two numeric targets, timed on the headline's own buffer right after it:
    RS(10,4) encode (file_part.rs:161-165) and 2-erasure reconstruct_data (file_part.rs:128)
    over every part, each launch bracketed by HIP events on `stream` (1 warmup launch, then
    `steps`), as a fraction of the 8 TB/s HBM peak.  After the rebuild, every data chunk is
    verified on the GPU against the digest the headline computed for it."""
    n = batch.n_parts
    t = d + p
    out = {}

    def time_launches(fn):
        fn()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(steps)]
        for a, b in evs:
            a.record(stream)
            fn()
            b.record(stream)
        torch.cuda.synchronize(device)
        return sum(a.elapsed_time(b) for a, b in evs) / steps

    def entry(call, kernel, ms, algo, cfgkey):
        gbs = algo / (ms / 1e3) / 1e9
        # this command's own PMC run (the c2 entries: profiles/summarize_shapes.py keeps the
        # full-size launch of each kernel), else the kernel's own config
        full = n == CONFIGS["c2"]["parts"]  # the profiled workload; else no committed figure
        tr, src = measured_traffic("c2", kernel, full, with_source=True)
        if tr is None:
            tr, src = measured_traffic(cfgkey, kernel, full, with_source=True)
        return {"call": call, "kernel": kernel, "ms": round(ms, 4), "algorithmic_bytes": algo,
                "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(gbs / HBM_PEAK_GBS, 4), "target_frac": 0.60,
                "meets_target": gbs / HBM_PEAK_GBS >= 0.60,
                "traffic": tr, "traffic_source": src}

    ms = time_launches(lambda: ce.encode_batch(codec, batch, stream))
    out["encode"] = entry("encode_sep (cec_encode_batch), every part: read d, write p chunks",
                          encode_kernel(d, p), ms, n * t * L, "c2enc")
    if snap is not None:  # the parity this encode kernel wrote, for the oracle check
        snap["north_star_encode"] = snapshot_parts(buf, None, snap["parts"])
    pres = two_erasures(n, t, rank)
    present = bytes(pres.flatten().tolist())
    buf.mul_(pres.to(device).view(n, t, 1))  # the erased chunks start zeroed
    ms = time_launches(lambda: ce.reconstruct_batch(codec, batch, present, True, stream))
    out["reconstruct_data_2_erasures"] = entry(
        "reconstruct_data (cec_reconstruct_batch, data_only), exactly 2 random erasures of the "
        f"{t} chunks per part (c3e2's sets): parts with a missing data chunk read d, write the "
        "missing data chunks", "rs_apply_var_kernel", ms, reconstruct_data_bytes(pres, d, L),
        "c3e2")
    # size-independent check: every rebuilt (and every untouched) data chunk hashes to the
    # digest the headline step computed before the erasure
    exp = digests[:, :d].contiguous()
    ok = torch.zeros((n, d), dtype=torch.uint8, device=device)
    ce.verify_batch(batch, 0, d, exp.data_ptr(), ok.data_ptr(), stream=stream)
    torch.cuda.synchronize(device)
    out["rebuilt_data_verified"] = bool(ok.all().item())
    out["basis"] = ("HIP events on the launch stream, average of the timed launches; algorithmic "
                    "bytes per SURVEY.md §8d (encode (d+p)·L per part, reconstruct_data (d+k)·L per "
                    "part with a missing data chunk); traffic = committed PMC bytes per launch of "
                    "the same kernel on the same workload (traffic_source), not measured in this "
                    "run")
    return out


def c3_erasures(n_parts: int, t: int, p: int, rank: int):
    """The c3 config's erasure sets: 1..p random erasures per part (seeded)."""
    g = torch.Generator().manual_seed(1234 + rank)
    pres = torch.ones((n_parts, t), dtype=torch.uint8)
    k = torch.randint(1, p + 1, (n_parts,), generator=g)
    for i in range(n_parts):
        pres[i, torch.randperm(t, generator=g)[: int(k[i])]] = 0
    return pres


def baseline_configs_block(codec, batch, buf, digests, stream, device, rank, d, p, L, steps,
                           snap=None):
    """BASELINE.json's other device-resident configurations in the default line, so the driver's
    run observes them too: configs[2] (C3: RS(10,4) reconstruct with 1-4 random erasures per
    part, data + parity, file_part.rs:304) on the headline's buffer, and configs[3] (C4: RS(20,8),
    4 096 parts x 256 KiB, fused encode + SHA-256 of all 28 chunks) on a buffer of its own.
    Each is checked size-independently on the GPU: after the rebuild every chunk (C3) / after an
    erase-and-rebuild round trip every chunk (C4) hashes to the digest its encode step computed."""
    n, t = batch.n_parts, d + p
    out = {}

    def timed(fn):
        fn()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(steps)]
        for a, b in evs:
            a.record(stream)
            fn()
            b.record(stream)
        torch.cuda.synchronize(device)
        return sum(a.elapsed_time(b) for a, b in evs) / steps

    def verified(bt, dg, nchunks, nparts):
        ok = torch.zeros((nparts, nchunks), dtype=torch.uint8, device=device)
        ce.verify_batch(bt, 0, nchunks, dg.data_ptr(), ok.data_ptr(), stream=stream)
        torch.cuda.synchronize(device)
        return bool(ok.all().item())

    # C3: restore the parity north_star's data-only rebuild left erased, then 1-4 erasures
    ce.encode_batch(codec, batch, stream)
    pres = c3_erasures(n, t, p, rank)
    present = bytes(pres.flatten().tolist())
    buf.mul_(pres.to(device).view(n, t, 1))
    ms = timed(lambda: ce.reconstruct_batch(codec, batch, present, False, stream))
    if snap is not None:  # every chunk after the rebuild (each sampled part lost 1-4 of them)
        snap["c3_reconstruct"] = snapshot_parts(buf, None, snap["parts"])
        snap["c3_erased"] = {k: [int(i) for i in (pres[k] == 0).nonzero().flatten()]
                             for k in snap["parts"]}
    touched = int((pres.sum(1) < t).sum().item())
    algo = touched * d * L + int((t - pres.sum(1)).sum().item()) * L
    gbs = algo / (ms / 1e3) / 1e9
    tr, src = measured_traffic("c3", "rs_apply_kernel(reconstruct)", n == CONFIGS["c3"]["parts"],
                               with_source=True)
    out["c3_reconstruct"] = {
        "config": "BASELINE configs[2]: RS(10,4) reconstruct (data + parity), 1-4 random erasures "
                  f"per part, {n} parts x {size_label(L)}", "kernel": "rs_apply_var_kernel",
        "ms": round(ms, 4), "algorithmic_bytes": algo, "achieved": round(gbs, 1),
        "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
        "traffic": tr, "traffic_source": src,
        "rebuilt_verified": verified(batch, digests, t, n)}

    # C4: RS(20,8) x 256 KiB, fused encode + SHA-256, then an 8-erasure round trip
    c4 = CONFIGS["c4"]
    # C4's 4096 parts at the headline's 4096; scaled with --parts (rehearsals, small tests)
    d4, p4, L4 = c4["d"], c4["p"], c4["chunk"]
    n4 = max(1, c4["parts"] * n // CONFIGS["c2"]["parts"])
    t4 = d4 + p4
    codec4 = ce.ReedSolomon(d4, p4)
    buf4 = torch.empty((n4, t4, L4), dtype=torch.uint8, device=device)
    dig4 = torch.empty((n4, t4, 32), dtype=torch.uint8, device=device)
    b4 = ce.PartBatch.from_tensor(buf4, L4)
    ce.fill_synthetic(b4, t4, rank_seed(0xC4C4, rank), stream)
    ms = timed(lambda: ce.encode_hash_batch(codec4, b4, dig4.data_ptr(), stream))
    if snap is not None:  # RS(20,8) parity + all 28 digests of the fused kernel
        snap["c4_encode_hash"] = snapshot_parts(buf4, dig4, (0, n4 - 1))
        if "c2_dev" in snap:  # and every part: the buffer stays for the cpu_baseline leg
            snap["c4_digests"] = dig4.cpu().numpy()
            snap["c4_dev"] = buf4
    data_gbs = n4 * d4 * L4 / (ms / 1e3) / 1e9
    hbm = n4 * t4 * (L4 + 32) / (ms / 1e3) / 1e9
    g = torch.Generator().manual_seed(2828 + rank)
    pres4 = torch.ones((n4, t4), dtype=torch.uint8)
    for i in range(n4):
        pres4[i, torch.randperm(t4, generator=g)[:p4]] = 0
    buf4.mul_(pres4.to(device).view(n4, t4, 1))
    ce.reconstruct_batch(codec4, b4, bytes(pres4.flatten().tolist()), False, stream)
    if snap is not None:  # the same parts after 8 erasures and reconstruct
        snap["c4_round_trip"] = snapshot_parts(buf4, None, (0, n4 - 1))
    tr, src = measured_traffic("c4", "encode_hash_kernel", n4 == c4["parts"], with_source=True)
    out["c4_encode_hash"] = {
        "config": f"BASELINE configs[3] per GPU: RS(20,8), {n4} parts x {size_label(L4)}, fused "
                  "encode + SHA-256 of all 28 chunks", "kernel": "encode_hash_kernel",
        "ms": round(ms, 4), "value": round(data_gbs, 2), "unit": "GB/s of data",
        "data_bytes": n4 * d4 * L4,
        "hbm_achieved": round(hbm, 1), "hbm_frac": round(hbm / HBM_PEAK_GBS, 4),
        "traffic": tr, "traffic_source": src,
        "round_trip_verified": verified(b4, dig4, t4, n4),
        "round_trip": "8 random erasures of 28 per part, reconstruct (data + parity), every "
                      "chunk re-hashed against the fused step's digests"}
    del buf4, dig4
    out["basis"] = ("HIP events on the launch stream, average of the timed launches after one "
                    "warmup; algorithmic bytes per SURVEY.md §8d")
    return out


def _segments(args, cfg, shards):
    """Parts per scheduler job: every shard gets 2 batches per job; --jobs-in-flight jobs are
    queued at once (the next ones queued while the first runs: no drain bubble)."""
    P = cfg["parts"]
    return 2 * P * shards


def run_stream_multi(args, cfg, codec, total_parts):
    """C5 through the single-process multi-GPU scheduler (cec_multi: one worker thread per
    shard, contiguous part ranges, NUMA-local staging): each job hands the scheduler a range of
    a pageable source ring of distinct parts (one job's worth, read cyclically); the shards' own
    copy threads stage the bytes into page-locked slots inside the timed region; parity and
    digests land in page-locked outputs.  --jobs-in-flight jobs queued at once."""
    d, p, L, P = cfg["d"], cfg["p"], cfg["chunk"], cfg["parts"]
    t = d + p
    devices = args.devices
    depth = STREAM_DEPTH
    m = ce.Multi(codec, L, P, depth, devices, kinds=ce.Multi.WRITE)
    S = _segments(args, cfg, len(devices))
    J = args.jobs_in_flight
    copier = HostCopier(rank_threads(1))
    ring = source_ring(S, d, L, 0xC5, copier)
    copier.close()
    outs = [(ce.HostBuffer(S * p * L, devices[0]), ce.HostBuffer(S * t * 32, devices[0]))
            for _ in range(J)]
    n_jobs = (total_parts + S - 1) // S

    def submit(i, first):
        par, dig = outs[i % J]
        n = min(S, total_parts - first)
        return m.encode_hash(ring[:n], n, par, dig), n

    for i in range(J):  # warmup: one job per output buffer (pipelines, staging, first pinning)
        m.wait(submit(i, 0)[0])
    t0 = time.perf_counter()
    jobs, first = [], 0
    for i in range(n_jobs):
        if len(jobs) == J:
            m.wait(jobs.pop(0))
        job, n = submit(i, first)
        jobs.append(job)
        first += n
    for job in jobs:
        m.wait(job)
    el = time.perf_counter() - t0
    total = total_parts * d * L
    per_shard = [m.shard_info(g) for g in range(len(devices))]
    print(json.dumps(_stream_line(
        args, cfg, len(set(devices)), n_jobs, J, el, total,
        {"slots": depth, "shards": len(devices), "parts_per_job": S, "jobs_in_flight": J,
         "parallelism": f"single process, {len(devices)} shard(s) on devices {devices}, contiguous "
                        "part ranges, no collective"},
        f"synthetic host stream: a pageable source ring of {S} distinct parts "
        f"({size_label(ring.nbytes)}) read cyclically, staged by the scheduler's copy threads "
        "inside the timed region",
        shards=[{"device": dv, "numa_node": nn, "parts": pp} for dv, nn, pp in per_shard])),
        flush=True)


RANK_FIELDS = ("device", "numa_node", "host_threads_numa_bound", "cpus", "step_ms",
               "end_to_end_GBs", "pcie_link_GBs", "north_star_encode_frac",
               "north_star_reconstruct_data_frac", "c3_reconstruct_frac", "c3_algorithmic_bytes",
               "c3_ms", "c4_ms", "c4_data_bytes", "read_repair_GBs", "quota_share_cpus",
               "host_threads", "multi_copy_threads", "check_vs_oracle")


def free_port() -> int:
    """A TCP port free on 127.0.0.1 now (the rendezvous port of the ranks launch_ranks starts)."""
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_launch_cmd(n: int, argv, port: int):
    """The command that runs this bench as n ranks on one node (the driver's own form:
    torch.distributed.run, one process per GPU, rendezvous on 127.0.0.1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", "--master-port", str(port),
            os.path.abspath(__file__), *argv]


def launch_ranks(n: int, argv) -> int:
    """`bench.py --gpus N` started without a launcher (no WORLD_SIZE): run the N ranks as a CHILD
    process (never exec: a process that may have touched the GPU must not replace itself) and
    return its exit status.  The ranks inherit stdout, so rank 0's JSON line is this run's line."""
    import subprocess
    cmd = rank_launch_cmd(n, argv, free_port())
    print(f"bench: --gpus {n} without WORLD_SIZE: starting {n} ranks: {' '.join(cmd)}",
          file=sys.stderr, flush=True)
    return subprocess.run(cmd, env=dict(os.environ)).returncode


def rccl_overcommit(world: int, backend: str, devices: int):
    """The error text when RCCL ranks would share a GPU (two ranks of one communicator cannot:
    the run would fail or hang in init), else None.  Only the gloo rehearsal
    (CEC_BENCH_BACKEND=gloo) puts several ranks on one device."""
    if backend != "nccl" or world <= 1 or world <= devices:
        return None
    return (f"bench: {world} RCCL ranks but {devices} visible GPU(s): one rank per GPU; "
            "CEC_BENCH_BACKEND=gloo rehearses several ranks on one GPU")


def world_mismatch(world: int, gpus: int):
    """The error text when this rank's world size is not what --gpus asked for, else None (a line
    measured on another number of ranks than it claims must not be printed)."""
    if world == gpus:
        return None
    return (f"bench: WORLD_SIZE={world} but --gpus={gpus}: the line would misstate the GPU count; "
            "run `bench.py --gpus N` alone (it starts the ranks) or under torch.distributed.run "
            "with --nproc-per-node equal to --gpus")


def rank_row(r: int, row) -> dict:
    """One rank's gathered figures (gather_rows order = RANK_FIELDS) as the line's `ranks` entry;
    a figure the rank did not produce (0) is None."""
    out = {"rank": r}
    for name, v in zip(RANK_FIELDS, row):
        if name in ("device", "numa_node", "cpus", "c3_algorithmic_bytes", "c4_data_bytes",
                    "host_threads", "multi_copy_threads"):
            out[name] = int(v)
        elif name == "host_threads_numa_bound":
            out[name] = bool(v)
        elif name == "check_vs_oracle":  # 1 passed, 0 failed, -1 not run
            out[name] = None if v < 0 else bool(v)
        elif name == "step_ms":
            out[name] = round(v, 3)
        elif name.endswith("_frac"):
            out[name] = round(v, 4) if v else None
        else:
            out[name] = round(v, 4) if v else None
    return out


def node_figures(ranks) -> dict:
    """BASELINE configs[2] and configs[3] at node level from the per-rank rows: each rank's GPU
    runs its own C3 / C4 batch, so the node figure is the data of all ranks over the slowest
    rank's time (C4: sum of data bytes / max ms), and the fractions are the weakest rank's
    (min over ranks).  None when a rank did not run the block."""
    out = {"ranks": len(ranks)}
    if all(r.get("c4_ms") for r in ranks):
        c4_ms = max(r["c4_ms"] for r in ranks)
        c4_bytes = sum(r["c4_data_bytes"] for r in ranks)
        out["c4_encode_hash"] = {
            "value": round(c4_bytes / (c4_ms / 1e3) / 1e9, 2), "unit": "GB/s of data per node",
            "data_bytes": c4_bytes, "max_ms": c4_ms,
            "basis": "configs[3] sharded across the node's GPUs: sum over ranks of each GPU's "
                     "RS(20,8) batch data / the slowest rank's fused encode + SHA-256 time"}
    if all(r.get("c3_ms") for r in ranks):
        c3_ms = max(r["c3_ms"] for r in ranks)
        c3_bytes = sum(r["c3_algorithmic_bytes"] for r in ranks)
        out["c3_reconstruct"] = {
            "achieved": round(c3_bytes / (c3_ms / 1e3) / 1e9, 1), "unit": "GB/s per node",
            "min_frac": min(r["c3_reconstruct_frac"] for r in ranks),
            "basis": "algorithmic bytes of every rank's reconstruct / the slowest rank's time; "
                     "min_frac = the weakest GPU's fraction of its own 8 TB/s"}
    for key in ("north_star_encode_frac", "north_star_reconstruct_data_frac"):
        vals = [r.get(key) for r in ranks]
        if all(vals):
            out["min_" + key] = min(vals)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--parts", type=int, default=None, help="override parts per GPU")
    ap.add_argument("--shape", default=None, help="d,p override for the encode-only configs")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-full-check", action="store_true",
                    help="c2: check only the sampled parts against the oracle, not every part's "
                         "digests")
    ap.add_argument("--e2e-gib", type=float, default=64.0,
                    help="c2: GiB per GPU of the PCIe-bound end-to-end figure (0 = skip)")
    ap.add_argument("--check", action="store_true", help="verify a sampled part vs the oracle")
    ap.add_argument("--no-north-star", action="store_true",
                    help="c2: skip the encode-only / 2-erasure reconstruct_data block")
    ap.add_argument("--stream-gib", type=float, default=1024.0,
                    help="c5: total stream size in GiB across all ranks")
    ap.add_argument("--separate", action="store_true",
                    help="encode_hash as two launches (encode kernel, then SHA-256 kernel) "
                         "instead of the fused encode_hash_kernel")
    ap.add_argument("--corrupt", type=float, default=0.01,
                    help="c5r / end_to_end.read_repair: fraction of fetched chunks damaged")
    ap.add_argument("--devices", default=None,
                    help="c5 only: run in ONE process through the multi-GPU scheduler "
                         "(cec_multi), one shard per listed device ordinal, e.g. 0,1,2,3 "
                         "(repeats allowed: 0,0 = two shards on GPU 0)")
    ap.add_argument("--jobs-in-flight", type=int, default=2,
                    help="--devices mode: scheduler jobs (segments of the stream) queued at once")
    args = ap.parse_args()
    args.devices = [int(x) for x in args.devices.split(",")] if args.devices else None
    if args.devices and args.config != "c5":
        ap.error("--devices applies to c5 (the scheduler's write stream)")

    cfg = dict(CONFIGS[args.config])
    if args.parts:
        cfg["parts"] = args.parts
    if args.shape:  # A/B of other (d, p) on the encode configs
        if cfg["op"] != "encode":
            ap.error("--shape applies to the encode-only configs")
        cfg["d"], cfg["p"] = (int(x) for x in args.shape.split(","))
        cfg["workload"] = cfg["workload"].replace(
            "RS(10,4)", f"RS({cfg['d']},{cfg['p']})").replace(
            "RS(3,2)", f"RS({cfg['d']},{cfg['p']})").replace("RS(20,8)", f"RS({cfg['d']},{cfg['p']})")
    # --gpus N > 1 with no launcher around this process: start the N ranks as a child (before
    # anything here touches the GPU) and exit with its status
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world, rank, local = dist_env()
    backend = os.environ.get("CEC_BENCH_BACKEND", "nccl")
    err = world_mismatch(world, args.gpus) or rccl_overcommit(world, backend,
                                                              torch.cuda.device_count())
    if err:
        print(err, file=sys.stderr, flush=True)
        sys.exit(2)
    # one rank per GPU; more ranks than GPUs (gloo rehearsal) share them round-robin
    ordinal = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(ordinal)
    device = torch.device("cuda", ordinal)
    # the process's own CPU set, before the NUMA binding below narrows the main thread's (the
    # CPU baseline runs with it restored; the line's `host` block reports it)
    full_affinity = os.sched_getaffinity(0)
    host_report = host_info()
    # host threads and the pinned slots of this rank on its GPU's NUMA node (the engine places
    # its own pinned buffers there anyway; this keeps the host copies local too)
    numa_bound = ce.bind_thread_to_device_node(ordinal)
    numa_node = ce.device_numa_node(ordinal)
    rank_cpus = len(os.sched_getaffinity(0))
    host_report["rank_cpus_after_numa_bind"] = rank_cpus
    # host threads of this rank's end-to-end reader: half its CPUs (the rest run the engine's
    # own threads), 8 at most, within its share of the job's cgroup CPU quota (all ranks of the
    # node share one quota); the scheduler's staging threads per shard likewise
    e2e_threads = rank_threads(world)
    if "CEC_MULTI_COPY_THREADS" not in os.environ:
        os.environ["CEC_MULTI_COPY_THREADS"] = str(multi_copy_threads(world))
        ce.reload_knobs()
    host_report["quota_share_cpus"] = quota_share(world)
    host_report["rank_host_threads"] = e2e_threads
    host_report["multi_copy_threads"] = int(os.environ["CEC_MULTI_COPY_THREADS"])
    # RCCL ("nccl") carries only the barrier and the max-over-ranks all-reduce.
    # CEC_BENCH_BACKEND=gloo rehearses N > 1 with several ranks on one GPU; CEC_BENCH_PG=1 starts
    # the process group at world 1 too, so one GPU runs the N > 1 line's RCCL branch (init with
    # device_id, barriers, the float64 all-reduces, the per-rank rows).
    if world > 1 or os.environ.get("CEC_BENCH_PG") == "1":
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)
    reduce_dev = device if backend == "nccl" else None

    d, p, L, n_parts = cfg["d"], cfg["p"], cfg["chunk"], cfg["parts"]
    t = d + p
    codec = ce.ReedSolomon(d, p)
    if cfg["op"] == "stream":
        return run_stream(args, cfg, codec, world, rank, device, reduce_dev)
    if cfg["op"] == "read_stream":
        return run_read_stream(args, cfg, codec, world, rank, device, reduce_dev)
    buf = torch.empty((n_parts, t, L), dtype=torch.uint8, device=device)
    digests = torch.empty((n_parts, t, 32), dtype=torch.uint8, device=device)
    batch = ce.PartBatch.from_tensor(buf, L)
    stream = torch.cuda.current_stream(device)
    seed = rank_seed(0x5EED0000, rank)
    ce.fill_synthetic(batch, t, seed, stream)  # data chunks + (overwritten) parity slots

    present = None
    if cfg["op"] == "reconstruct_e2":
        ce.encode_batch(codec, batch, stream)
        # exactly 2 erasures per part, uniform over the 14 chunks (seeded); rebuilt in place
        pres = two_erasures(n_parts, t, rank)
        present = bytes(pres.flatten().tolist())
        algo_data = reconstruct_data_bytes(pres, d, L)
        # reconstruct: every part reads d chunks and writes its 2 missing ones
        algo_full = n_parts * (d + 2) * L
        # the erased chunks start zeroed, so the first step really rebuilds them
        buf.mul_(pres.to(device).view(n_parts, t, 1))
    elif cfg["op"] == "reconstruct":
        ce.encode_batch(codec, batch, stream)
        # 1..4 random erasures per part (seeded); rebuilt in place every step
        pres = c3_erasures(n_parts, t, p, rank)
        present = bytes(pres.flatten().tolist())
        missing_bytes = int((t - pres.sum(1)).sum().item()) * L
    elif cfg["op"] == "read":
        ce.encode_hash_batch(codec, batch, digests.data_ptr(), stream)
        # d random chunks loaded per part (the reference's read); the others are rebuilt (data)
        # or left alone (parity) in place every step
        g = torch.Generator().manual_seed(4321 + rank)
        pres = torch.zeros((n_parts, t), dtype=torch.uint8)
        for i in range(n_parts):
            pres[i, torch.randperm(t, generator=g)[:d]] = 1
        present = bytes(pres.flatten().tolist())
        # the chunks that were not loaded start zeroed, so the first step really rebuilds them
        buf.mul_(pres.to(device).view(n_parts, t, 1))
        missing_data = int((d - pres[:, :d].sum(1)).sum().item())
        touched = int(((d - pres[:, :d].sum(1)) > 0).sum().item())

    # One step = the hot path over the batch.  Each library call is one kernel launch on
    # `stream`; events bracket each launch so per-kernel averages come from the timed steps.
    fused = cfg["op"] == "encode_hash" and not args.separate
    read_status = []

    def step(evs=None):
        if cfg["op"] == "encode_hash" and fused:
            if evs is not None:
                evs[0].record(stream)
            ce.encode_hash_batch(codec, batch, digests.data_ptr(), stream)
            if evs is not None:
                evs[1].record(stream)
        elif cfg["op"] == "encode_hash":
            if evs is not None:
                evs[0].record(stream)
            ce.encode_batch(codec, batch, stream)
            if evs is not None:
                evs[1].record(stream)
            ce.sha256_batch(batch, 0, t, digests.data_ptr(), stream)
            if evs is not None:
                evs[2].record(stream)
        elif cfg["op"] == "encode":
            if evs is not None:
                evs[0].record(stream)
            ce.encode_batch(codec, batch, stream)
            if evs is not None:
                evs[1].record(stream)
        elif cfg["op"] == "reconstruct_e2":
            if evs is not None:
                evs[0].record(stream)
            ce.reconstruct_batch(codec, batch, present, True, stream)
            if evs is not None:
                evs[1].record(stream)
        elif cfg["op"] == "read":
            if evs is not None:
                evs[0].record(stream)
            _, st = ce.read_batch(codec, batch, present, digests.data_ptr(), stream)
            if evs is not None:
                evs[1].record(stream)
            read_status.append(sum(1 for x in st if x != ce.OK))
        else:
            if evs is not None:
                evs[0].record(stream)
            ce.reconstruct_batch(codec, batch, present, False, stream)
            if evs is not None:
                evs[1].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(device)
    barrier(world)

    n_ev = 3 if (cfg["op"] == "encode_hash" and not fused) else 2
    events = [[torch.cuda.Event(enable_timing=True) for _ in range(n_ev)]
              for _ in range(args.steps)]
    barrier(world)
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(events[k])
    torch.cuda.synchronize(device)
    barrier(world)
    t1 = time.perf_counter()
    local_s = (t1 - t0) / args.steps
    step_s = max_over_ranks(local_s, world, reduce_dev)

    # per-kernel averages over the timed steps
    def avg_ms(i, j):
        return sum(events[k][i].elapsed_time(events[k][j]) for k in range(args.steps)) / args.steps

    data_bytes = n_parts * d * L
    kernels = {}
    if cfg["op"] == "encode_hash" and fused:
        ms = avg_ms(0, 1)
        kernels["encode_hash_kernel"] = {"ms": round(ms, 4),
                                         "algorithmic_bytes": n_parts * t * L + n_parts * t * 32,
                                         "GBs": round((n_parts * t * (L + 32)) / ms / 1e6, 1)}
    elif cfg["op"] == "encode_hash":
        enc_ms, sha_ms = avg_ms(0, 1), avg_ms(1, 2)
        kernels[encode_kernel(d, t - d)] = {"ms": round(enc_ms, 4),
                                            "algorithmic_bytes": n_parts * t * L,
                                            "GBs": round(n_parts * t * L / enc_ms / 1e6, 1)}
        kernels["sha256_kernel"] = {"ms": round(sha_ms, 4),
                                    "algorithmic_bytes": n_parts * t * (L + 32),
                                    "GBs": round(n_parts * t * (L + 32) / sha_ms / 1e6, 1)}
    elif cfg["op"] == "encode":
        enc_ms = avg_ms(0, 1)
        kernels[encode_kernel(d, t - d)] = {"ms": round(enc_ms, 4),
                                            "algorithmic_bytes": n_parts * t * L,
                                            "GBs": round(n_parts * t * L / enc_ms / 1e6, 1)}
    elif cfg["op"] == "reconstruct_e2":
        ms = avg_ms(0, 1)
        kernels["rs_apply_kernel(reconstruct_data)"] = {
            "ms": round(ms, 4), "algorithmic_bytes": algo_data,
            "GBs": round(algo_data / ms / 1e6, 1)}
        # reconstruct (data + parity) of the same erasure sets, timed the same way
        evf = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(args.steps)]
        ce.reconstruct_batch(codec, batch, present, False, stream)
        for k in range(args.steps):
            evf[k][0].record(stream)
            ce.reconstruct_batch(codec, batch, present, False, stream)
            evf[k][1].record(stream)
        torch.cuda.synchronize(device)
        ms_f = sum(e[0].elapsed_time(e[1]) for e in evf) / args.steps
        full_gbs = algo_full / (ms_f / 1e3) / 1e9
        kernels["also_reconstruct"] = {
            "call": "reconstruct (data + parity, file_part.rs:304), same parts and erasures",
            "ms": round(ms_f, 4), "algorithmic_bytes": algo_full,
            "GBs": round(full_gbs, 1),
            "roofline": {"bound": "hbm", "kernel": "rs_apply_var_kernel",
                         "achieved": round(full_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(full_gbs / HBM_PEAK_GBS, 4)}}
    elif cfg["op"] == "read":
        # one read_batch call: verify (sha256_lane_kernel, d chunks per part) on the caller's
        # stream, the speculative decode (rs_apply_var_kernel) beside it on a side stream
        ms = avg_ms(0, 1)
        algo = n_parts * d * (L + 32) + touched * d * L + missing_data * L
        kernels["read_batch(verify+decode)"] = {"ms": round(ms, 4), "algorithmic_bytes": algo,
                                                "GBs": round(algo / ms / 1e6, 1)}
    else:
        rec_ms = avg_ms(0, 1)
        # each part with k missing reads d chunks and writes k: (d*parts_touched + missing)
        touched = sum(1 for i in range(n_parts) if any(present[i * t + j] == 0 for j in range(t)))
        algo = touched * d * L + missing_bytes
        kernels["rs_apply_kernel(reconstruct)"] = {"ms": round(rec_ms, 4),
                                                   "algorithmic_bytes": algo,
                                                   "GBs": round(algo / rec_ms / 1e6, 1)}
    dom_name = max((k for k in kernels if not k.startswith("also_")), key=lambda k: kernels[k]["ms"])
    dom = kernels[dom_name]
    achieved = dom["algorithmic_bytes"] / (dom["ms"] / 1e3) / 1e9
    traffic, traffic_src = measured_traffic(
        args.config + ("sep" if cfg["op"] == "encode_hash" and not fused else ""),
        dom_name, n_parts == CONFIGS[args.config]["parts"] and not args.shape, with_source=True)

    valu = None
    if cfg["op"] in ("encode_hash", "read"):
        # useful SHA work: one lane-block per 64-byte block of every chunk (incl. FIPS padding)
        blocks = L // 64 + (1 if L % 64 + 9 <= 64 else 2)
        sha_kernel = ("read_batch(verify+decode)" if cfg["op"] == "read" else
                      "encode_hash_kernel" if fused else "sha256_kernel")
        sha_ms = kernels[sha_kernel]["ms"]
        hashed = d if cfg["op"] == "read" else t
        wave_inst = n_parts * hashed * blocks * SHA_VALU_PER_BLOCK / 64
        achieved_g = wave_inst / (sha_ms / 1e3) / 1e9
        peak_g = MI355X_SIMDS * MI355X_CLOCK_GHZ / SHA_SIMD_CYCLES
        valu = {"bound": "valu", "kernel": sha_kernel,
                "achieved": round(achieved_g, 1), "peak": round(peak_g, 1),
                "unit": "G wave64-inst/s", "frac": round(achieved_g / peak_g, 4),
                "basis": f"SHA-256: {SHA_VALU_PER_BLOCK} VALU/64-B block/lane, "
                         f"{SHA_SIMD_CYCLES:.2f} SIMD cycles/inst saturated, "
                         f"{MI355X_SIMDS} SIMDs x {MI355X_CLOCK_GHZ} GHz"}
        # The design's own bound: one SHA wave per SIMD issues at most one VALU op per 4 cycles
        # (MI355X_MICROARCH.md, one wave alone), and a chunk's chain is serial, so the step can
        # take no less than blocks x ops x 4 cycles; at the nominal clock (the chip held
        # 2.36-2.38 GHz under this load, profiles/r2f_c2_summary.md, so this reads low).
        floor_ms = blocks * SHA_VALU_PER_BLOCK * 4 / (MI355X_CLOCK_GHZ * 1e9) * 1e3
        if n_parts * hashed <= MI355X_SIMDS * 64:  # one SHA wave per SIMD (C2, c3r; not C4)
            valu["lone_wave_issue_floor"] = {
                "ms": round(floor_ms, 2), "frac": round(floor_ms / sha_ms, 4),
                "basis": f"{blocks} blocks per chunk x {SHA_VALU_PER_BLOCK} VALU x 4 cycles per "
                         f"instruction of one wave alone, {MI355X_CLOCK_GHZ} GHz"}
        # the same kernel's VALU issue measured by rocprofv3 SQ counters (committed run of this
        # command, not this run): SQ_INSTS_VALU over (GRBM_GUI_ACTIVE / 8 XCDs) x 1024 SIMDs
        counters = measured_valu(args.config, sha_kernel,
                                 n_parts == CONFIGS[args.config]["parts"] and not args.shape)
        if counters:
            valu["counters"] = counters

    # --check: a sampled part of this rank's own buffer against the oracle, on EVERY rank (ANDed
    # over the ranks below)
    ok = None
    if args.check and cfg["op"] == "read":
        import numpy as np
        import oracle
        k = n_parts // 2
        host = buf[k].cpu().numpy()
        pr = present[k * t:(k + 1) * t]
        st, out = oracle.reconstruct(d, p, [host[i] if pr[i] else None for i in range(t)],
                                     data_only=True)
        ok = (st == 0 and not any(read_status) and
              all(np.array_equal(out[i], host[i]) for i in range(d)))
    elif args.check and cfg["op"] != "reconstruct":
        import hashlib
        import numpy as np
        import oracle
        k = n_parts // 2
        host = buf[k].cpu().numpy()
        st, par = oracle.encode_sep(d, p, [host[j] for j in range(d)])
        ok = st == 0 and all(np.array_equal(par[i], host[d + i]) for i in range(p))
        if cfg["op"] == "encode_hash":
            dg = digests[k].cpu().numpy()
            ok = ok and all(hashlib.sha256(host[j].tobytes()).digest() == dg[j].tobytes()
                            for j in range(t))

    # sampled whole parts of the buffers behind value / north_star / baseline_configs, checked
    # against the oracle after every timed region: at N = 1 in the cpu_baseline leg (with every
    # part of the C2 / C4 buffers), at N > 1 on every rank, its own buffers, ANDed over the ranks
    snap = None
    if args.config == "c2" and fused and (world > 1 or not args.no_cpu_baseline):
        snap = {"parts": (0, n_parts // 2, n_parts - 1)}
        snap["headline"] = snapshot_parts(buf, digests, snap["parts"])
        if world == 1 and not args.no_full_check:
            snap["c2_digests"] = digests.cpu().numpy()
            snap["c2_dev"] = buf  # checked whole in the cpu_baseline leg (batch_vs_oracle)
    # north_star's two >= 60 % targets on the same buffer (C2 only)
    nstar = None
    if args.config == "c2" and not args.separate and not args.no_north_star:
        nstar = north_star_block(codec, batch, buf, digests, stream, device, rank, d, p, L,
                                 args.steps, snap)
    others = None
    if args.config == "c2" and not args.separate and not args.no_north_star:
        others = baseline_configs_block(codec, batch, buf, digests, stream, device, rank, d, p,
                                        L, args.steps, snap)
    # the end-to-end forms below use their own buffers (with the whole-batch check on, `snap`
    # keeps the C2 and C4 device buffers, ~84 GiB of HBM, for the cpu_baseline leg)
    del buf, digests
    torch.cuda.empty_cache()

    # every rank streams its own share (barriers inside): the PCIe-inclusive figure
    e2e = stream = None
    if args.config == "c2" and args.e2e_gib > 0 and not args.separate:
        e2e = end_to_end(codec, d, p, L, args.e2e_gib, world, rank, reduce_dev, e2e_threads,
                         ordinal, device, args.corrupt,
                         full_check=snap is not None and "c2_dev" in snap)

    # N > 1: every rank checks the sampled whole parts of ITS OWN buffers (headline, north_star,
    # C3, C4: the snapshots above) against the oracle, after every timed region; the line's
    # check_vs_oracle is the AND over the ranks (the rows below carry each rank's result)
    rank_ok, rank_detail = ok, None
    if snap is not None and world > 1:
        t0 = time.perf_counter()
        rank_detail = check_vs_oracle(snap, d, p, max(1, e2e_threads))
        rank_detail["seconds"] = round(time.perf_counter() - t0, 2)
        rank_ok = rank_detail["ok"] and (ok is None or ok)

    # per-rank figures for the N > 1 line (a straggler or a cross-NUMA placement must be
    # visible from the line alone)
    ranks = node = None
    if dist.is_initialized():
        e2e_v, link_v = (e2e or {}).get("_local") or (0.0, 0.0)
        rr_v = ((e2e or {}).get("read_repair") or {}).get("_local") or 0.0
        # each rank's own north_star / C3 / C4 figures (the blocks run on every rank, on its
        # own GPU)
        ns_enc = (nstar or {}).get("encode", {}).get("frac") or 0.0
        ns_rec = (nstar or {}).get("reconstruct_data_2_erasures", {}).get("frac") or 0.0
        c3 = (others or {}).get("c3_reconstruct", {})
        c4 = (others or {}).get("c4_encode_hash", {})
        row = [ordinal, numa_node, 1.0 if numa_bound else 0.0, rank_cpus, local_s * 1e3, e2e_v,
               link_v, ns_enc, ns_rec, c3.get("frac") or 0.0, c3.get("algorithmic_bytes") or 0,
               c3.get("ms") or 0.0, c4.get("ms") or 0.0, c4.get("data_bytes") or 0, rr_v,
               quota_share(world) or 0.0, e2e_threads, int(os.environ["CEC_MULTI_COPY_THREADS"]),
               -1.0 if rank_ok is None else float(bool(rank_ok))]
        rows = gather_rows(row, world, reduce_dev)
        ranks = [rank_row(r, row) for r, row in enumerate(rows)]
        node = node_figures(ranks)
        if world > 1:
            checks = [r["check_vs_oracle"] for r in ranks]
            # every rank ran its check (or none did: --no-north-star etc. with no --check)
            ok = None if all(c is None for c in checks) else all(c is True for c in checks)

    if rank == 0:
        total_data = data_bytes * world
        value = total_data / step_s / 1e9
        line = {
            "metric": METRIC if args.config == "c2" else f"{METRIC} [{args.config}]",
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(step_s * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (counter-based generator on device; inputs resident in HBM)",
            "config": {
                "workload": workload(cfg, args),
                "d": d, "p": p, "chunk_bytes": L, "parts_per_gpu": n_parts,
                "data_bytes_per_step": total_data,
                "parallelism": f"part-sharded x{world}, no collective",
                "host_threads_numa_bound": numa_bound,
            },
            "roofline": {
                "bound": "hbm",
                "kernel": dom_name,
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
            },
            "kernels": kernels,
        }
        if valu is not None:
            line["valu_roofline"] = valu
        if nstar is not None:
            line["north_star"] = nstar
        if others is not None:
            line["baseline_configs"] = others
        if e2e is not None:
            e2e.pop("_local", None)
            stream = e2e.pop("_stream", None)
            (e2e.get("read_repair") or {}).pop("_local", None)
            line["end_to_end"] = e2e
        if ranks is not None:
            steps_ms = [r["step_ms"] for r in ranks]
            line["ranks"] = ranks
            line["node"] = node
            line["step_ms_over_ranks"] = {"max": round(max(steps_ms), 3),
                                          "mean": round(sum(steps_ms) / len(steps_ms), 3),
                                          "min": round(min(steps_ms), 3)}
        if ok is not None:
            line["check_vs_oracle"] = bool(ok)
        if world > 1 and ok is not None:
            line["check_vs_oracle_detail"] = {
                "all_ranks_ok": bool(ok),
                "ranks_ok": [r["check_vs_oracle"] for r in ranks],
                "rank0": rank_detail,
                "basis": "each rank's own sampled whole parts (headline C2 buffer, north_star's "
                         "re-encode, C3's rebuild, C4's fused encode and round trip; plus --check's "
                         "part) vs oracle.encode_sep and hashlib SHA-256, after every timed region; "
                         "ANDed over the ranks (every part of the buffers: N = 1 only)"}
        line["host"] = host_report
        if world == 1 and not args.no_cpu_baseline and cfg["op"] in ("encode_hash", "encode"):
            # the cpu_baseline leg (after every timed region), the one place the bench runs the
            # oracle: first this run's own buffers against it, then the timed CPU baseline; both
            # on the process's full CPU set (the main thread was bound to GPU0's NUMA node above)
            os.sched_setaffinity(0, full_affinity)
            avail, quota = len(full_affinity), cpu_quota()[1]
            threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, avail)
            if snap is not None:
                t0 = time.perf_counter()
                detail = check_vs_oracle(snap, d, p, threads)
                if stream is not None:  # every part of end_to_end's write stream
                    bad = stream_check(stream[0], stream[1], d, p, threads)
                    detail["checks"]["end_to_end_all_parts"] = not bad
                    detail["end_to_end_all_parts_checked"] = {
                        "parts": len(stream[1]), "digests": int(stream[1].size // 32)}
                    detail["end_to_end_all_parts_mismatched"] = bad[:8]
                    detail["ok"] = detail["ok"] and not bad
                    stream = None
                detail["seconds"] = round(time.perf_counter() - t0, 2)
                snap.pop("c2_dev", None)
                snap.pop("c4_dev", None)
                line["check_vs_oracle"] = detail["ok"]
                line["check_vs_oracle_detail"] = detail
            line["cpu_baseline"] = cpu_baseline(cfg, threads, os.cpu_count() or avail, avail,
                                                quota)
        # the process's peak resident host memory (page-locked slots, rings, the full-check
        # copies): what the run asks of the box
        import resource
        host_report["peak_rss_gib"] = round(
            resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / (1 << 20), 1)
        print(json.dumps(line), flush=True)

    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
