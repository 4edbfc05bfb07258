"""`chunky-shards encode-shards / decode-shards` (chunky-bits_amd/cli/chunky_shards.cpp): the
reference CLI's direct use of the erasure crate (src/bin/chunky-bits/main.rs:235-312, argument
rules of get_shard_encoder at :521-559), on local files through the per-call C-ABI.

CPU tests cover the argument rules and the crate errors raised before any device work; the GPU
tests check shard files bit-exact against the oracle, decode after losing up to p shards, and the
"Error <target>: ..." lines for unreadable targets.  The crate's own Display text for its errors
is not available offline (the crate source is not vendored): error lines carry the variant name,
which is "parity unpinned" as far as the exact wording goes.
"""
import os
import subprocess

import numpy as np
import pytest

import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "chunky-bits_amd", "bin", "chunky-shards")


def _bin():
    if not os.path.exists(BIN):
        pytest.skip("chunky-shards not built (make -C chunky-bits_amd/csrc)")
    return BIN


def run(*args, stdin=None, cwd=None):
    return subprocess.run([_bin(), *map(str, args)], input=stdin, capture_output=True,
                          cwd=cwd, timeout=120)


def _gpu():
    import torch
    return torch.cuda.is_available()


# ---- argument rules (no device work) ----------------------------------------------------------

def test_parity_count_is_required(tmp_path):
    r = run("encode-shards", "-", "a", "b", "c", cwd=tmp_path, stdin=b"x")
    assert r.returncode == 1
    assert r.stderr.decode().strip() == "Parity Chunk Count must be known to decode shards"
    r = run("--data-chunks", 2, "decode-shards", "a", "b", "c", cwd=tmp_path)
    assert r.returncode == 1 and b"Parity Chunk Count must be known" in r.stderr


def test_target_count_rules(tmp_path):
    r = run("--data-chunks", 3, "--parity-chunks", 2, "encode-shards", "-", "a", "b", "c",
            cwd=tmp_path, stdin=b"x")
    assert r.returncode == 1
    assert r.stderr.decode().strip() == "Invalid targets: Expected 5 targets but got 3"
    r = run("--parity-chunks", 3, "decode-shards", "a", "b", "c", cwd=tmp_path)
    assert r.returncode == 1
    assert r.stderr.decode().strip() == "Invalid targets: Expected more than 3 targets but got 3"
    assert not any(os.path.exists(tmp_path / t) for t in "abc")


def test_crate_errors_from_new_and_encode(tmp_path):
    # ReedSolomon::new(d, 0) -> TooFewParityShards; d + p > 256 -> TooManyShards
    r = run("--parity-chunks", 0, "decode-shards", "a", "b", cwd=tmp_path)
    assert r.returncode == 1 and r.stderr.decode().strip() == "TooFewParityShards"
    r = run("--data-chunks", 200, "--parity-chunks", 100, "decode-shards",
            *[f"s{i}" for i in range(300)], cwd=tmp_path)
    assert r.returncode == 1 and r.stderr.decode().strip() == "TooManyShards"
    # an empty source gives zero-length shards: encode_sep -> EmptyShard, nothing written
    r = run("--parity-chunks", 2, "encode-shards", "-", "a", "b", "c", cwd=tmp_path, stdin=b"")
    assert r.returncode == 1 and r.stderr.decode().strip() == "EmptyShard"
    assert not any(os.path.exists(tmp_path / t) for t in "abc")


def test_option_values_follow_sized_int(tmp_path):
    """DataChunkCount 1..=255, ParityChunkCount 0..=255 (cluster/sized_int.rs:139-157, parsed
    as u8): clap rejects others with the SizeError text and exit status 2."""
    r = run("--data-chunks", 256, "--parity-chunks", 1, "decode-shards", "a", cwd=tmp_path)
    assert r.returncode == 2
    assert r.stderr.decode().strip().endswith(
        "DataChunkCount must be greater than 1 and less than 256")
    r = run("--data-chunks", 0, "--parity-chunks", 1, "decode-shards", "a", cwd=tmp_path)
    assert r.returncode == 2
    r = run("--parity-chunks=x", "decode-shards", "a", cwd=tmp_path)
    assert r.returncode == 2 and b"ParityChunkCount must be greater than 0" in r.stderr


def test_without_gpu_fails_loudly(tmp_path):
    if _gpu():
        pytest.skip("GPU present")
    r = run("--parity-chunks", 2, "encode-shards", "-", "a", "b", "c", cwd=tmp_path,
            stdin=b"hello")
    assert r.returncode == 1 and b"no HIP device" in r.stderr
    assert not any(os.path.exists(tmp_path / t) for t in "abc")


# ---- on the GPU -------------------------------------------------------------------------------

def _encode(tmp_path, data, d, p, with_d=True):
    src = tmp_path / "src.bin"
    src.write_bytes(data)
    targets = [tmp_path / f"shard{i}" for i in range(d + p)]
    opts = (["--data-chunks", d] if with_d else []) + ["--parity-chunks", p]
    r = run(*opts, "encode-shards", src, *targets)
    assert r.returncode == 0, r.stderr
    assert r.stderr == b""
    return targets


@pytest.mark.gpu
@pytest.mark.parametrize("d,p,n", [(3, 2, 50 * 1024 + 1), (10, 4, 3 * 1024 * 1024 + 17),
                                   (5, 5, 10), (1, 1, 4096), (20, 8, 1 << 20)])
def test_encode_shards_bit_exact_vs_oracle(tmp_path, d, p, n):
    data = np.random.default_rng(n + d).integers(0, 256, n, dtype=np.uint8).tobytes()
    targets = _encode(tmp_path, data, d, p, with_d=(d != 5))
    L = (n + d - 1) // d
    padded = np.frombuffer(data + bytes(L * d - n), np.uint8)
    shards = [padded[j * L:(j + 1) * L] for j in range(d)]
    st, par = oracle.encode_sep(d, p, shards)
    assert st == 0
    for i, t in enumerate(targets):
        want = shards[i] if i < d else par[i - d]
        assert t.read_bytes() == want.tobytes(), i


@pytest.mark.gpu
@pytest.mark.parametrize("d,p", [(3, 2), (10, 4), (20, 8)])
def test_decode_shards_after_losing_p(tmp_path, d, p):
    n = 777 * d + 5
    data = np.random.default_rng(d * 31 + p).integers(0, 256, n, dtype=np.uint8).tobytes()
    targets = _encode(tmp_path, data, d, p)
    L = (n + d - 1) // d
    rng = np.random.default_rng(d)
    lost = sorted(rng.choice(d + p, p, replace=False).tolist())
    for i in lost:
        os.remove(targets[i])
    r = run("--parity-chunks", p, "decode-shards", *targets)
    assert r.returncode == 0, r.stderr
    # padding is not stripped (the reference writes the d data shards as they are)
    assert r.stdout == data + bytes(L * d - n)
    lines = r.stderr.decode().splitlines()
    assert lines == [f"Error {targets[i]}: {targets[i]}: No such file or directory (os error 2)"
                     for i in lost]


@pytest.mark.gpu
def test_decode_shards_errors(tmp_path):
    d, p = 4, 2
    data = bytes(range(256)) * 40
    targets = _encode(tmp_path, data, d, p)
    for i in (0, 3, 5):
        os.remove(targets[i])
    r = run("--parity-chunks", p, "decode-shards", *targets)
    assert r.returncode == 1 and r.stdout == b""
    assert r.stderr.decode().splitlines()[-1] == "TooFewShardsPresent"
    # shards of different lengths: IncorrectShardSize
    targets = _encode(tmp_path, data, d, p)
    with open(targets[1], "ab") as f:
        f.write(b"\0")
    r = run("--parity-chunks", p, "decode-shards", *targets)
    assert r.returncode == 1 and r.stderr.decode().strip() == "IncorrectShardSize"


@pytest.mark.gpu
def test_stdio_locations(tmp_path):
    """`-` is stdin for the source and stdout for a target (ClusterLocation::Stdio)."""
    d, p = 2, 1
    data = b"chunky bits shard cli"
    r = run("--parity-chunks", p, "encode-shards", "-", tmp_path / "a", "-", tmp_path / "c",
            stdin=data)
    assert r.returncode == 0, r.stderr
    L = (len(data) + 1) // 2
    padded = data + bytes(2 * L - len(data))
    assert (tmp_path / "a").read_bytes() == padded[:L]
    assert r.stdout == padded[L:]
    st, par = oracle.encode_sep(d, p, [np.frombuffer(padded[:L], np.uint8),
                                       np.frombuffer(padded[L:], np.uint8)])
    assert (tmp_path / "c").read_bytes() == par[0].tobytes()
