"""The C++ host layer (include/chunky_ec.hpp) and its test program, which restates the
reference's own tests (tests/hash.rs, tests/file.rs, tests/cluster.rs) plus the crate KATs and
golden digests in C++ against the engine.  The binary is built in-tree by
`make -C chunky-bits_amd/csrc` (__graft_entry__.build())."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "reference_mirror_test")
NAMES = ["sha256", "test_file_write", "test_resilver", "test_cluster_digests", "test_cp_50mib",
         "test_range_reads",
         "test_write_concurrency",
         "test_batched_paths", "test_multi_device_paths", "test_mixed_shape_read",
         "test_batched_verify_resilver", "test_locations_bad_then_good", "test_one_encode",
         "test_matrix_rows", "test_errors", "test_reconstruct_every_pattern"]


def _binary():
    if not os.path.exists(BIN):
        pytest.skip("reference_mirror_test not built (make -C chunky-bits_amd/csrc)")
    return BIN


def test_mirror_binary_lists_the_reference_tests():
    out = subprocess.run([_binary(), "--list"], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0
    assert out.stdout.split() == NAMES


def test_mirror_without_gpu_fails_loudly():
    """No CPU fallback: with no HIP device every computation raises EngineError (NoDevice)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    out = subprocess.run([_binary(), "sha256"], capture_output=True, text=True, timeout=60)
    assert out.returncode == 1
    assert "no HIP device" in out.stderr


@pytest.mark.gpu
def test_mirror_reference_tests_pass_on_gpu():
    out = subprocess.run([_binary()], capture_output=True, text=True, timeout=110)
    print(out.stdout, out.stderr)
    assert out.returncode == 0, out.stdout + out.stderr
    for name in NAMES:
        assert f"{name} ... ok" in out.stdout
