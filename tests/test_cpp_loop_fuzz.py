"""The C++ host layer's batched loops (include/chunky_ec.hpp; the read: FileReference::read_to
over read_run / retry_start / retry_round / retry_collect, the twin of chunky_ec.batchreader and
the Rust BatchReader) on the CPU: tests/cpp/host_loop_fuzz.cpp links the header against a stand-in
scheduler that keeps cec_multi's job contract (jobs computed only when they complete, after a
seeded number of cec_multi_query polls; carry ids kept per part and used once) and computes with
the oracle.  Random location mixes, window sizes, depths, shard lists and carry switches: every
part comes out as stored and in order, a part without d good chunks fails the read with
TooFewShardsPresent (file_part.rs:92-107), and no job or carry id is left behind.  Then the
batched verify / resilver loop (check_run) against the per-part FilePart::verify / resilver on
copies of the same file and store: same reports, same write-backs, and the resilvered file reads
back whole (file_part.rs:228-390); and each seed first writes a file through the batched write
(FileWriteBuilder::batch over cec_multi_encode_hash jobs) and the per-part write: same parts,
digests, locations and stored bytes (writer.rs:117-255).  The fuzz found a read that failed with a retry round in flight
keeping that round's carry ids (fixed)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def fuzz_bin(tmp_path_factory):
    if not (shutil.which("gcc") and shutil.which("g++")):
        pytest.skip("no host compiler")
    d = tmp_path_factory.mktemp("read_fuzz")
    obj, exe = str(d / "oracle.o"), str(d / "host_loop_fuzz")
    subprocess.run(["gcc", "-O2", "-c", os.path.join(ROOT, "oracle", "cec_oracle.c"), "-o", obj],
                   check=True)
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "host_loop_fuzz.cpp"), obj, "-lpthread",
                    "-o", exe], check=True)
    return exe


@pytest.mark.parametrize("first", [0, 1000])
def test_cpp_host_loop_fuzz(fuzz_bin, first):
    r = subprocess.run([fuzz_bin, str(first), "300"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "0 failed, 0 contract violations" in r.stdout


def test_cpp_host_loop_fuzz_under_sanitizers(tmp_path):
    """The same fuzz built with AddressSanitizer + UndefinedBehaviorSanitizer (host code only:
    the header's loops, the stand-in and the oracle): no out-of-bounds access, use after free,
    leak or undefined behaviour over 100 seeds."""
    if not (shutil.which("gcc") and shutil.which("g++")):
        pytest.skip("no host compiler")
    san = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-g", "-O0"]
    obj, exe = str(tmp_path / "oracle_san.o"), str(tmp_path / "host_loop_fuzz_san")
    subprocess.run(["gcc", *san, "-c", os.path.join(ROOT, "oracle", "cec_oracle.c"), "-o", obj],
                   check=True)
    subprocess.run(["g++", "-std=c++17", *san, "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "host_loop_fuzz.cpp"), obj, "-lpthread",
                    "-o", exe], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe, "5000", "100"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "0 failed, 0 contract violations" in r.stdout
