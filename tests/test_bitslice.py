"""CPU checks of the bit-sliced encoder's construction (rs_encode_bs_kernel).

tests/cpp/bitslice_check.cpp restates the kernel's data path on the host (bit transpose, XOR
network over the compile-time bit matrices, transpose back) and checks it against the direct
GF(2^8) encode; here its compile-time parity rows are also compared with the oracle's encode
(unit-vector columns of encode_sep, oracle/cec_oracle.c).  The kernel itself is compared with the
oracle by the -m gpu tests (every RS(3,2) / RS(10,4) / RS(20,8) encode at aligned layouts).
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "chunky-bits_amd", "csrc")


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    if not shutil.which("g++"):
        pytest.skip("no g++")
    exe = str(tmp_path_factory.mktemp("bs") / "bitslice_check")
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-I" + CSRC,
                    os.path.join(ROOT, "tests", "cpp", "bitslice_check.cpp"),
                    os.path.join(CSRC, "gf256.cpp"), "-o", exe], check=True, timeout=120)
    return exe


def test_network_reproduces_the_field_multiply(checker):
    out = subprocess.run([checker], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout
    assert out.stdout.strip() == "ok"


def test_compiled_parity_rows_equal_the_oracle(checker):
    out = subprocess.run([checker, "--print"], capture_output=True, text=True, timeout=60,
                         check=True)
    shapes = [list(map(int, line.split())) for line in out.stdout.splitlines()]
    assert [(s[0], s[1]) for s in shapes] == [(3, 2), (10, 4), (20, 8)]
    for s in shapes:
        d, p, coefs = s[0], s[1], np.array(s[2:], np.uint8).reshape(s[1], s[0])
        for j in range(d):
            data = [np.full(1, 1 if i == j else 0, np.uint8) for i in range(d)]
            st, par = oracle.encode_sep(d, p, data)
            assert st == 0
            assert [int(x[0]) for x in par] == list(coefs[:, j]), (d, p, j)


def test_compiled_rows_match_survey_appendix_a(checker):
    """RS(3,2) and RS(10,4) parity rows of the restatement that matched
    the crate's published KATs."""
    out = subprocess.run([checker, "--print"], capture_output=True, text=True, timeout=60,
                         check=True)
    rows = {(s[0], s[1]): s[2:] for s in (list(map(int, l.split())) for l in out.stdout.splitlines())}
    assert rows[(3, 2)] == [1, 1, 1, 15, 8, 6]
    assert rows[(10, 4)] == [129, 150, 175, 184, 210, 196, 254, 232, 3, 2,
                             150, 129, 184, 175, 196, 210, 232, 254, 2, 3,
                             191, 214, 98, 10, 6, 111, 223, 183, 5, 4,
                             214, 191, 10, 98, 111, 6, 183, 223, 4, 5]
