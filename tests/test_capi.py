"""C-ABI library checks that need no GPU: it loads, exports every function include/chunky_ec.h
declares, and its host-only entry points (codec construction, coding matrix, status names,
the synthetic-data mirror) behave like the crate / oracle."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "chunky_ec.h")
LIB = os.path.join(ROOT, "chunky-bits_amd", "chunky_ec", "libchunky_ec.so")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"\b([a-z_0-9]+)\s*\(", src)
    return sorted({n for n in names if n.startswith("cec_")})


def test_header_declares_expected_surface():
    fns = declared_functions()
    for must in ["cec_codec_new", "cec_encode_sep", "cec_reconstruct", "cec_reconstruct_data",
                 "cec_sha256", "cec_part_encode", "cec_encode_batch", "cec_encode_hash_batch",
                 "cec_reconstruct_batch", "cec_sha256_batch"]:
        assert must in fns


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB), "build first: make -C chunky-bits_amd/csrc"
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r" T (cec_\w+)", out))
    missing = [f for f in declared_functions() if f not in exported]
    assert not missing, missing
    lib = ctypes.CDLL(LIB)
    for f in declared_functions():
        getattr(lib, f)


def test_library_has_gfx950_code_object():
    data = open(LIB, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data  # offload bundle entry id of the .hip_fatbin


def test_library_was_built_from_these_sources():
    """Build provenance: the library's cec_build_id is the hash of the sources in this tree
    (csrc/source_hash.py), so the .so a GPU run loads was built from HEAD's sources, and the
    binding refuses one that was not."""
    import importlib.util
    import chunky_ec as ce
    spec = importlib.util.spec_from_file_location(
        "sh", os.path.join(ROOT, "chunky-bits_amd", "csrc", "source_hash.py"))
    sh = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(sh)
    assert ce.BUILD_ID == sh.source_hash() == ce.SOURCE_HASH
    assert ce.BUILD_MATCHES_SOURCE
    assert "include/chunky_ec.h" in sh.source_files()
    assert any(f.endswith("rs_kernels.hip") for f in sh.source_files())


def test_status_codes_match_crate_order():
    import chunky_ec as ce
    names = ["Ok", "TooFewShards", "TooManyShards", "TooFewDataShards", "TooManyDataShards",
             "TooFewParityShards", "TooManyParityShards", "TooFewBufferShards",
             "TooManyBufferShards", "IncorrectShardSize", "TooFewShardsPresent", "EmptyShard",
             "InvalidShardFlags", "InvalidIndex"]
    for code, name in enumerate(names):
        assert ce.status_name(code) == name
    assert ce.abi_version() == ce.ABI_VERSION == 3


@pytest.mark.parametrize("d,p", [(1, 1), (3, 2), (10, 4), (20, 8), (5, 5), (17, 3), (128, 128),
                                 (1, 255)])
def test_codec_matrix_matches_oracle(d, p):
    import chunky_ec as ce
    rs = ce.ReedSolomon(d, p)
    assert (rs.data_shard_count(), rs.parity_shard_count(), rs.total_shard_count()) == (d, p, d + p)
    assert np.array_equal(np.array(rs.matrix(), dtype=np.uint8), oracle.coding_matrix(d, p))


def test_codec_matrix_kat_rows(kats):
    """The engine's own RS(5,5) matrix (csrc/gf256.cpp, not the oracle) against the published
    decode-matrix KAT (crate_kats.json matrix_inverse[1]: rows 0, 1, 3, 4, 5) and RS(5,5)'s
    one-encode parity."""
    import chunky_ec as ce
    m = np.array(ce.ReedSolomon(5, 5).matrix(), dtype=np.uint8)
    assert m[[0, 1, 3, 4, 5]].tolist() == kats["matrix_inverse"][1]["m"]
    k = kats["rs_one_encode"]
    data = np.array(k["data"], np.uint8)
    par = [[0, 0] for _ in range(5)]
    for r in range(5):
        for j in range(5):
            for c in range(2):
                par[r][c] ^= oracle.gf_mul(int(m[5 + r, j]), int(data[j, c]))
    assert par == k["parity"]
    for v in kats["coding_matrix_published"]:  # the engine's own matrix at RS(4,2)
        d, p = v["data_shards"], v["parity_shards"]
        m = np.array(ce.ReedSolomon(d, p).matrix(), dtype=np.uint8)
        assert m[d:].tolist() == v["parity_rows"]


def test_codec_new_errors():
    import chunky_ec as ce
    for (d, p), code in [((0, 1), ce.TOO_FEW_DATA_SHARDS), ((1, 0), ce.TOO_FEW_PARITY_SHARDS),
                         ((0, 0), ce.TOO_FEW_DATA_SHARDS), ((200, 57), ce.TOO_MANY_SHARDS)]:
        with pytest.raises(ce.Error) as e:
            ce.ReedSolomon(d, p)
        assert e.value.code == code
    ce.ReedSolomon(128, 128)


def test_argument_errors_precede_device_use():
    """Crate argument errors are reported before any HIP call (so they hold with or without a
    GPU); compute entry points without a device report NoDevice rather than computing on CPU."""
    import chunky_ec as ce
    rs = ce.ReedSolomon(3, 2)
    with pytest.raises(ce.Error) as e:
        rs.encode_sep([b"ab", b"ab"], [bytearray(2), bytearray(2)])
    assert e.value.code == ce.TOO_FEW_DATA_SHARDS
    with pytest.raises(ce.Error) as e:
        rs.encode_sep([b"ab", b"ab", b"a"], [bytearray(2), bytearray(2)])
    assert e.value.code == ce.INCORRECT_SHARD_SIZE
    with pytest.raises(ce.Error) as e:
        rs.reconstruct([b"ab", None, None, None, b"ab"])
    assert e.value.code == ce.TOO_FEW_SHARDS_PRESENT
    shards = [b"ab"] * 5
    rs.reconstruct(shards)  # nothing missing: Ok without touching the device
    if ce.device_count() == 0:
        with pytest.raises(ce.Error) as e:
            rs.encode_sep([b"ab"] * 3, [bytearray(2), bytearray(2)])
        assert e.value.code == ce.ERR_NO_DEVICE


def test_read_pipeline_argument_checks_precede_device_use():
    """cec_read_pipeline_new_ex rejects unknown flags (CEC_SUBMIT_PACKED is a submit flag),
    exclusive default modes (RESILVER with VERIFY_ONLY) and bad shapes before any HIP call;
    without a device a valid request reports NoDevice (no host-side fallback pipeline).  CARRY
    goes with any default mode since ABI 3 (modes are per submit; only read submits keep
    chunks)."""
    import chunky_ec as ce
    rs = ce.ReedSolomon(10, 4)
    for args in [(1 << 20, 4, 2, 32), (1 << 20, 4, 2, 64), (1 << 20, 4, 2, 12),
                 (1 << 20, 4, 2, 16 | 12), (0, 4, 2, 0), (1 << 20, 0, 2, 0),
                 (1 << 20, 4, 0, 0),
                 (1 << 20, 4, 17, 0)]:
        with pytest.raises(ce.Error) as e:
            ce.ReadPipeline(rs, *args)
        assert e.value.code == ce.ERR_INVALID_ARGUMENT, args
    if ce.device_count() == 0:
        with pytest.raises(ce.Error) as e:
            ce.ReadPipeline(rs, 1 << 20, 4, 2, ce.ReadPipeline.REBUILT_ONLY)
        assert e.value.code == ce.ERR_NO_DEVICE
        for flags in (ce.ReadPipeline.REBUILT_ONLY | ce.ReadPipeline.CARRY,
                      ce.READ_RESILVER | ce.ReadPipeline.CARRY | ce.PIPE_EXTERNAL):
            with pytest.raises(ce.Error) as e:
                ce.ReadPipeline(rs, 1 << 20, 4, 2, flags)
            assert e.value.code == ce.ERR_NO_DEVICE


def test_synth_byte_host_mirror_is_deterministic():
    import chunky_ec as ce
    a = [ce.synth_byte(7, k, c, o) for k in range(3) for c in range(3) for o in (0, 1, 7, 8, 1000)]
    b = [ce.synth_byte(7, k, c, o) for k in range(3) for c in range(3) for o in (0, 1, 7, 8, 1000)]
    assert a == b and len(set(a)) > 10


def test_write_pipeline_and_multi_argument_checks_precede_device_use():
    """Shape / flag / device-list checks of cec_pipeline_new_ex and cec_multi_new come before any
    HIP call; without a device a valid request reports NoDevice (no host-side fallback)."""
    import chunky_ec as ce
    rs = ce.ReedSolomon(10, 4)
    for args in [(1 << 20, 4, 2, 1), (0, 4, 2, 0), (1 << 20, 0, 2, 0), (1 << 20, 4, 17, 0)]:
        with pytest.raises(ce.Error) as e:
            ce.Pipeline(rs, *args)
        assert e.value.code == ce.ERR_INVALID_ARGUMENT, args
    for devices in ([], list(range(65))):
        with pytest.raises(ce.Error) as e:
            ce.Multi(rs, 1 << 20, 4, 2, devices)
        assert e.value.code == ce.ERR_INVALID_ARGUMENT
    for kinds in (0, 4, ce.Multi.WRITE | 8):  # no job kind / an unknown one
        with pytest.raises(ce.Error) as e:
            ce.Multi(rs, 1 << 20, 4, 2, [0], kinds=kinds)
        assert e.value.code == ce.ERR_INVALID_ARGUMENT
    if ce.device_count() == 0:
        with pytest.raises(ce.Error) as e:
            ce.Multi(rs, 1 << 20, 4, 2, [0])
        assert e.value.code == ce.ERR_NO_DEVICE
        with pytest.raises(ce.Error) as e:
            ce.HostBuffer(4096)
        assert e.value.code == ce.ERR_NO_DEVICE
    # no scheduler: the job calls refuse it before anything else
    assert ce._lib.cec_multi_query(None, 1) == ce.ERR_INVALID_ARGUMENT
    assert ce._lib.cec_multi_wait(None, 1) == ce.ERR_INVALID_ARGUMENT


def test_product_library_has_no_attribution_kernels():
    """The A/B attribution modes (wrong outputs by design) are compiled only into the separate
    tools/ab build: the product library reports ab_tools=0."""
    import chunky_ec as ce
    assert ce.build_info().startswith("chunky_ec gfx950 ab_tools=0")


def test_decode_cache_bounded_without_device():
    """Decode matrices are built on the host before any device use, and the codec keeps at most
    4096 of them (least recently used evicted)."""
    import chunky_ec as ce
    if ce.device_count() != 0:
        pytest.skip("host-only check (the GPU variant is in test_gpu_multi.py)")
    rs = ce.ReedSolomon(20, 8)
    rng = np.random.default_rng(5)
    seen = set()
    while len(seen) < 4200:
        miss = tuple(sorted(rng.choice(28, 4, replace=False).tolist()))
        if miss in seen:
            continue
        seen.add(miss)
        shards = [None if i in miss else bytearray(b"x") for i in range(28)]
        with pytest.raises(ce.Error) as e:
            rs.reconstruct(shards)
        assert e.value.code == ce.ERR_NO_DEVICE
    assert rs.cached_patterns() == 4096


def test_part_encode_rejects_length_past_data_buf():
    """file_part.rs:150 asserts length <= data_buf.len(): the binding refuses before reading
    past the buffer (no device needed)."""
    import chunky_ec as ce
    rs = ce.ReedSolomon(3, 2)
    with pytest.raises(ValueError):
        ce.part_encode(rs, b"abcdef", 7)


def test_knobs_are_read_once_not_per_launch():
    """Every CEC_* knob is parsed in knobs.cpp into a snapshot (cec_reload_knobs re-reads it,
    test-only); no other engine source calls getenv, so a launch from a tokio worker never races
    a setenv elsewhere in the host process."""
    csrc = os.path.join(ROOT, "chunky-bits_amd", "csrc")
    offenders = []
    for name in sorted(os.listdir(csrc)):
        if name.endswith((".cpp", ".hip", ".hpp")) and name != "knobs.cpp":
            src = re.sub(r"//[^\n]*", "", open(os.path.join(csrc, name)).read())
            if "getenv" in src:
                offenders.append(name)
    assert not offenders, offenders
    import chunky_ec as ce
    ce.reload_knobs()  # host-only: parses the environment, touches no device
