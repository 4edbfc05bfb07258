"""bench.py's JSON contract on the GPU, at a small size (a subprocess, as the driver runs it):
one line with the BASELINE metric, the roofline / VALU-roofline / north_star blocks and the CPU
baseline, every GPU-side check in it true.  The full-size line is the driver's own run."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT,
                         capture_output=True, text=True, timeout=150)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [x for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


def test_default_line_contract_small():
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    line = _run("--parts", "256", "--steps", "2", "--warmup", "1", "--e2e-gib", "0")
    assert line["metric"] == base["metric"]
    assert line["unit"] == "GB/s" and line["n_gpus"] == 1 and line["steps"] == 2
    assert line["higher_is_better"] is True and line["scaling"] == "weak"
    assert line["dtype"] == "u8" and line["value"] > 0 and line["ms_per_step"] > 0
    assert line["config"]["parts_per_gpu"] == 256 and line["config"]["d"] == 10
    rf = line["roofline"]
    assert rf["bound"] == "hbm" and rf["kernel"] == "encode_hash_kernel" and 0 < rf["frac"] < 1
    assert line["valu_roofline"]["bound"] == "valu"
    ns = line["north_star"]
    assert ns["rebuilt_data_verified"] is True
    assert ns["encode"]["kernel"] == "rs_encode_bs_kernel" and ns["encode"]["frac"] > 0
    assert ns["reconstruct_data_2_erasures"]["frac"] > 0
    cb = line["cpu_baseline"]
    assert cb["value"] > 0 and cb["kind"] == "port" and cb["cores"] >= 1
    bc = line["baseline_configs"]  # C3 on the headline's buffer, C4 scaled to 256 parts
    assert bc["c3_reconstruct"]["rebuilt_verified"] is True
    assert bc["c4_encode_hash"]["round_trip_verified"] is True
    assert bc["c4_encode_hash"]["traffic"] is None  # no committed PMC figure at this size
    assert line["check_vs_oracle"] is True
    assert all(line["check_vs_oracle_detail"]["checks"].values())


def test_reconstruct_config_line_small():
    line = _run("--config", "c3e2", "--parts", "128", "--steps", "2", "--warmup", "1",
                "--check", "--no-cpu-baseline")
    assert line["check_vs_oracle"] is True
    assert line["roofline"]["kernel"] == "rs_apply_kernel(reconstruct_data)"
    assert line["kernels"]["also_reconstruct"]["ms"] > 0


def test_default_line_checks_vs_oracle_small():
    """The default line's oracle leg on its own buffers (headline fused kernel, north_star's
    bit-sliced re-encode, C3 and C4 scaled to --parts) and the whole-batch digest checks."""
    line = _run("--parts", "64", "--steps", "1", "--warmup", "1", "--e2e-gib", "0")
    assert line["check_vs_oracle"] is True
    det = line["check_vs_oracle_detail"]["checks"]
    assert det["headline"] is True and det["north_star_encode"] is True
    # every part of the C2 buffer (after north_star's and C3's rebuilds) and of C4's (after its
    # round trip): parity vs the oracle's encode of the data, 14 / 28 digests vs the fused
    # kernel's (C4 scaled with --parts: 64 parts)
    det_all = line["check_vs_oracle_detail"]
    assert det["c2_all_parts"] is True and det["c4_all_parts"] is True
    assert det_all["c2_all_parts_checked"] == {"parts": 64, "digests": 64 * 14}
    assert det_all["c4_all_parts_checked"] == {"parts": 64, "digests": 64 * 28}
    assert det_all["c2_all_parts_mismatched"] == det_all["c4_all_parts_mismatched"] == []


def test_end_to_end_read_repair_small():
    """end_to_end at 3 GiB: the ring-fed write form and the read_repair form with 2 % damaged
    fetches, every damaged chunk rejected and its part retried, nothing undecodable."""
    line = _run("--parts", "64", "--steps", "1", "--warmup", "1", "--e2e-gib", "3",
                "--no-north-star", "--no-cpu-baseline", "--corrupt", "0.02")
    e2e = line["end_to_end"]
    assert e2e["value"] > 0 and e2e["sampled_digest_matches_source"] is True
    rr = e2e["read_repair"]
    assert rr["value"] > 0 and rr["sampled_parts_equal_stored"] is True
    assert rr["undecodable_parts"] == 0 and rr["retries"] > 0
    assert rr["rejected_chunks"] == rr["damaged_loads"] > 0
    assert any(c["attempts"] > 1 for c in rr["checks"])


def test_end_to_end_write_stream_checked_whole():
    """With the cpu_baseline leg on, every part of end_to_end's ring-fed write stream is checked
    against the oracle (3 GiB asked; the stream is at least 4 batches: 1 024 parts; the ring's
    wrap-around is covered on the CPU, tests/test_bench_host.py)."""
    line = _run("--parts", "64", "--steps", "1", "--warmup", "1", "--e2e-gib", "3",
                "--no-north-star")
    det = line["check_vs_oracle_detail"]
    n = (3 << 30) // (10 << 20)
    assert det["checks"]["end_to_end_all_parts"] is True and line["check_vs_oracle"] is True
    assert det["end_to_end_all_parts_checked"] == {"parts": max(n, 4 * 256), "digests":
                                                   max(n, 4 * 256) * 14}
    assert det["end_to_end_all_parts_mismatched"] == []


def test_stream_configs_small():
    """C5 and its verify/repair side at 4 GiB, fed from the pageable rings inside the timed
    region."""
    line = _run("--config", "c5", "--stream-gib", "4", "--check")
    assert line["check_digests_vs_source"] is True and line["value"] > 0
    # --check: every part of the stream re-derived through the oracle
    whole = line["check_all_parts_vs_oracle"]
    assert whole["ok"] is True and whole["parts"] == (4 << 30) // (10 << 20)
    assert line["config"]["stream_bytes"] == (4 << 30) // (10 << 20) * (10 << 20)
    line = _run("--config", "c5r", "--stream-gib", "4", "--corrupt", "0.02")
    rr = line["read_repair"]
    assert line["check_vs_stored"] is True and line["value"] > 0
    assert rr["undecodable_parts"] == 0 and rr["retried_parts"] > 0
    assert rr["rejected_chunks"] == rr["damaged_loads"] > 0
    assert rr["parts"] == (4 << 30) // (10 << 20)
