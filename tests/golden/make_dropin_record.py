"""Record the reference's own reader on a store the ENGINE wrote and repaired.

Run in the build container (it executes /root/reference/python/chunky-bits.py, which does not
exist on the GPU box), after tools/dropin_cp_repair.py ran on the GPU box and its store came back
in gpurun_out/dropin/:

    python tests/golden/make_dropin_record.py [gpurun_out/dropin]

The GPU side cut the file into parts with the batched writer, stored every chunk as a
`sha256-<hex>` file with a FileReference YAML, deleted one data and one parity chunk of two parts
and damaged a third part's data chunk, read the file back through the batched reader and
repaired the store through the scheduler's resilver.  Here the reference's python/chunky-bits.py
reads that YAML: it checks every data chunk's SHA-256 (mismatches go to stderr), truncates to
`length` and writes the file to stdout.  Committed:

* tests/golden/dropin_file_reference.yaml -- the FileReference the engine wrote;
* tests/golden/dropin_reference_run.json -- the reader's exit status, stdout length / SHA-256 and
  stderr on the repaired store, the GPU side's summary (what was deleted, damaged, read back and
  repaired), and a control run with one data chunk flipped again.

tests/test_format_fixture.py checks the record, and that the YAML -- data AND parity digests --
equals the oracle's FileReference for the same input (tests/_gen.py gen_bytes).
"""
import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REFERENCE_SCRIPT = "/root/reference/python/chunky-bits.py"


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "dropin")
    summary = json.load(open(os.path.join(src, "summary.json")))
    with tempfile.TemporaryDirectory() as tmp:
        for f in os.listdir(src):
            if os.path.isfile(os.path.join(src, f)):
                shutil.copy(os.path.join(src, f), tmp)
        shutil.copytree(os.path.join(src, "stale"), os.path.join(tmp, "stale"))
        run = subprocess.run([sys.executable, REFERENCE_SCRIPT, "file.yaml"], cwd=tmp,
                             capture_output=True, check=False)
        # stale.yaml lists p + 1 chunks per part as [stale copy, good copy]; the reference's python
        # reader checks only each data chunk's first location, so it must name exactly the data
        # chunks whose first copy is stale (the engine's reader walked on to the good copy)
        stale_run = subprocess.run([sys.executable, REFERENCE_SCRIPT, "stale.yaml"], cwd=tmp,
                                   capture_output=True, check=False)
        import yaml
        ref = yaml.safe_load(open(os.path.join(tmp, "file.yaml")))
        bad = os.path.join(tmp, ref["parts"][2]["data"][0]["locations"][0])
        with open(bad, "r+b") as fh:
            b = fh.read(1)
            fh.seek(0)
            fh.write(bytes([b[0] ^ 0x01]))
        control = subprocess.run([sys.executable, REFERENCE_SCRIPT, "file.yaml"], cwd=tmp,
                                 capture_output=True, check=False)
        shutil.copy(os.path.join(src, "file.yaml"),
                    os.path.join(HERE, "dropin_file_reference.yaml"))
        stale_ref = yaml.safe_load(open(os.path.join(tmp, "stale.yaml")))
    record = {
        "script": "python/chunky-bits.py (the reference's own reader, run in the build container "
                  "by tests/golden/make_dropin_record.py) on the store tools/dropin_cp_repair.py "
                  "wrote and repaired on the GPU",
        "gpu_side": summary,
        "returncode": run.returncode,
        "stdout_len": len(run.stdout),
        "stdout_sha256": hashlib.sha256(run.stdout).hexdigest(),
        "stderr": run.stderr.decode(errors="replace"),
        "corrupted_control": {
            "what": "part 2, data chunk 0, first byte flipped after the repair",
            "stderr_lines": len(control.stderr.decode().strip().splitlines()),
            "stderr_names_the_chunk": ref["parts"][2]["data"][0]["sha256"] in
            control.stderr.decode(),
            "stdout_sha256_differs": hashlib.sha256(control.stdout).hexdigest() !=
            hashlib.sha256(run.stdout).hexdigest()},
        "stale_file": {
            "what": "stale.yaml: p + 1 chunks per part listed [stale copy, good copy]; the "
                    "reader checks data chunks' first location only",
            "returncode": stale_run.returncode,
            "stderr_lines": stale_run.stderr.decode().strip().splitlines(),
            "stale_data_chunks": [[k, i] for k, i in summary["stale"]["stale_chunks"] if i < 3],
            "stale_data_hashes": [stale_ref["parts"][k]["data"][i]["sha256"]
                                  for k, i in summary["stale"]["stale_chunks"] if i < 3]},
    }
    with open(os.path.join(HERE, "dropin_reference_run.json"), "w") as fh:
        json.dump(record, fh, indent=1)
        fh.write("\n")
    print(json.dumps(record, indent=1))
    st = record["stale_file"]
    assert sorted(line.split(" != ")[0] for line in st["stderr_lines"]) == \
        sorted(st["stale_data_hashes"]), "reference reader and the stale copies disagree"
    assert run.returncode == 0 and not run.stderr and \
        record["stdout_sha256"] == summary["input_sha256"], "reference reader disagrees"


if __name__ == "__main__":
    main()
