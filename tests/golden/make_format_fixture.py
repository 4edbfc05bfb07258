"""Generate the C1 format fixture, checked by the reference's OWN reader script.

Run in the build container only (it executes /root/reference/python/chunky-bits.py, which does
not exist on the GPU box):

    python tests/golden/make_format_fixture.py

C1 (BASELINE.json configs[0]): a 50 MiB file, d=3, p=2, 1 MiB chunks -> 16 full parts and one
part of 699 051-byte chunks.  The file is cut into parts exactly as FileWriteBuilder::write and
FilePart::write_with_encoder do (writer.rs:170-197: part = min(d*chunk_size, remaining) bytes in
a zeroed d*chunk_size buffer; file_part.rs:150-158: L = ceil(part/d), data chunk j = buf[L*j ..
L*(j+1)]), parity comes from the oracle (oracle/cec_oracle.c) and every chunk is hashed (oracle
SHA-256, cross-checked with hashlib).  The chunks are written as files named `sha256-<hex>`
(location.rs:612) and described by a FileReference YAML in the reference's serde layout
(file_reference.rs:39-46: length, parts; file_part.rs:57-65: chunksize, data, parity;
chunk.rs:10-17 + any.rs:54-58: the flattened lowercase `sha256` hash + locations).

The reference's python/chunky-bits.py then reads the YAML: it checks each data chunk's SHA-256
against the metadata (mismatches go to stderr), truncates to `length` and writes the file to
stdout.  Committed:

* tests/golden/c1_file_reference.yaml -- the metadata the script read (relative locations);
* tests/golden/c1_reference_run.json  -- the script's exit status, stdout length and SHA-256,
  and its stderr (must be empty), with the input's definition.

tests/test_format_fixture.py checks the oracle against the YAML on the CPU, and the engine's
part slicing, chunk sizes, digests and data bytes against it on the GPU.  What this pins: the
in-order data-then-parity layout, the `sha256` hex digests, the per-part chunk size and the
length truncation, by the reference's own code.  It does NOT pin RS parity bytes (the script
reads data chunks only); the parity digests in the YAML are the oracle's.
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

import numpy as np  # noqa: E402
import yaml  # noqa: E402

import oracle  # noqa: E402
from _gen import gen_bytes  # noqa: E402

REFERENCE_SCRIPT = "/root/reference/python/chunky-bits.py"
SEED, LENGTH, D, P, CHUNK = 0xC1, 50 << 20, 3, 2, 1 << 20


def c1_input() -> np.ndarray:
    return gen_bytes(SEED, LENGTH)


def parts_of(data: np.ndarray, d: int, p: int, chunk: int):
    """(L, [d+p chunks as numpy arrays]) per part, as writer.rs + file_part.rs cut them."""
    out = []
    for off in range(0, len(data), d * chunk):
        n = min(d * chunk, len(data) - off)
        buf = np.zeros(d * chunk, np.uint8)
        buf[:n] = data[off:off + n]
        L = (n + d - 1) // d
        chunks = [buf[j * L:(j + 1) * L] for j in range(d)]
        st, par = oracle.encode_sep(d, p, chunks)
        assert st == 0
        out.append((L, chunks + list(par)))
    return out


def file_reference(data: np.ndarray) -> dict:
    parts = []
    for L, chunks in parts_of(data, D, P, CHUNK):
        hexes = []
        for c in chunks:
            h = oracle.sha256(c).hex()
            assert h == hashlib.sha256(c.tobytes()).hexdigest()
            hexes.append(h)
        parts.append({
            "chunksize": L,
            "data": [{"sha256": h, "locations": [f"sha256-{h}"]} for h in hexes[:D]],
            "parity": [{"sha256": h, "locations": [f"sha256-{h}"]} for h in hexes[D:]],
        })
    return {"length": LENGTH, "parts": parts}


def main():
    data = c1_input()
    ref = file_reference(data)
    with tempfile.TemporaryDirectory() as tmp:
        for L, chunks in parts_of(data, D, P, CHUNK):
            for c in chunks:
                with open(os.path.join(tmp, f"sha256-{hashlib.sha256(c.tobytes()).hexdigest()}"),
                          "wb") as fh:
                    fh.write(c.tobytes())
        yml = os.path.join(tmp, "c1.yaml")
        with open(yml, "w") as fh:
            yaml.safe_dump(ref, fh, sort_keys=False)
        run = subprocess.run([sys.executable, REFERENCE_SCRIPT, "c1.yaml"], cwd=tmp,
                             capture_output=True, check=False)
        # negative control: one flipped byte in part 5's data chunk 1 must be reported on
        # stderr (so the empty stderr above means every data chunk was checked)
        bad = os.path.join(tmp, ref["parts"][5]["data"][1]["locations"][0])
        with open(bad, "r+b") as fh:
            b = fh.read(1)
            fh.seek(0)
            fh.write(bytes([b[0] ^ 0x01]))
        control = subprocess.run([sys.executable, REFERENCE_SCRIPT, "c1.yaml"], cwd=tmp,
                                 capture_output=True, check=False)
        with open(yml) as fi, open(os.path.join(HERE, "c1_file_reference.yaml"), "w") as fo:
            fo.write(fi.read())
    result = {
        "script": "python/chunky-bits.py (the reference's own reader, run in the build "
                  "container by tests/golden/make_format_fixture.py)",
        "input": f"tests/_gen.py gen_bytes({SEED:#x}, {LENGTH}): C1, d={D}, p={P}, "
                 f"chunk_size={CHUNK}",
        "returncode": run.returncode,
        "stdout_len": len(run.stdout),
        "stdout_sha256": hashlib.sha256(run.stdout).hexdigest(),
        "stderr": run.stderr.decode(errors="replace"),
        "input_sha256": hashlib.sha256(data.tobytes()).hexdigest(),
        "corrupted_control": {
            "what": "part 5, data chunk 1, first byte flipped",
            "stderr_lines": len(control.stderr.decode().strip().splitlines()),
            "stderr_names_the_chunk": ref["parts"][5]["data"][1]["sha256"] in
            control.stderr.decode(),
            "stdout_sha256_differs": hashlib.sha256(control.stdout).hexdigest() !=
            hashlib.sha256(run.stdout).hexdigest()},
        "parts": len(ref["parts"]),
        "last_chunksize": ref["parts"][-1]["chunksize"],
    }
    with open(os.path.join(HERE, "c1_reference_run.json"), "w") as fh:
        json.dump(result, fh, indent=1)
        fh.write("\n")
    print(json.dumps(result, indent=1))
    assert run.returncode == 0 and not run.stderr and result["stdout_sha256"] == \
        result["input_sha256"], "the reference's reader did not reproduce the file"


if __name__ == "__main__":
    main()
