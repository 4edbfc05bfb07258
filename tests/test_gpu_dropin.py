"""tools/dropin_cp_repair.py on the GPU (cp / cat / repair of a 22 MiB file in the reference's
on-disk format through the batched loops and the scheduler's resilver): the file reads back
equal to its input, every deleted or damaged chunk file is rewritten with bytes that hash to its
metadata digest, and the FileReference the engine wrote -- parity digests included -- equals the
oracle's for the same input.  (The reference's own reader reads such a store in the build
container: tests/golden/make_dropin_record.py, checked by tests/test_format_fixture.py.)"""
import hashlib
import json
import os
import subprocess
import sys

import pytest
import yaml

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import make_format_fixture as fx  # noqa: E402  (oracle slicing)
from _gen import gen_bytes  # noqa: E402


def test_dropin_cp_cat_repair(tmp_path):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "dropin_cp_repair.py"),
                          str(tmp_path)], capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    s = json.load(open(tmp_path / "summary.json"))
    assert s["cat_equals_input"] is True and s["cat_after_repair_equals_input"] is True
    # the stale file: p + 1 chunks per part listed [bad, good], read / verified / not rebuilt
    assert s["stale"]["cat_equals_input"] is True and s["stale"]["repaired"] == []
    assert sorted(x[:2] for x in s["stale"]["verify"]["invalid"]) == \
        sorted(s["stale"]["stale_chunks"])
    ref = yaml.safe_load(open(tmp_path / "file.yaml"))
    data = gen_bytes(s["seed"], s["length"])
    assert s["input_sha256"] == hashlib.sha256(data.tobytes()).hexdigest()
    for k, (L, chunks) in enumerate(fx.parts_of(data, s["d"], s["p"], s["chunk_size"])):
        part = ref["parts"][k]
        assert part["chunksize"] == L
        for c, entry in zip(chunks, part["data"] + part["parity"]):
            h = hashlib.sha256(c.tobytes()).hexdigest()
            assert entry["sha256"] == h, (k, entry)
            # every chunk file exists after the repair and holds exactly that chunk; a repaired
            # chunk lists its rewritten location a second time (appended, file_part.rs:346)
            assert open(tmp_path / f"sha256-{h}", "rb").read() == c.tobytes(), (k, h)
            assert set(entry["locations"]) == {f"sha256-{h}"}
            assert len(entry["locations"]) == (2 if [k, (part["data"] + part["parity"]).index(
                entry)] in s["repaired"] else 1)
