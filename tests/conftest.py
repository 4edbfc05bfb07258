import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "chunky-bits_amd"), os.path.dirname(os.path.abspath(__file__))):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: full-size (BASELINE config) GPU cases")


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "golden_vectors.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def kats():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "crate_kats.json")) as f:
        return json.load(f)


@pytest.fixture
def knob_env(monkeypatch):
    """Sets CEC_* engine knobs for one test.  The library reads its knobs once per process
    (cec_reload_knobs, include/chunky_ec.h), so every change reloads them, and teardown restores
    the environment and reloads again."""
    import chunky_ec as ce

    class _KnobEnv:
        def set(self, name, value):
            monkeypatch.setenv(name, value)
            ce.reload_knobs()

        def delenv(self, name):
            monkeypatch.delenv(name, raising=False)
            ce.reload_knobs()

    yield _KnobEnv()
    monkeypatch.undo()
    ce.reload_knobs()
