"""The per-call tier's idle staging on the GPU: cec_release_cached frees the idle contexts'
HBM (the pool kept up to 1 GiB per device for the process lifetime) and the
next call makes new ones; results are unchanged.  Knob reloads (cec_reload_knobs) between
calls leave results unchanged too."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

import chunky_ec as ce  # noqa: E402
import oracle  # noqa: E402


def _encode(rs, data, L):
    parity = [bytearray(L) for _ in range(4)]
    rs.encode_sep([d.tobytes() for d in data], parity)
    return [bytes(x) for x in parity]


def test_release_cached_frees_idle_staging_and_calls_still_work():
    rs = ce.ReedSolomon(10, 4)
    L = 1 << 20
    data = list(np.random.default_rng(3).integers(0, 256, size=(10, L), dtype=np.uint8))
    st, want = oracle.encode_sep(10, 4, data)
    assert st == 0
    first = _encode(rs, data, L)
    freed = ce.release_cached(0)
    assert freed >= 10 * L  # at least the call's device staging (data + parity) was idle
    assert ce.release_cached(-1) == 0  # nothing idle left on any device
    second = _encode(rs, data, L)
    assert first == second == [w.tobytes() for w in want]


def test_knob_reload_between_calls_keeps_results(knob_env):
    rs = ce.ReedSolomon(10, 4)
    L = 65536
    data = list(np.random.default_rng(4).integers(0, 256, size=(10, L), dtype=np.uint8))
    base = _encode(rs, data, L)
    for name, val in (("CEC_APPLY_BS", "0"), ("CEC_COALESCE_US", "0"),
                      ("CEC_COALESCE_INFLIGHT", "1")):
        knob_env.set(name, val)
        assert _encode(rs, data, L) == base, name
    ce.reload_knobs()
    assert _encode(rs, data, L) == base
