import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device; runs through the C-ABI")
    config.addinivalue_line("markers", "slow: long-running case")


def load_golden(name: str) -> dict:
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def unhex(v):
    """Decode a fixture value: float.hex strings -> float; lists recursively."""
    if isinstance(v, str):
        return float.fromhex(v)
    if isinstance(v, list):
        return [unhex(x) for x in v]
    return v


def check_rolling_case(got, case, tag=""):
    """One transcribed rolling assertion (tests/golden/rolling_cases.json)
    against `got` (a list, None for null outputs)."""
    import math

    def same(g, e):
        if e is None or g is None:
            return g is None and e is None
        if isinstance(e, float) and math.isnan(e):
            return isinstance(g, float) and math.isnan(g)
        if case.get("approx"):
            return math.isclose(g, e, rel_tol=1e-6, abs_tol=1e-12)
        return g == e

    name = (case["name"], tag)
    if "round" in case:
        got = [None if g is None else round(g, case["round"]) for g in got]
    if "expected_null_count" in case:
        assert sum(g is None for g in got) == case["expected_null_count"], name
        assert sum(g is None or g != g for g in got) == case["expected_nan_or_null"], name
    elif "expected_last" in case:
        assert got[-1] == case["expected_last"], name
    elif "expected_sum" in case:
        assert sum(g for g in got if g is not None) == case["expected_sum"], (name, got)
    elif "expected_at" in case:
        i, e = case["expected_at"]
        assert same(got[i], unhex(e) if isinstance(e, str) else e), (name, got)
    else:
        exp = [unhex(v) if isinstance(v, str) else v for v in case["expected"]]
        assert len(got) == len(exp) and all(same(g, e) for g, e in zip(got, exp)), (name, got, exp)


@pytest.fixture
def plgpu_option():
    """Set library options (plgpu_set_option test hooks) for one test; every
    option touched is restored afterwards."""
    from polaroid_amd import _native as N

    saved = []

    def setter(name, value):
        saved.append((name, N.set_option(name, value)))

    yield setter
    for name, prev in reversed(saved):
        N.set_option(name, prev)


@pytest.fixture(autouse=True)
def _checked_build_invariants(request):
    """Under the checked library (PLGPU_LIB=...checked.so), every GPU test
    ends by reading the kernels' violated-invariant bits: any is a failure."""
    yield
    if "checked" not in os.environ.get("PLGPU_LIB", "") or request.node.get_closest_marker("gpu") is None:
        return
    import ctypes as C

    from polaroid_amd import _native as N

    bits = C.c_uint32(0)
    N.check(N.lib().plgpu_debug_checks(C.byref(bits)))
    assert bits.value == 0, f"kernel index invariants violated: bits {bits.value:#x} (groupby.hip CK_*)"


@pytest.fixture(scope="session")
def gpu():
    """Skip-free guard: a GPU test must run on a device; fail loudly otherwise."""
    import polaroid_amd as pl

    n = pl.device_count()
    assert n > 0, "no HIP device visible: -m gpu tests must run on an MI355X"
    return n
