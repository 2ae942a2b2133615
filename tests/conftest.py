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
