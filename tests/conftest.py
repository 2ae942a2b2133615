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


@pytest.fixture(scope="session")
def gpu():
    """Skip-free guard: a GPU test must run on a device; fail loudly otherwise."""
    import polaroid_amd as pl

    n = pl.device_count()
    assert n > 0, "no HIP device visible: -m gpu tests must run on an MI355X"
    return n
