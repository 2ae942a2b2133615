"""GPU parity of the multi-column sort (plgpu_arg_sort_multi) against the
oracle's restatement of arg_sort_multiple_impl (oracle.arg_sort_multi) and
the multi-column fixtures of operations/test_sort.py.

Bar: the permutation is bit-exact (the GPU sort is stable, so it equals the
reference's maintain_order=True result).
"""

import numpy as np
import pytest

import polaroid_amd as pl
from conftest import load_golden
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def test_sort_multi_golden(gpu):
    for case in load_golden("sort_multi_cases.json")["cases"]:
        df = pl.DataFrame([pl.Series(k, v, pl.Int64) for k, v in case["frame"].items()])
        out = df.sort(case["by"], **case["args"])
        for c, exp in case["expected"].items():
            assert out[c].to_list() == exp, (case["name"], c)


def _cols(rng, n):
    f = np.array([0.0, -0.0, 1.5, np.nan, -np.inf, np.inf])[rng.integers(0, 6, n)]
    i = rng.integers(-3, 3, n).astype(np.int64) * (1 << 40)
    j = rng.integers(0, 4, n).astype(np.int32)
    u = rng.integers(0, 3, n).astype(np.uint32)
    b = rng.random(n) < 0.5
    return {"f": (f, rng.random(n) > 0.1), "i": (i, None), "j": (j, rng.random(n) > 0.2), "u": (u, None),
            "b": (b, rng.random(n) > 0.1)}


@pytest.mark.parametrize("n", [0, 1, 100, 4097, 200_003])
@pytest.mark.parametrize("by", [("f", "i"), ("j", "f", "b"), ("u", "j", "i", "f", "b")])
@pytest.mark.parametrize("flags", [0, 1, 2, 3])
def test_sort_multi_vs_oracle(gpu, n, by, flags):
    rng = np.random.default_rng(n + len(by) + flags)
    cols = _cols(rng, n)
    desc = [bool((flags + k) & 1) for k in range(len(by))]
    nl = [bool(((flags >> 1) + k) & 1) for k in range(len(by))]
    df = pl.DataFrame([pl.Series.from_numpy(k, v, m) for k, (v, m) in cols.items()] +
                      [pl.Series.from_numpy("row", np.arange(n, dtype=np.int64))])
    out = df.sort(list(by), descending=desc, nulls_last=nl)
    perm = O.arg_sort_multi([cols[k] for k in by], desc, nl)
    assert np.array_equal(out["row"].to_numpy(), perm)
    assert out.columns == df.columns


def test_sort_multi_errors_and_lazy(gpu):
    df = pl.DataFrame({"a": [2, 1, 2], "b": [1, 2, 0]})
    with pytest.raises(ValueError, match="length of `descending`"):
        df.sort(["a", "b"], descending=[True])
    out = df.lazy().sort("a", "b", descending=[False, True]).collect()
    assert out.rows() == [(1, 2), (2, 1), (2, 0)]
    # a single Boolean column sorts through the multi-column path
    s = pl.DataFrame({"t": pl.Series("t", [True, None, False, True], pl.Boolean), "r": [0, 1, 2, 3]})
    assert s.sort("t")["r"].to_list() == [1, 2, 0, 3]
    assert s.sort("t", descending=True, nulls_last=True)["r"].to_list() == [0, 3, 2, 1]
