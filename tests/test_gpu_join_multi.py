"""GPU parity of the multi-key inner join (plgpu_join_inner_multi) against
the oracle's row-encoding restatement (oracle.join_inner_multi, after
polars-ops/src/frame/join/mod.rs:625 prepare_keys_multiple) and the
multi-key golden cases of operations/test_join.py.

Bar: bit-exact pair sequences for the ordered modes, multisets for
maintain_order="none" (unspecified in the reference).
"""

import numpy as np
import pytest

import polaroid_amd as pl
from conftest import load_golden
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _frame(d):
    return pl.DataFrame([pl.Series(k, v, pl.Int64) for k, v in d.items()])


def test_join_multi_golden(gpu):
    for case in load_golden("join_multi_cases.json")["cases"]:
        left, right = _frame(case["left"]), _frame(case["right"])
        out = left.join(right, on=case["on"], **case["args"])
        if "expected_height" in case:
            assert out.height == case["expected_height"], case["name"]
            assert out.width == case["expected_width"], case["name"]
            continue
        cols = list(case["expected"])
        rows = list(zip(*[out[c].to_list() for c in out.columns]))
        if "post_filter" in case:
            c, op, v = case["post_filter"]
            j = out.columns.index(c)
            rows = [r for r in rows if r[j] is not None and r[j] <= v]
        got = [tuple(r[out.columns.index(c)] for c in cols) for r in rows]
        assert got == list(zip(*case["expected"].values())), case["name"]


def _keys(rng, n, card):
    a = rng.integers(0, card, n).astype(np.int64)
    b = rng.integers(-2, 2, n).astype(np.int32)
    bv = rng.random(n) > 0.1
    f = np.array([0.0, -0.0, np.nan, 2.5])[rng.integers(0, 4, n)]
    t = rng.random(n) < 0.5
    return [(a, None), (b, bv), (f, None), (t, None)]


def _df(keys, names, idxname):
    n = keys[0][0].shape[0]
    s = [pl.Series.from_numpy(nm, v, m) for nm, (v, m) in zip(names, keys)]
    s.append(pl.Series.from_numpy(idxname, np.arange(n, dtype=np.int64)))
    return pl.DataFrame(s)


@pytest.mark.parametrize("nl,nr,card", [(0, 10, 5), (10, 0, 5), (2000, 300, 40), (300, 2000, 40),
                                        (200003, 30000, 5000)])
@pytest.mark.parametrize("nkeys", [2, 4])
@pytest.mark.parametrize("nulls_equal", [False, True])
@pytest.mark.parametrize("order", ["none", "left", "right", "left_right", "right_left"])
@pytest.mark.parametrize("pack", [True, False])
def test_join_multi_pairs_vs_oracle(gpu, nl, nr, card, nkeys, nulls_equal, order, pack, plgpu_option):
    """Key sets without Float64 pack into one exact Int64 key; PLGPU_NO_PACK
    forces the hash + pair-verify path."""
    if not pack:
        plgpu_option("no_pack", 1)
    rng = np.random.default_rng(nl + 3 * nr + card + nkeys)
    lk, rk = _keys(rng, nl, card)[:nkeys], _keys(rng, nr, card)[:nkeys]
    names = ["a", "b", "f", "t"][:nkeys]
    ol, orr = O.join_inner_multi(lk, rk, nulls_equal)
    out = _df(lk, names, "li").join(_df(rk, names, "ri"), on=names, nulls_equal=nulls_equal, maintain_order=order)
    assert out.columns == names + ["li", "ri"]
    gl, gr = out["li"].to_numpy(), out["ri"].to_numpy()
    assert gl.shape == ol.shape
    if order in ("right", "right_left"):
        perm = np.lexsort((ol, orr))
        ol, orr = ol[perm], orr[perm]
    if order == "none":
        a = np.lexsort((gr, gl))
        gl, gr = gl[a], gr[a]
    assert np.array_equal(gl, ol) and np.array_equal(gr, orr)


def test_join_multi_validate_and_errors(gpu):
    left = pl.DataFrame({"a": [1, 1, 2], "b": [1, 2, 1], "x": [10, 20, 30]})
    right = pl.DataFrame({"a": [1, 1, 2], "b": [1, 2, 2], "y": [5, 6, 7]})
    out = left.join(right, on=["a", "b"], validate="1:1", maintain_order="left")
    assert out.rows() == [(1, 1, 10, 5), (1, 2, 20, 6)]
    dup = pl.DataFrame({"a": [1, 1], "b": [2, 2], "y": [1, 2]})
    with pytest.raises(pl.ComputeError, match="validation"):
        left.join(dup, on=["a", "b"], validate="m:1")
    left.join(dup, on=["a", "b"], validate="1:m")
    with pytest.raises(pl.InvalidOperationError):
        left.join(right, left_on=["a", "b"], right_on=["a"])
    f = pl.DataFrame({"a": pl.Series("a", [1.0, 2.0], pl.Float64), "b": [1, 2]})
    with pytest.raises(pl.InvalidOperationError, match="dtype"):
        left.join(f, on=["a", "b"])


def test_join_multi_left_right_on_and_collisions(gpu, plgpu_option):
    """Different key names per side; a forced 3-bit first hash must be
    caught by the pair verification and re-run."""
    plgpu_option("mk_collide", 1)
    plgpu_option("no_pack", 1)
    rng = np.random.default_rng(2)
    lk, rk = _keys(rng, 5000, 30), _keys(rng, 700, 30)
    ol, orr = O.join_inner_multi(lk[:3], rk[:3], False)
    left = _df(lk[:3], ["a", "b", "f"], "li")
    right = _df(rk[:3], ["p", "q", "r"], "ri")
    out = left.join(right, left_on=["a", "b", "f"], right_on=["p", "q", "r"], maintain_order="left_right",
                    validate="m:m")
    assert out.columns == ["a", "b", "f", "li", "ri"]
    assert np.array_equal(out["li"].to_numpy(), ol) and np.array_equal(out["ri"].to_numpy(), orr)
