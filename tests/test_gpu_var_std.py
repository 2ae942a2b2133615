"""GPU parity of the std() / var() group-by aggregations (polars-expr/src/
reduce/var_std.rs; finalize at polars-compute/src/moment.rs:126: null when
the group's non-null count <= ddof, else M2 / (count - ddof), std = sqrt).
The checker is a two-pass restatement with math.fsum per group.  Tolerance:
1e-12 relative (+1e-300 absolute) — the reference's Welford merge and the
executor's two exact passes round differently; validity is exact."""

import math

import numpy as np
import pytest

import polaroid_amd as pl

pytestmark = pytest.mark.gpu


def _oracle(key, x, valid, ddof, sel):
    """Per group (first-occurrence order of selected rows): var, std, valid."""
    order, groups = [], {}
    for r in np.flatnonzero(sel):
        k = int(key[r])
        if k not in groups:
            groups[k] = []
            order.append(k)
        if valid[r]:
            groups[k].append(float(x[r]))
    var, ok = [], []
    for k in order:
        v = groups[k]
        if len(v) <= ddof:
            var.append(0.0)
            ok.append(False)
            continue
        m = math.fsum(v) / len(v)
        var.append(max(math.fsum((a - m) * (a - m) for a in v) / (len(v) - ddof), 0.0))
        ok.append(True)
    var = np.array(var)
    return np.array(order, dtype=np.int64), var, np.sqrt(var), np.array(ok, dtype=bool)


def _close(got, want, ok):
    assert np.allclose(got[ok], want[ok], rtol=1e-12, atol=1e-300)


@pytest.mark.parametrize("n,card", [(1, 1), (50, 7), (100_003, 100), (60_001, 20_000)])
@pytest.mark.parametrize("ddof", [0, 1, 2])
@pytest.mark.parametrize("pred", [False, True])
def test_var_std_vs_oracle(gpu, n, card, ddof, pred):
    rng = np.random.default_rng(n + card + 10 * ddof + pred)
    key = rng.integers(0, card, n).astype(np.int64)
    x = rng.standard_normal(n) * 1e3 + 5e6  # large mean: catastrophic for one-pass formulas
    xv = rng.random(n) > 0.15
    i = rng.integers(-1000, 1000, n).astype(np.int64)
    df = pl.DataFrame({"k": pl.Series.from_numpy("k", key), "x": pl.Series.from_numpy("x", x, xv),
                       "i": pl.Series.from_numpy("i", i)})
    lf = df.lazy()
    sel = np.ones(n, dtype=bool)
    if pred:
        lf = lf.filter(pl.col("i") > -300)
        sel = i > -300
    out = (lf.group_by("k", maintain_order=True)
           .agg(pl.col("x").var(ddof).alias("xv"), pl.col("x").sum().alias("xs"),
                pl.col("x").std(ddof).alias("xsd"), pl.col("i").std(ddof).alias("isd"))
           .collect())
    keys, var, std, ok = _oracle(key, x, xv, ddof, sel)
    assert out.columns == ["k", "xv", "xs", "xsd", "isd"]
    assert np.array_equal(out["k"].to_numpy(), keys)
    assert np.array_equal(out["xv"].validity_numpy(), ok)
    assert np.array_equal(out["xsd"].validity_numpy(), ok)
    _close(out["xv"].to_numpy(), var, ok)
    _close(out["xsd"].to_numpy(), std, ok)
    _, _, istd, iok = _oracle(key, i.astype(np.float64), np.ones(n, bool), ddof, sel)
    assert np.array_equal(out["isd"].validity_numpy(), iok)
    _close(out["isd"].to_numpy(), istd, iok)


def test_var_null_keys_and_constant_groups(gpu):
    k = np.array([1, 0, 1, 0, 2, 2, 2], dtype=np.int64)
    km = np.array([1, 0, 1, 0, 1, 1, 1], dtype=bool)
    x = np.array([3.0, 1.0, 3.0, 4.0, 7.0, 7.0, 7.0])
    df = pl.DataFrame({"k": pl.Series.from_numpy("k", k, km), "x": pl.Series.from_numpy("x", x)})
    out = df.lazy().group_by("k", maintain_order=True).agg(pl.col("x").var()).collect()
    assert out["k"].validity_numpy().tolist() == [True, False, True]
    v = out["x"].to_numpy()
    assert v[0] == 0.0 and v[2] == 0.0 and v[1] == 4.5


@pytest.mark.parametrize("kind", ["multi", "string", "u32_nullkey"])
def test_var_std_key_kinds(gpu, kind):
    """The join-composed path (multi-key, String keys) and the direct
    group-key-table path with a nullable UInt32 key."""
    rng = np.random.default_rng(len(kind))
    n = 40_000
    a = rng.integers(0, 30, n).astype(np.int64)
    b = rng.integers(0, 4, n).astype(np.int64)
    x = rng.standard_normal(n) * 10 + 1e4
    if kind == "multi":
        df = pl.DataFrame({"a": pl.Series.from_numpy("a", a), "b": pl.Series.from_numpy("b", b),
                           "x": pl.Series.from_numpy("x", x)})
        key, gk = ["a", "b"], a * 4 + b
    elif kind == "string":
        names = np.array([f"name-{v:03d}-longer-than-seven" for v in a], dtype=object)
        df = pl.DataFrame({"s": pl.Series("s", names.tolist()), "x": pl.Series.from_numpy("x", x)})
        key, gk = "s", a
    else:
        km = rng.random(n) > 0.05
        df = pl.DataFrame({"u": pl.Series.from_numpy("u", a.astype(np.uint32), km),
                           "x": pl.Series.from_numpy("x", x)})
        key, gk = "u", np.where(km, a, -1)
    out = df.lazy().group_by(key, maintain_order=True).agg(pl.col("x").std(), pl.col("x").var(0).alias("v0")).collect()
    keys, var, std, ok = _oracle(gk, x, np.ones(n, bool), 1, np.ones(n, bool))
    _, var0, _, ok0 = _oracle(gk, x, np.ones(n, bool), 0, np.ones(n, bool))
    assert out.height == len(keys)
    assert np.array_equal(out["x"].validity_numpy(), ok)
    _close(out["x"].to_numpy(), std, ok)
    _close(out["v0"].to_numpy(), var0, ok0)


@pytest.mark.parametrize("dt", [np.int32, np.uint32, np.int64])
def test_var_std_integer_sums_past_input_width(gpu, dt):
    """Groups whose integer sum overflows the column's width: the group mean
    comes from the exact f64 sum, so three rows of 2e9 (Int32 / UInt32) have
    variance 0, not ~2e18 from a wrapped sum (var_std.rs casts to f64)."""
    big = {np.int32: 2_000_000_000, np.uint32: 4_000_000_000, np.int64: 4_000_000_000_000_000_000}[dt]
    key = np.array([0, 0, 0, 1, 1, 2], np.int64)
    x = np.array([big, big, big, big, big - 2, 7], dt)
    df = pl.DataFrame({"k": pl.Series.from_numpy("k", key), "x": pl.Series.from_numpy("x", x)})
    out = df.group_by("k", maintain_order=True).agg(pl.col("x").var().alias("v"), pl.col("x").std(0).alias("s"))
    xs = x.astype(np.float64)
    want_v = [0.0, float(np.var(xs[3:5], ddof=1)), None]
    got_v = out["v"].to_list()
    assert got_v[0] == 0.0 and got_v[2] is None
    assert abs(got_v[1] - want_v[1]) <= 1e-12 * abs(want_v[1])
    assert out["s"].to_list()[0] == 0.0 and out["s"].to_list()[2] == 0.0
