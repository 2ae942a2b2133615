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


def _exact_var(vals, ddof):
    """The exact variance of the f64 values (rational arithmetic), rounded once."""
    from fractions import Fraction

    fv = [Fraction(float(v)) for v in vals]
    n = len(fv)
    s1 = sum(fv)
    s2 = sum(v * v for v in fv)
    return float((n * s2 - s1 * s1) / (n * (n - ddof)))


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


def _var_frame(rng, n, card, nulls=True):
    key = rng.integers(0, card, n).astype(np.int64)
    x = rng.standard_normal(n) * 1e3 + 5e6  # large mean: catastrophic for a rounded one-pass formula
    y = rng.uniform(-5, 5, n)
    xv = (rng.random(n) > 0.15) if nulls else np.ones(n, bool)
    return key, x, y, xv


@pytest.mark.parametrize("n,card", [(1, 1), (50, 7), (100_003, 100), (60_001, 20_000), (1_000_003, 300)])
@pytest.mark.parametrize("ddof", [0, 1, 2])
@pytest.mark.parametrize("pred", [False, True])
def test_var_std_fused_vs_exact(gpu, n, card, ddof, pred):
    """var / std in one pass (exact sums of x and of x * x's two parts,
    combined exactly per group): within 1e-12 of the exact two-pass checker,
    validity exact, the fused path taken (info["var_path"])."""
    rng = np.random.default_rng(n + card + 7 * ddof + pred)
    key, x, y, xv = _var_frame(rng, n, card)
    df = pl.DataFrame({"k": pl.Series.from_numpy("k", key), "x": pl.Series.from_numpy("x", x, xv),
                       "y": pl.Series.from_numpy("y", y)})
    lf = df.lazy()
    sel = np.ones(n, dtype=bool)
    if pred:
        lf = lf.filter(pl.col("y") > -1.0)
        sel = y > -1.0
    info = {}
    out = (lf.group_by("k", maintain_order=True)
           .agg(pl.col("x").var(ddof).alias("xv"), pl.col("x").std(ddof).alias("xsd"),
                pl.col("y").var(ddof).alias("yv"), pl.col("x").mean().alias("xm"))
           .collect(info=info))
    assert info["var_path"] == "fused", info
    keys, var, std, ok = _oracle(key, x, xv, ddof, sel)
    assert np.array_equal(out["k"].to_numpy(), keys)
    assert np.array_equal(out["xv"].validity_numpy(), ok)
    _close(out["xv"].to_numpy(), var, ok)
    _close(out["xsd"].to_numpy(), std, ok)
    _, yvar, _, yok = _oracle(key, y, np.ones(n, bool), ddof, sel)
    assert np.array_equal(out["yv"].validity_numpy(), yok)
    _close(out["yv"].to_numpy(), yvar, yok)


def test_var_fused_exact_cases(gpu):
    """Constant groups give exactly 0; a mean of 1e9 with spread 1e-3 keeps
    full precision (the exact state has no cancellation error); NaN / inf
    make the group's var NaN; integer columns run as their f64 values;
    global and multi-key forms."""
    rng = np.random.default_rng(5)
    n = 200_000
    key = rng.integers(0, 50, n).astype(np.int64)
    const = np.where(key % 2 == 0, 7.25, -3.5)
    tight = 1e9 + rng.standard_normal(n) * 1e-3
    sp = rng.standard_normal(n)
    sp[key == 3] = np.nan
    sp[(key == 4) & (rng.random(n) < 0.1)] = np.inf
    iv = rng.integers(-2**40, 2**40, n).astype(np.int64)
    df = pl.DataFrame({"k": pl.Series.from_numpy("k", key), "c": pl.Series.from_numpy("c", const),
                       "t": pl.Series.from_numpy("t", tight), "s": pl.Series.from_numpy("s", sp),
                       "i": pl.Series.from_numpy("i", iv)})
    info = {}
    out = (df.lazy().group_by("k", maintain_order=True)
           .agg(pl.col("c").var().alias("cv"), pl.col("t").var().alias("tv"), pl.col("s").std().alias("ss"),
                pl.col("i").var(0).alias("iv")).collect(info=info))
    assert info["var_path"] == "fused"
    assert out["cv"].to_list() == [0.0] * out.height
    ones = np.ones(n, bool)
    # the two-pass checker's rounded mean (error ~ulp(1e9) / 2) shifts every
    # deviation and costs it ~1e-9 here: check against the exact variance
    tv_got = out["tv"].to_numpy()
    for j, kk_ in enumerate(out["k"].to_numpy()[:10]):
        exact = _exact_var(tight[key == kk_], 1)
        assert math.isclose(tv_got[j], exact, rel_tol=4e-16), (tv_got[j], exact)
    _, ss, sstd, sok = _oracle(key, sp, ones, 1, ones)
    got = out["ss"].to_numpy()
    kk = out["k"].to_numpy()
    assert np.isnan(got[kk == 3]).all() and np.isnan(got[kk == 4]).all()
    fin = (kk != 3) & (kk != 4)
    _close(got[fin], sstd[fin], sok[fin])
    _, ivar, _, iok = _oracle(key, iv.astype(np.float64), ones, 0, ones)
    _close(out["iv"].to_numpy(), ivar, iok)
    # global var / std and two keys
    g = df.lazy().select(pl.col("t").var().alias("v"), pl.col("t").std(0).alias("s")).collect(info=(gi := {}))
    assert gi["var_path"] == "fused"
    assert math.isclose(g["v"].to_list()[0], _exact_var(tight, 1), rel_tol=4e-16)
    assert math.isclose(g["s"].to_list()[0], math.sqrt(_exact_var(tight, 0)), rel_tol=4e-16)
    k2 = (key % 3).astype(np.int64)
    df2 = pl.DataFrame({"a": pl.Series.from_numpy("a", key), "b": pl.Series.from_numpy("b", k2),
                        "t": pl.Series.from_numpy("t", tight)})
    o2 = df2.lazy().group_by("a", "b", maintain_order=True).agg(pl.col("t").var().alias("v")).collect(info=(i2 := {}))
    assert i2["var_path"] == "fused"
    for a_, b_, v_ in list(zip(o2["a"].to_list(), o2["b"].to_list(), o2["v"].to_list()))[:12]:
        assert math.isclose(v_, _exact_var(tight[(key == a_) & (k2 == b_)], 1), rel_tol=4e-16)


def test_var_fused_batches_count_len(gpu, monkeypatch):
    """len() rides on the first var column's accumulator: two var columns
    (six accumulators) next to len() run as one fused pass, not
    as batches nor the two-pass path, and stay within 1e-12 of
    the checker."""
    from polaroid_amd import frame as F

    calls = []
    inner = F._group_by_plain
    monkeypatch.setattr(F, "_group_by_plain", lambda *a, **k: calls.append(1) or inner(*a, **k))
    rng = np.random.default_rng(5)
    n = 100_003
    key, x, y, xv = _var_frame(rng, n, 50)
    df = pl.DataFrame({"k": pl.Series.from_numpy("k", key), "x": pl.Series.from_numpy("x", x, xv),
                       "y": pl.Series.from_numpy("y", y)})
    info = {}
    out = (df.lazy().group_by("k", maintain_order=True)
           .agg(pl.col("x").var().alias("xv"), pl.col("y").var().alias("yv"), pl.len())
           .collect(info=info))
    assert info["var_path"] == "fused", info
    assert len(calls) == 1, calls
    ones = np.ones(n, bool)
    keys, var, _, ok = _oracle(key, x, xv, 1, ones)
    assert np.array_equal(out["k"].to_numpy(), keys)
    _close(out["xv"].to_numpy(), var, ok)
    _, yvar, _, yok = _oracle(key, y, ones, 1, ones)
    _close(out["yv"].to_numpy(), yvar, yok)
    assert out["len"].to_list() == [int((key == k).sum()) for k in keys]


@pytest.mark.parametrize("case", ["tiny", "huge", "wide"])
def test_var_fused_out_of_range_falls_back(gpu, case):
    """Inputs whose exact fused state would leave its range take the two
    passes (info["var_path"] == "two_pass") and are still right: |x| below
    2^-484 (x * x's error would be subnormal), x * x overflowing, and values
    spanning more binades than one sum window."""
    rng = np.random.default_rng(len(case))
    n = 30_000
    key = rng.integers(0, 20, n).astype(np.int64)
    x = rng.standard_normal(n)
    if case == "tiny":
        x *= 1e-150
    elif case == "huge":
        x *= 1e160
    else:
        x[rng.random(n) < 0.3] *= 1e250
        x[rng.random(n) < 0.3] *= 1e-250
    df = pl.DataFrame({"k": pl.Series.from_numpy("k", key), "x": pl.Series.from_numpy("x", x)})
    info = {}
    out = df.lazy().group_by("k", maintain_order=True).agg(pl.col("x").var().alias("v")).collect(info=info)
    assert info["var_path"] == "two_pass", info
    keys, var, _, ok = _oracle(key, x, np.ones(n, bool), 1, np.ones(n, bool))
    assert np.array_equal(out["k"].to_numpy(), keys)
    got = out["v"].to_numpy()
    assert np.allclose(got[ok], var[ok], rtol=1e-12, atol=0) or case == "huge" and np.isinf(var[ok]).any()


@pytest.mark.parametrize("n", [1, 1023, 1024, 1025, 100_003, 1_000_003])
@pytest.mark.parametrize("pred", ["none", "on_x", "other"])
@pytest.mark.parametrize("kind", ["var0", "std1"])
def test_var_single_column_triple_kernel(gpu, n, pred, kind):
    """One var / std column as the only aggregation (no maintain_order): the
    fused kernel's variance-triple variant (info["path"] == 4: x loaded once,
    x * x and its exact error computed in registers), on the 2-limb window
    here, across the masked tail tile, with no predicate, a predicate on x
    itself (the predicate reuses x's registers) and on another column;
    within 1e-12 of the two-pass checker, validity exact."""
    rng = np.random.default_rng(n + len(pred) + len(kind))
    key = rng.integers(0, 100, n).astype(np.int64)
    x = 250 + rng.random(n) * 250
    y = rng.uniform(-5, 5, n)
    df = pl.DataFrame({"k": pl.Series.from_numpy("k", key), "x": pl.Series.from_numpy("x", x),
                       "y": pl.Series.from_numpy("y", y)})
    lf, sel = df.lazy(), np.ones(n, dtype=bool)
    if pred == "on_x":
        lf, sel = lf.filter(pl.col("x") > 300.0), x > 300.0
    elif pred == "other":
        lf, sel = lf.filter(pl.col("y") > -1.0), y > -1.0
    ddof = int(kind[-1])
    e = pl.col("x").var(ddof) if kind.startswith("var") else pl.col("x").std(ddof)
    info = {}
    out = lf.group_by("k").agg(e.alias("v")).collect(info=info)
    assert info["var_path"] == "fused"
    if n >= 1024:
        assert info["path"] == 4, info
    keys, var, std, ok = _oracle(key, x, np.ones(n, bool), ddof, sel)
    order = np.argsort(keys)
    got_k = out["k"].to_numpy()
    go = np.argsort(got_k)
    assert np.array_equal(got_k[go], keys[order])
    want = (var if kind.startswith("var") else std)[order]
    okk = ok[order]
    assert np.array_equal(out["v"].validity_numpy()[go], okk)
    _close(out["v"].to_numpy()[go], want, okk)


@pytest.mark.parametrize("n", [1025, 100_003, 1_000_003])
@pytest.mark.parametrize("pred", [False, True])
def test_var_triple_kernel_maintain_order(gpu, n, pred):
    """maintain_order=True (the first-row field: not the sum-only layout):
    one std column still runs the variance-triple variant (path 4), groups in
    first-occurrence order, within 1e-12 of the two-pass checker."""
    rng = np.random.default_rng(n + pred)
    key = rng.integers(0, 100, n).astype(np.int64)
    x = 250 + rng.random(n) * 250
    df = pl.DataFrame({"k": pl.Series.from_numpy("k", key), "x": pl.Series.from_numpy("x", x)})
    lf, sel = df.lazy(), np.ones(n, dtype=bool)
    if pred:
        lf, sel = lf.filter(pl.col("x") < 450.0), x < 450.0
    info = {}
    out = lf.group_by("k", maintain_order=True).agg(pl.col("x").std().alias("s")).collect(info=info)
    assert info["var_path"] == "fused" and info["path"] == 4, info
    keys, _, std, ok = _oracle(key, x, np.ones(n, bool), 1, sel)
    assert np.array_equal(out["k"].to_numpy(), keys)
    assert np.array_equal(out["s"].validity_numpy(), ok)
    _close(out["s"].to_numpy(), std, ok)


@pytest.mark.parametrize("spread", ["narrow", "wide"])
def test_var_triple_kernel_windows(gpu, spread):
    """The variance-triple kernel on both windows: values spanning few
    binades run on 2 limbs; values from 1e-3 to 1e3 (x * x over ~40 binades)
    on 3 limbs; both exact within 1e-12, the same kernel variant."""
    rng = np.random.default_rng(11 if spread == "narrow" else 12)
    n = 300_001
    key = rng.integers(0, 37, n).astype(np.int64)
    if spread == "narrow":
        x = 1e6 + rng.standard_normal(n) * 3.0
    else:
        x = np.exp(rng.uniform(np.log(1e-3), np.log(1e3), n)) * np.where(rng.random(n) < 0.5, -1, 1)
    df = pl.DataFrame({"k": pl.Series.from_numpy("k", key), "x": pl.Series.from_numpy("x", x)})
    info = {}
    out = df.lazy().group_by("k").agg(pl.col("x").var().alias("v")).collect(info=info)
    assert info["var_path"] == "fused" and info["path"] == 4, info
    assert info["sum_limbs"] == (2 if spread == "narrow" else 3), info
    got = dict(zip(out["k"].to_list(), out["v"].to_list()))
    for k in range(37):
        assert math.isclose(got[k], _exact_var(x[key == k], 1), rel_tol=1e-12), k


def test_var_triple_sorted_keys_take_the_register_run_path(gpu):
    """Symbol-sorted rows: the plan picks the register-run kernel (the
    variance triple is not used there) and the result is the same."""
    rng = np.random.default_rng(3)
    n = 200_000
    key = np.sort(rng.integers(0, 50, n)).astype(np.int64)
    x = 100 + rng.random(n)
    df = pl.DataFrame({"k": pl.Series.from_numpy("k", key), "x": pl.Series.from_numpy("x", x)})
    info = {}
    out = df.lazy().group_by("k").agg(pl.col("x").std().alias("s")).collect(info=info)
    assert info["var_path"] == "fused" and info["path"] != 4
    got = dict(zip(out["k"].to_list(), out["s"].to_list()))
    for k in np.unique(key)[:20]:
        assert math.isclose(got[int(k)], math.sqrt(_exact_var(x[key == k], 1)), rel_tol=1e-12)


@pytest.mark.parametrize("pname", ["gt0", "ge0", "gt250", "eq"])
def test_var_triple_nonneg_predicate(gpu, plgpu_option, pname):
    """A predicate on x that keeps no value below a non-negative literal
    (x > c, x >= c, x == c, c >= 0) runs the triple variant whose x limbs
    carry no sign (gb_fast_kernel VAR 4, option var_pos): bit-identical to
    the signed variant on data with negatives, zeros, -0.0, NaN and +inf
    (the predicate drops the negatives; NaN compares greatest and is kept),
    and against the exact variance per group."""
    rng = np.random.default_rng(len(pname))
    n = 300_003
    key = rng.integers(0, 100, n).astype(np.int64)
    x = rng.uniform(-500, 500, n)
    x[rng.random(n) < 0.05] = 0.0
    x[rng.random(n) < 0.05] = -0.0
    x[rng.random(n) < 0.05] = 3.5
    x[rng.integers(0, n, 3)] = np.nan
    x[rng.integers(0, n, 2)] = np.inf
    df = pl.DataFrame({"k": pl.Series.from_numpy("k", key), "x": pl.Series.from_numpy("x", x)})
    p = {"gt0": pl.col("x") > 0.0, "ge0": pl.col("x") >= 0.0, "gt250": pl.col("x") > 250.0,
         "eq": pl.col("x") == 3.5}[pname]
    res = []
    for on in (1, 0):
        plgpu_option("var_pos", on)
        info = {}
        out = (df.lazy().filter(p).group_by("k").agg(pl.col("x").std(1).alias("s"), )
               .collect(info=info))
        assert info["path"] == 4, info
        o = np.argsort(out["k"].to_numpy())
        res.append((out["k"].to_numpy()[o], out["s"].to_numpy()[o].view(np.int64), out["s"].validity_numpy()[o]))
    for a, b in zip(res[0], res[1]):
        assert np.array_equal(a, b), pname
    # and against the exact value (rational arithmetic, rounded once; the
    # fused triple's std is sqrt of the correctly rounded variance): groups
    # with a kept NaN / inf are NaN, a single kept row is null
    sel = {"gt0": x > 0.0, "ge0": x >= 0.0, "gt250": x > 250.0, "eq": x == 3.5}[pname] | (np.isnan(x) & (pname != "eq"))
    ks, sbits, sok = res[0]
    sv = sbits.view(np.float64)
    assert np.array_equal(ks, np.unique(key[sel]))
    for i, k in enumerate(ks.tolist()):
        vals = x[sel & (key == k)]
        if vals.size <= 1:
            assert not sok[i], k
        elif not np.all(np.isfinite(vals)):
            assert sok[i] and math.isnan(sv[i]), k
        else:
            assert sok[i] and math.isclose(sv[i], math.sqrt(_exact_var(vals, 1)), rel_tol=4e-16, abs_tol=0.0), k
