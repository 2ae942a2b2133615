"""GPU parity of the first() / last() group-by aggregations (polars-expr/
src/reduce/first_last.rs First / Last: the value of each group's first /
last selected row, a null value included) against the oracle's restatement
(oracle/polars_oracle.c:or_group_by_agg).  Bar: bit-exact values and
validity, on every group-by path (LDS table, global table, partitioned
many-groups path, multi-key tuples)."""

import numpy as np
import pytest

import polaroid_amd as pl
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _frame(key, cols):
    data = {"k": pl.Series.from_numpy("k", key)}
    for name, (v, m) in cols.items():
        data[name] = pl.Series.from_numpy(name, v, m)
    return pl.DataFrame(data)


def _check(out, keys, outs, names, maintain_order):
    gk = out["k"].to_numpy()
    if maintain_order:
        order = np.arange(len(keys))
        assert np.array_equal(gk, keys)
    else:
        assert sorted(gk.tolist()) == sorted(keys.tolist())
        pos = {int(k): i for i, k in enumerate(gk)}
        order = np.array([pos[int(k)] for k in keys], dtype=np.int64)
    for nm, (vals, valid) in zip(names, outs):
        s = out[nm]
        gv, gm = s.to_numpy()[order], s.validity_numpy()[order]
        assert np.array_equal(gm, valid), nm
        if vals.dtype == np.float64:
            assert np.array_equal(gv[valid].view(np.uint64), vals[valid].view(np.uint64)), nm
        else:
            assert np.array_equal(gv[valid].astype(np.int64), vals[valid].astype(np.int64)), nm


@pytest.mark.parametrize("n,card", [(1, 1), (1000, 7), (200_003, 100), (300_001, 60_000), (2_000_000, 700_000)])
@pytest.mark.parametrize("maintain_order", [False, True])
@pytest.mark.parametrize("pred", [False, True])
def test_first_last_vs_oracle(gpu, n, card, maintain_order, pred):
    rng = np.random.default_rng(n + card + 2 * maintain_order + pred)
    key = rng.integers(0, card, n).astype(np.int64)
    f = rng.standard_normal(n)
    fv = rng.random(n) > 0.1
    i = rng.integers(-2**40, 2**40, n).astype(np.int64)
    u = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    uv = rng.random(n) > 0.3
    df = _frame(key, {"f": (f, fv), "i": (i, None), "u": (u, uv)})
    aggs = [pl.col("f").first().alias("f_first"), pl.col("f").last().alias("f_last"),
            pl.col("i").first().alias("i_first"), pl.col("u").last().alias("u_last"),
            pl.col("f").sum().alias("f_sum")]
    lf = df.lazy()
    program = []
    if pred:
        lf = lf.filter(pl.col("f") > 0.25)
        program = [(1, 0, 0), (2, 0, 0.25), (24, 0, 0)]
    out = lf.group_by("k", maintain_order=maintain_order).agg(*aggs).collect()
    cols = [O.HostCol(f, fv), O.HostCol(i), O.HostCol(u, uv)]
    keys, kvalid, outs = O.group_by_agg(O.HostCol(key), cols, program,
                                        [("first", 0), ("last", 0), ("first", 1), ("last", 2), ("sum", 0)], n)
    _check(out, keys, outs, ["f_first", "f_last", "i_first", "u_last", "f_sum"], maintain_order)
    assert out["u_last"].dtype == pl.UInt32 and out["i_first"].dtype == pl.Int64


def test_ohlcv_bar(gpu):
    """The OHLCV bar of a resample: open.first, high.max, low.min,
    close.last, volume.sum per symbol."""
    rng = np.random.default_rng(1)
    n = 1_000_000
    sym = rng.integers(0, 100, n).astype(np.int64)
    o, h, lo, c = (rng.uniform(1, 500, n) for _ in range(4))
    v = rng.integers(1, 10_000, n).astype(np.int64)
    df = _frame(sym, {"open": (o, None), "high": (h, None), "low": (lo, None), "close": (c, None),
                      "volume": (v, None)})
    out = df.group_by("k", maintain_order=True).agg(
        pl.col("open").first(), pl.col("high").max(), pl.col("low").min(), pl.col("close").last(),
        pl.col("volume").sum())
    cols = [O.HostCol(x) for x in (o, h, lo, c, v)]
    keys, _, outs = O.group_by_agg(O.HostCol(sym), cols, [],
                                   [("first", 0), ("max", 1), ("min", 2), ("last", 3), ("sum", 4)], n)
    _check(out, keys, outs, ["open", "high", "low", "close", "volume"], True)


@pytest.mark.parametrize("pack", [True, False])
def test_first_last_multi_key(gpu, pack, plgpu_option):
    if not pack:
        plgpu_option("no_pack", 1)
    rng = np.random.default_rng(3)
    n = 100_000
    a = rng.integers(0, 50, n).astype(np.int64)
    b = rng.integers(0, 20, n).astype(np.int32)
    bv = rng.random(n) > 0.05
    x = rng.standard_normal(n)
    xv = rng.random(n) > 0.2
    df = pl.DataFrame({"a": pl.Series.from_numpy("a", a), "b": pl.Series.from_numpy("b", b, bv),
                       "x": pl.Series.from_numpy("x", x, xv)})
    out = df.group_by("a", "b", maintain_order=True).agg(pl.col("x").first().alias("xf"),
                                                         pl.col("x").last().alias("xl"))
    okeys, outs = O.group_by_agg_multi([(a, None), (b, bv)], [O.HostCol(x, xv)], None,
                                       [("first", 0), ("last", 0)], n)
    assert np.array_equal(out["a"].to_numpy(), okeys[0][0])
    for nm, (vals, valid) in zip(["xf", "xl"], outs):
        assert np.array_equal(out[nm].validity_numpy(), valid)
        assert np.array_equal(out[nm].to_numpy()[valid], vals[valid])


def test_first_last_refused_on_partitioned_path(gpu):
    import ctypes as C

    from polaroid_amd import _native as N

    key = pl.Series("k", [1, 2, 1], pl.Int64)
    col = pl.Series("v", [1.0, 2.0, 3.0], pl.Float64)
    aggs = (N.Agg * 1)()
    aggs[0].kind, aggs[0].col = N.AGG["first"], 0
    h = C.c_void_p()
    recs, ref = C.c_int64(), C.c_int32()
    bu, hint = (C.c_int32 * 6)(), (C.c_int32 * 6)()
    rc = N.lib().plgpu_gb_partial_begin(C.byref(key._col), C.byref(col._col), 1, None, 0, aggs, 1, None, 1,
                                        C.byref(h), C.byref(recs), bu, C.byref(ref), hint, None, None)
    assert rc == N.ERR_INVALID and b"first / last" in N.lib().plgpu_last_error()
