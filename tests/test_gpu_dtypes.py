"""GPU parity over the dtype breadth of the path (round 2): Int8 / Int16 /
UInt8 / UInt16 / UInt64 / Float32 columns and the temporal logical types
(Datetime / Date / Duration over their physical integers), through
expression evaluation, filter, group-by, sort, join, rolling and the Arrow
boundary.  The checker is the oracle's typed evaluator (pinned by
tests/test_arith_types.py against tests/golden/arith_cases.json) and, for
the reductions, the reference's per-dtype rules restated in numpy
(reduce/sum.rs:40 out_dtype, reduce/mean.rs:29, min_max.rs).  Integer /
byte / index results are bit-exact; Float32 sums are the exact sum rounded
to f64 and then to f32 (within 1 ULP of the reference's f32 pairwise sum).
"""

import datetime as dt
import math
import zlib

import numpy as np
import pyarrow as pa
import pytest

import polaroid_amd as pl
from oracle import oracle as O
from polaroid_amd import _native as N
from polaroid_amd.expr import col, lit, lower

from conftest import load_golden, unhex

pytestmark = pytest.mark.gpu

NP = {"Int8": np.int8, "Int16": np.int16, "Int32": np.int32, "Int64": np.int64, "UInt8": np.uint8,
      "UInt16": np.uint16, "UInt32": np.uint32, "UInt64": np.uint64, "Float32": np.float32, "Float64": np.float64}
PLT = {k: getattr(pl, k) for k in NP}
INTS = [k for k in NP if not k.startswith("Float")]


def rand(dt_, n, rng, small=False):
    if dt_.startswith("Float"):
        x = rng.standard_normal(n) * (10 if small else 1e3)
        x[rng.random(n) < 0.03] = np.nan
        x[rng.random(n) < 0.02] = 0.0
        x[rng.random(n) < 0.01] = -0.0
        x[rng.random(n) < 0.01] = np.inf
        return x.astype(NP[dt_])
    info = np.iinfo(NP[dt_])
    if small:
        lo, hi = max(info.min, -50), min(info.max, 50)
        return rng.integers(lo, hi, n, endpoint=True).astype(NP[dt_])
    v = rng.integers(info.min, info.max, n, dtype=NP[dt_], endpoint=True)
    v[: min(n, 8)] = np.array([info.min, info.max, 0, 1, info.max - 1, info.min + 1, 2, 3][: min(n, 8)], NP[dt_])
    return v


def frame(cols: dict):
    """{name: (np values, valid or None)} -> device DataFrame + oracle HostCols."""
    series, hosts = [], []
    for nm, (v, ok) in cols.items():
        series.append(pl.Series.from_numpy(nm, v, ok))
        hosts.append(O.HostCol(v, ok))
    return pl.DataFrame(series), hosts


def check_eval(df, hosts, names, expr, n):
    out = df.select(expr.alias("out"))["out"]
    prog = lower(expr, {nm: i for i, nm in enumerate(names)},
                 {nm: df[nm].dtype.physical().code for nm in names})
    odt, want, wvalid = O.eval_program(hosts, prog, n)
    assert out.dtype.code == odt, (expr, out.dtype, odt)
    got_valid = out.validity_numpy()
    assert np.array_equal(got_valid, wvalid), expr
    got = out.to_numpy()
    if odt == N.BOOL:
        assert np.array_equal(got[wvalid], want[wvalid]), expr
    elif odt in (N.F64, N.F32):
        # a NaN's sign and payload are the ALU's (x86 yields the negative
        # default NaN, gfx950 the positive one); polars' TotalOrd treats every
        # NaN as one value, so NaNs compare by position and the rest by bits
        g, w = got[wvalid], want[wvalid]
        assert np.array_equal(np.isnan(g), np.isnan(w)), expr
        keep = ~np.isnan(w)
        assert np.array_equal(g[keep].view(np.uint8), w[keep].view(np.uint8)), expr
    else:
        assert np.array_equal(got[wvalid].view(np.uint8), want[wvalid].view(np.uint8)), expr


# ---------------------------------------------------------------- golden
CASES = load_golden("arith_cases.json")["cases"]


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_golden_arith_on_gpu(gpu, case):
    series = []
    for nm, (d, vals) in case["cols"].items():
        vals = unhex(vals)
        valid = np.array([v is not None for v in vals], bool)
        arr = np.array([0 if v is None else v for v in vals], dtype=NP[d])
        series.append(pl.Series.from_numpy(nm, arr, None if valid.all() else valid))
    df = pl.DataFrame(series)
    expr = eval(case["expr"], {"pl": pl, "col": col, "lit": lit})
    if case.get("raises"):
        with pytest.raises(getattr(pl, case["raises"])):
            df.select(expr)
        return
    out = df.select(expr)
    s = out[out.columns[0]]
    assert out.columns[0] == case.get("expected_name", list(case["cols"])[0])
    assert repr(s.dtype) == case["expected_dtype"]
    want = unhex(case["expected"])
    got = s.to_list()
    for g, w in zip(got, want):
        if w is None or g is None:
            assert g is w
        elif isinstance(w, float) and case.get("approx"):
            assert math.isclose(g, w, rel_tol=1e-5, abs_tol=1e-8)
        else:
            assert g == w and (not isinstance(w, float) or math.copysign(1, g) == math.copysign(1, w))


# ------------------------------------------------- random ops vs oracle
PAIRS = [("Int8", "Int8"), ("Int16", "UInt8"), ("UInt8", "UInt8"), ("UInt16", "Int32"), ("Int32", "UInt32"),
         ("UInt64", "UInt64"), ("Int64", "UInt64"), ("Float32", "Float32"), ("Float32", "Int16"),
         ("Float32", "Float64"), ("Int8", "Float32"), ("UInt32", "Float32"), ("Int64", "Int8")]
OPS = ["+", "-", "*", "/", "//", "%", "<", "<=", "==", "!=", ">", ">=", "eq_missing"]


@pytest.mark.parametrize("a_dt,b_dt", PAIRS)
def test_binary_ops_vs_oracle(gpu, a_dt, b_dt):
    rng = np.random.default_rng(zlib.crc32(f"{a_dt},{b_dt}".encode()))
    n = 20_000
    a, b = rand(a_dt, n, rng), rand(b_dt, n, rng)
    if not b_dt.startswith("Float"):
        b[rng.random(n) < 0.02] = 0
    av, bv = rng.random(n) > 0.05, rng.random(n) > 0.05
    df, hosts = frame({"a": (a, av), "b": (b, bv)})
    for op in OPS:
        e = {"eq_missing": col("a").eq_missing(col("b"))}.get(op)
        if e is None:
            e = eval(f"col('a') {op} col('b')")
        check_eval(df, hosts, ["a", "b"], e, n)
    if a_dt in INTS and b_dt in INTS:
        for e in (col("a") & col("b"), col("a") | col("b"), col("a") ^ col("b")):
            if {a_dt, b_dt} == {"Int64", "UInt64"}:
                # their supertype is Float64, and polars has no bitwise ops on floats
                with pytest.raises(pl.PolaroidError):
                    df.select(e.alias("out"))
                continue
            check_eval(df, hosts, ["a", "b"], e, n)


LITS = [3, -7, 1000, 2.5, -0.75, 1e30, 0, 0.0, 7.0]


@pytest.mark.parametrize("a_dt", list(NP))
def test_scalar_literal_ops_vs_oracle(gpu, a_dt):
    """Column-with-literal forms: dynamic literals take the column's type
    (supertype.rs:463), a float divisor literal divides by reciprocal
    (float.rs:113 true_div_scalar, :78-98 floor / mod), x // 0 -> null."""
    rng = np.random.default_rng(len(a_dt))
    n = 8000
    a = rand(a_dt, n, rng)
    df, hosts = frame({"a": (a, rng.random(n) > 0.1)})
    for v in LITS:
        if a_dt.startswith("U") and isinstance(v, int) and v < 0:
            continue
        for e in (col("a") + v, col("a") - v, col("a") * v, col("a") / v, col("a") // v, col("a") % v, v / col("a"),
                  v // col("a"), col("a") > v, col("a") == v):
            check_eval(df, hosts, ["a"], e, n)


CASTS = list(NP) + ["Boolean"]


@pytest.mark.parametrize("src", list(NP))
def test_cast_matrix_vs_oracle(gpu, src):
    rng = np.random.default_rng(len(src) * 7)
    n = 6000
    a = rand(src, n, rng)
    if src.startswith("Float"):
        a[:6] = np.array([1e20, -1e20, 255.9, -128.9, 3e9, -0.5], NP[src])
    df, hosts = frame({"a": (a, rng.random(n) > 0.1)})
    for dst in CASTS:
        t = getattr(pl, dst)
        check_eval(df, hosts, ["a"], col("a").cast(t, strict=False), n)
        if src in INTS and dst in INTS:
            check_eval(df, hosts, ["a"], col("a").cast(t, wrap_numerical=True), n)


def test_strict_cast_raises_only_when_a_value_does_not_fit(gpu):
    df = pl.DataFrame([pl.Series.from_numpy("a", np.array([1, 2, 300], np.int64))])
    with pytest.raises(pl.InvalidOperationError, match="strict=False"):
        df.select(col("a").cast(pl.UInt8))
    assert df.select(col("a").cast(pl.UInt16))["a"].to_list() == [1, 2, 300]
    assert df.select(col("a").cast(pl.Float32))["a"].to_list() == [1.0, 2.0, 300.0]
    assert df.select(col("a").cast(pl.UInt8, strict=False))["a"].to_list() == [1, 2, None]


@pytest.mark.parametrize("dt_", ["Int8", "UInt16", "Float32", "Int64", "Float64"])
def test_when_fill_null_is_in_between_vs_oracle(gpu, dt_):
    rng = np.random.default_rng(5)
    n = 10_000
    a, b = rand(dt_, n, rng, small=True), rand(dt_, n, rng, small=True)
    c = rng.random(n) < 0.5
    df, hosts = frame({"a": (a, rng.random(n) > 0.1), "b": (b, rng.random(n) > 0.1), "c": (c, rng.random(n) > 0.1)})
    names = ["a", "b", "c"]
    for e in (pl.when(col("c")).then(col("a")).otherwise(col("b")),
              pl.when(col("a") > col("b")).then(col("a") - col("b")).otherwise(0),
              pl.when(col("c")).then(col("a")).when(col("a") > 3).then(lit(7)).otherwise(None),
              col("a").fill_null(col("b")), col("a").fill_null(3), col("a").fill_null(2.5),
              col("a").is_in([1, 2, 3, 40]), col("a").is_in([5, None], nulls_equal=True), col("a").is_in([]),
              col("a").is_between(-3, 10), col("a").is_between(col("b"), 20, closed="none"),
              col("c") ^ (col("a") > 0)):
        check_eval(df, hosts, names, e, n)


# ------------------------------------------------------------- filter
@pytest.mark.parametrize("dt_", list(NP))
def test_filter_typed_columns_vs_oracle(gpu, dt_):
    rng = np.random.default_rng(11)
    n = 50_003
    x = rand(dt_, n, rng)
    k = rand("Int16", n, rng, small=True)
    xv = rng.random(n) > 0.2
    df, hosts = frame({"x": (x, xv), "k": (k, None)})
    pred = (col("k") > 3) | col("x").is_null()
    out = df.filter(pred)
    prog = lower(pred, {"x": 0, "k": 1}, {"x": df["x"].dtype.code, "k": N.I16})
    for i, nm in enumerate(("x", "k")):
        vals, valid = O.filter_column(hosts, prog, n, i)
        assert out[nm].dtype is getattr(pl, dt_ if nm == "x" else "Int16")
        assert np.array_equal(out[nm].validity_numpy(), valid)
        m = out[nm].validity_numpy()
        assert np.array_equal(out[nm].to_numpy()[m].view(np.uint8), vals[m].view(np.uint8))


# ------------------------------------------------------------ group-by
def _np_groups(key, kvalid, sel):
    order, members = [], {}
    for r in np.flatnonzero(sel):
        g = ("null",) if not kvalid[r] else key[r].item()
        if g not in members:
            members[g] = []
            order.append(g)
        members[g].append(r)
    return order, members


SUM_OUT = {"Int8": np.int64, "Int16": np.int64, "UInt8": np.int64, "UInt16": np.int64, "Int32": np.int32,
           "UInt32": np.uint32, "Int64": np.int64, "UInt64": np.uint64}


@pytest.mark.parametrize("kdt", INTS)
@pytest.mark.parametrize("vdt", ["Int8", "UInt16", "Int32", "UInt64", "Float32"])
def test_group_by_typed_vs_reference_rules(gpu, kdt, vdt):
    rng = np.random.default_rng(zlib.crc32(f"{kdt},{vdt}".encode()))
    n = 30_000
    key = rand(kdt, n, rng, small=True)
    kv = rng.random(n) > 0.03
    x = rand(vdt, n, rng)
    if vdt == "Float32":
        x[np.isinf(x)] = 1.0
    xv = rng.random(n) > 0.1
    f = rng.random(n)
    df, _ = frame({"k": (key, kv), "x": (x, xv), "f": (f, None)})
    out = (df.lazy().filter(col("f") > 0.3).group_by("k", maintain_order=True)
           .agg(col("x").sum().alias("s"), col("x").mean().alias("m"), col("x").min().alias("lo"),
                col("x").max().alias("hi"), col("x").first().alias("fi"), col("x").last().alias("la"),
                col("x").count().alias("c"), pl.len()).collect())
    sel = f > 0.3
    order, members = _np_groups(key, kv, sel)
    assert out.height == len(order)
    assert repr(out["k"].dtype) == kdt
    got_keys = out["k"].to_list()
    assert got_keys == [None if g == ("null",) else g for g in order]
    isf = vdt.startswith("Float")
    assert repr(out["s"].dtype) == ("Float32" if isf else np.dtype(SUM_OUT[vdt]).name.capitalize().replace("Uint", "UInt"))
    assert repr(out["m"].dtype) == ("Float32" if isf else "Float64")
    assert repr(out["lo"].dtype) == vdt and repr(out["fi"].dtype) == vdt
    cols = {c: out[c].to_list() for c in ("s", "m", "lo", "hi", "fi", "la", "c", "len")}
    for gi, g in enumerate(order):
        rows = np.array(members[g])
        vals = x[rows][xv[rows]]
        assert cols["len"][gi] == len(rows) and cols["c"][gi] == len(vals)
        assert cols["fi"][gi] == (x[rows[0]].item() if xv[rows[0]] else None) or (
            isf and math.isnan(cols["fi"][gi]) and math.isnan(x[rows[0]]))
        if len(vals) == 0:
            assert cols["m"][gi] is None and cols["lo"][gi] is None
            continue
        if isf:
            exact = math.fsum(float(v) for v in vals)
            want = float(np.float32(exact)) if not np.isnan(vals).any() else math.nan
            got = cols["s"][gi]
            assert (math.isnan(got) and math.isnan(want)) or got == want
            nn = vals[~np.isnan(vals)]
            if len(nn):
                assert cols["lo"][gi] == float(nn.min()) and cols["hi"][gi] == float(nn.max())
        else:
            wide = sum(int(v) for v in vals)
            bits = np.dtype(SUM_OUT[vdt]).itemsize * 8
            want = wide % (1 << bits)
            if np.dtype(SUM_OUT[vdt]).kind == "i" and want >= 1 << (bits - 1):
                want -= 1 << bits
            assert cols["s"][gi] == want
            assert cols["lo"][gi] == int(vals.min()) and cols["hi"][gi] == int(vals.max())
            assert cols["m"][gi] == float(np.float64(math.fsum(float(v) for v in vals)) / len(vals)) or \
                math.isclose(cols["m"][gi], wide / len(vals), rel_tol=1e-15)


# --------------------------------------------------------- sort / join
@pytest.mark.parametrize("dt_", list(NP))
@pytest.mark.parametrize("desc,nl", [(False, False), (True, True)])
def test_sort_typed_vs_oracle(gpu, dt_, desc, nl):
    rng = np.random.default_rng(17)
    n = 40_000
    x = rand(dt_, n, rng)
    xv = rng.random(n) > 0.05
    df, hosts = frame({"x": (x, xv)})
    got = df["x"].arg_sort(descending=desc, nulls_last=nl).to_numpy()
    want = O.arg_sort(hosts[0], desc, nl)
    assert np.array_equal(got.astype(np.int64), want)


@pytest.mark.parametrize("dt_", INTS)
def test_join_typed_keys_vs_oracle(gpu, dt_):
    rng = np.random.default_rng(23)
    lk, rk = rand(dt_, 20_000, rng, small=True), rand(dt_, 300, rng, small=True)
    left = pl.DataFrame([pl.Series.from_numpy("k", lk), pl.Series.from_numpy("a", np.arange(20_000))])
    right = pl.DataFrame([pl.Series.from_numpy("k", rk), pl.Series.from_numpy("b", np.arange(300))])
    out = left.join(right, on="k", maintain_order="left_right")
    li, ri = O.join_inner(O.HostCol(lk), O.HostCol(rk))
    assert out["a"].to_list() == li.tolist() and out["b"].to_list() == ri.tolist()
    assert repr(out["k"].dtype) == dt_


# ------------------------------------------------------------- temporal
def test_temporal_columns_through_the_path(gpu):
    base = dt.datetime(2024, 1, 1)
    n = 5000
    rng = np.random.default_rng(3)
    secs = rng.integers(0, 86400 * 30, n)
    ts = np.array([np.datetime64(base + dt.timedelta(seconds=int(s)), "ns") for s in secs])
    day0 = (base.date() - dt.date(1970, 1, 1)).days  # date32 = days since the epoch
    days = (day0 + secs // 86400).astype(np.int32)
    dur = rng.integers(-10**9, 10**9, n).astype("timedelta64[ns]")
    sym = rng.integers(0, 7, n).astype(np.int64)
    px = rng.random(n) * 100
    table = pa.table({"ts": pa.array(ts.astype("datetime64[ns]")), "day": pa.array(days, pa.date32()),
                      "dur": pa.array(dur), "sym": pa.array(sym), "px": pa.array(px)})
    df = pl.DataFrame.from_batches(table.to_batches(max_chunksize=999))
    assert repr(df["ts"].dtype) == "Datetime(time_unit='ns', time_zone=None)" and df["day"].dtype is pl.Date
    assert df.to_arrow().schema == table.schema
    cut = base + dt.timedelta(days=10)
    f = df.filter(col("ts") >= cut)
    want = ts >= np.datetime64(cut, "ns")
    assert f.height == int(want.sum())
    assert f["ts"].to_arrow().type == pa.timestamp("ns")
    f2 = df.filter(col("day") < dt.date(2024, 1, 5))
    assert f2.height == int((days < day0 + 4).sum())
    g = df.group_by("sym", maintain_order=True).agg(col("ts").min().alias("first_ts"), col("ts").max().alias("t1"),
                                                    col("dur").sum().alias("d"))
    assert repr(g["first_ts"].dtype).startswith("Datetime") and repr(g["d"].dtype).startswith("Duration")
    for i, s in enumerate(g["sym"].to_list()):
        m = sym == s
        assert g["first_ts"].to_numpy()[i] == ts[m].astype(np.int64).min()
        assert g["d"].to_numpy()[i] == dur[m].astype(np.int64).sum()
    d = df.select((col("ts") - col("ts").alias("x")).alias("zero"), (col("ts") + col("dur")).alias("shift"),
                  (col("ts") - dt.timedelta(hours=1)).alias("back"))
    assert repr(d["zero"].dtype) == "Duration(time_unit='ns')" and set(d["zero"].to_numpy().tolist()) == {0}
    assert np.array_equal(d["shift"].to_numpy(), ts.astype(np.int64) + dur.astype(np.int64))
    assert np.array_equal(d["back"].to_numpy(), ts.astype(np.int64) - 3_600_000_000_000)
    s = df.sort("ts")
    assert np.array_equal(s["ts"].to_numpy(), np.sort(ts.astype(np.int64), kind="stable"))
    with pytest.raises(pl.InvalidOperationError):
        df.select(col("ts") + col("ts"))
    with pytest.raises(pl.InvalidOperationError):
        df.group_by("sym").agg(col("ts").sum())


def _same(g, r) -> bool:
    """Equal as polars values: both null, both NaN, or equal."""
    if g is None or r is None:
        return g is None and r is None
    if isinstance(g, float) and isinstance(r, float) and math.isnan(g):
        return math.isnan(r)
    return g == r


@pytest.mark.parametrize("dt_", ["Int8", "UInt16", "Float32", "UInt32"])
def test_rolling_typed(gpu, dt_):
    rng = np.random.default_rng(9)
    n = 4000
    x = rand(dt_, n, rng, small=True)
    s = pl.Series.from_numpy("x", x)
    wide = pl.Series.from_numpy("x", x.astype(np.float64) if dt_ == "Float32" else x.astype(np.int64))
    mn = s.rolling_min(7)
    assert repr(mn.dtype) == dt_
    assert all(_same(g, r) for g, r in zip(mn.to_list(), wide.rolling_min(7).to_list()))
    mean = s.rolling_mean(5)
    assert repr(mean.dtype) == ("Float32" if dt_ == "Float32" else "Float64")
    if dt_ != "UInt32":
        sm = s.rolling_sum(5)
        assert repr(sm.dtype) == ("Float32" if dt_ == "Float32" else "Int64")
        ref = wide.rolling_sum(5).to_list()
        got = sm.to_list()
        if dt_ == "Float32":
            assert all(_same(g, None if r is None else float(np.float32(r))) for g, r in zip(got, ref))
        else:
            assert got == ref
    else:
        with pytest.raises(pl.InvalidOperationError):
            s.rolling_sum(5)
