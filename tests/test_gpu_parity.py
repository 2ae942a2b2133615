"""GPU parity: the HIP path (through the C-ABI) against the oracle.

Bar: bit-exact for filter / comparison / integer
aggregation / min / max / count / len; f64 sum is the correctly rounded
exact sum (== the oracle's exact leg bit for bit; within 1 ULP of the
reference's Kahan fold); f64 mean == exact_sum / count, IEEE-divided.
"""

import math
import os

import numpy as np
import pytest

import polaroid_amd as pl
from conftest import load_golden, unhex
from oracle import oracle as O

pytestmark = pytest.mark.gpu

OPNAMES = ["eq", "ne", "lt", "le", "gt", "ge", "eq_missing", "ne_missing"]


def _apply(e, op, rhs):
    return {
        "eq": lambda: e == rhs, "ne": lambda: e != rhs, "lt": lambda: e < rhs, "le": lambda: e <= rhs,
        "gt": lambda: e > rhs, "ge": lambda: e >= rhs, "eq_missing": lambda: e.eq_missing(rhs),
        "ne_missing": lambda: e.ne_missing(rhs),
    }[op]()


def _bits(a):
    return np.asarray(a, dtype=np.float64).view(np.uint64)


def test_native_library_is_loaded(gpu):
    df = pl.DataFrame({"a": [1.0, 2.0]})
    out = df.select(pl.col("a") > 1.0)
    assert out["a"].to_list() == [False, True]
    maps = open("/proc/self/maps").read()
    assert os.path.basename(pl.native_library_path()) in maps


# ----------------------------------------------------------- comparisons
def test_compare_truth_table(gpu):
    """operations/test_comparison.py total-order table, column-vs-column and
    column-vs-scalar, evaluated by the GPU kernels."""
    cases = load_golden("compare_total_order.json")["cases"]
    lhs = [unhex(c["lhs"]) for c in cases]
    rhs = [unhex(c["rhs"]) for c in cases]
    df = pl.DataFrame({"l": pl.Series("l", lhs, pl.Float64), "r": pl.Series("r", rhs, pl.Float64)})
    for op in OPNAMES:
        got = df.select(_apply(pl.col("l"), op, pl.col("r")).alias("x"))["x"].to_list()
        exp = [c["expected"][op] for c in cases]
        assert got == exp, op
    # scalar right-hand side, `pl.col("l") <op> rhs` with a dummy second row
    for c in cases:
        lv, rv = unhex(c["lhs"]), unhex(c["rhs"])
        one = pl.DataFrame({"l": pl.Series("l", [lv, 0.0], pl.Float64)})
        got = one.select(*[_apply(pl.col("l"), op, rv).alias(op) for op in OPNAMES])
        for op in OPNAMES:
            assert got[op].to_list()[0] == c["expected"][op], (lv, rv, op)


def _same(a, b):
    if a is None or b is None:
        return a is None and b is None
    if math.isnan(a) or math.isnan(b):
        return math.isnan(a) and math.isnan(b) and math.copysign(1, a) == math.copysign(1, b)
    return a == b and math.copysign(1, a) == math.copysign(1, b)


# ----------------------------------------------------------------- filter
SIZES = list(range(64)) + [100, 1000, 10000]
SELECTIVITIES = [0.0, 0.01, 0.1, 0.5, 0.9, 0.99, 1.0 + 1e-6]


@pytest.mark.parametrize("dtype", ["Boolean", "Int32", "Int64", "Float64"])
def test_filter_parametric(gpu, dtype):
    """Mirror of operations/test_filter.py:270-285 (same PCG64 seeds): the
    reference there is numpy masking of the same payload."""
    npd = {"Boolean": np.bool_, "Int32": np.int32, "Int64": np.int64, "Float64": np.float64}[dtype]
    pdt = getattr(pl, dtype)
    for size in SIZES:
        for sel in SELECTIVITIES:
            rng = np.random.Generator(np.random.PCG64(size * 100 + int(100 * sel)))
            payload = rng.uniform(size=size) * 100.0
            mask = rng.uniform(size=size) < sel
            typed = payload.astype(npd)
            s = pl.Series.from_numpy("p", typed, dtype=pdt)
            m = pl.Series.from_numpy("m", mask, dtype=pl.Boolean)
            got = s.filter(m).to_numpy()
            assert got.dtype == typed.dtype
            assert np.array_equal(got, typed[mask]), (dtype, size, sel)


def _rand_frame(rng, n, null_frac=0.1):
    a = rng.standard_normal(n) * 100
    a[rng.random(n) < 0.02] = np.nan
    a[rng.random(n) < 0.01] = np.inf
    a[rng.random(n) < 0.01] = -0.0
    b = rng.integers(-1000, 1000, n).astype(np.int64)
    c = rng.integers(-50, 50, n).astype(np.int32)
    d = rng.uniform(-5, 5, n)
    va = rng.random(n) >= null_frac
    vb = rng.random(n) >= null_frac
    vd = rng.random(n) >= null_frac
    cols = {"a": (a, va), "b": (b, vb), "c": (c, None), "d": (d, vd)}
    return cols


def _gpu_df(cols):
    return pl.DataFrame({k: pl.Series.from_numpy(k, v, m) for k, (v, m) in cols.items()})


def _host_cols(cols, names):
    return [O.HostCol(cols[k][0], cols[k][1]) for k in names]


PREDICATES = {
    "simple_f64": (lambda: pl.col("a") > 1.5, ["a"], [(1, 0, 0), (2, 0, 1.5), (24, 0, 0)]),
    "simple_i64": (lambda: pl.col("b") <= 10, ["b"], [(1, 0, 0), (3, 0, 10), (23, 0, 0)]),
    "i32_ne": (lambda: pl.col("c") != 3, ["c"], [(1, 0, 0), (3, 0, 3), (21, 0, 0)]),
    "nan_eq": (lambda: pl.col("a") == float("nan"), ["a"], [(1, 0, 0), (2, 0, float("nan")), (20, 0, 0)]),
    "program": (lambda: ((pl.col("a") * 2 + pl.col("b")) > pl.col("d")) & ~pl.col("d").is_null(),
                ["a", "b", "d"],
                [(1, 0, 0), (3, 0, 2), (12, 0, 0), (1, 1, 0), (10, 0, 0), (1, 2, 0), (24, 0, 0),
                 (1, 2, 0), (33, 0, 0), (32, 0, 0), (30, 0, 0)]),
    "kleene_or": (lambda: (pl.col("a") < 0.0) | (pl.col("b") >= 0), ["a", "b"],
                  [(1, 0, 0), (2, 0, 0.0), (22, 0, 0), (1, 1, 0), (3, 0, 0), (25, 0, 0), (31, 0, 0)]),
    "div_isfinite": (lambda: (pl.col("d") / pl.col("b")).is_finite(), ["d", "b"],
                     [(1, 0, 0), (1, 1, 0), (13, 0, 0), (36, 0, 0)]),
}


@pytest.mark.parametrize("n", [0, 1, 63, 64, 65, 4095, 4096, 4097, 100003])
@pytest.mark.parametrize("pname", list(PREDICATES))
def test_filter_expr_vs_oracle(gpu, n, pname):
    rng = np.random.default_rng(n * 7 + len(pname))
    cols = _rand_frame(rng, n)
    mk, names, prog = PREDICATES[pname]
    df = _gpu_df(cols)
    out = df.filter(mk())
    allnames = names + [k for k in cols if k not in names]
    hc = _host_cols(cols, allnames)
    for i, k in enumerate(allnames):
        ev, evalid = O.filter_column(hc, prog, n, i)
        s = out[k]
        assert s.len() == ev.shape[0], (pname, k)
        gv, gvalid = s.to_numpy(), s.validity_numpy()
        assert np.array_equal(gvalid, evalid), (pname, k)
        if ev.dtype == np.float64:
            assert np.array_equal(_bits(gv)[evalid], _bits(ev)[evalid]), (pname, k)
        else:
            assert np.array_equal(gv[evalid], ev[evalid]), (pname, k)


@pytest.mark.parametrize("n", [1, 64, 1000, 65537])
def test_eval_arith_vs_oracle(gpu, n):
    rng = np.random.default_rng(n)
    cols = _rand_frame(rng, n)
    df = _gpu_df(cols)
    names = ["a", "b", "c", "d"]
    hc = _host_cols(cols, names)
    exprs = [
        (pl.col("a") * pl.col("d") - pl.col("b"), [(1, 0, 0), (1, 3, 0), (12, 0, 0), (1, 1, 0), (11, 0, 0)]),
        (pl.col("b") * 3037000499 + pl.col("c"), [(1, 1, 0), (3, 0, 3037000499), (12, 0, 0), (1, 2, 0), (10, 0, 0)]),
        (pl.col("b") / pl.col("c"), [(1, 1, 0), (1, 2, 0), (13, 0, 0)]),
        (-pl.col("a").abs(), [(1, 0, 0), (15, 0, 0), (14, 0, 0)]),
        (pl.col("d").is_nan() | pl.col("a").is_null(), [(1, 3, 0), (35, 0, 0), (1, 0, 0), (33, 0, 0), (31, 0, 0)]),
    ]
    for e, prog in exprs:
        s = df.select(e.alias("x"))["x"]
        dt, ev, evalid = O.eval_program(hc, prog, n)
        gvalid = s.validity_numpy()
        assert np.array_equal(gvalid, evalid), repr(e)
        gv = s.to_numpy()
        if dt == O.F64:
            assert np.array_equal(_bits(gv)[evalid], _bits(ev)[evalid]), repr(e)
        else:
            assert np.array_equal(gv[evalid].astype(ev.dtype), ev[evalid]), repr(e)


@pytest.mark.parametrize("n", [1, 4095, 4096, 4097, 64 * 4096 + 5, 3_000_001])
@pytest.mark.parametrize("fused", [1, 0])
def test_filter_one_pass_lookback(gpu, plgpu_option, n, fused):
    """The one-pass filter (filter_fused8_kernel: tiles by ticket, output
    offsets by decoupled look-back over up to ~730 predecessors) on null-free
    8-byte columns, against numpy and against the three-pass path (option
    filt_fused off): half / all / none selected, NaN in the predicate column
    (NaN > k holds: NaN sorts above every number), an Int64 predicate and
    sliced inputs."""
    plgpu_option("filt_fused", fused)
    rng = np.random.default_rng(n + fused)
    x = rng.uniform(0, 500, n + 3)
    x[rng.random(n + 3) < 0.01] = np.nan
    b = rng.integers(-1000, 1000, n + 3).astype(np.int64)
    c = rng.standard_normal(n + 3)
    for off in (0, 3):
        xs, bs, cs = x[off:off + n], b[off:off + n], c[off:off + n]
        full = [pl.Series.from_numpy("x", x), pl.Series.from_numpy("b", b), pl.Series.from_numpy("c", c)]
        df = pl.DataFrame([f.slice(off, n) for f in full])
        cases = [(pl.col("x") > 250.0, (xs > 250.0) | np.isnan(xs)),
                 (pl.col("x") > -1.0, np.ones(n, bool)),
                 (pl.col("x") < -1.0, np.zeros(n, bool)),
                 (pl.col("b") >= 10, bs >= 10)]
        for e, m in cases:
            out = df.filter(e)
            assert out.height == int(m.sum())
            assert np.array_equal(_bits(out["x"].to_numpy()), _bits(xs[m]))
            assert np.array_equal(out["b"].to_numpy(), bs[m])
            assert np.array_equal(_bits(out["c"].to_numpy()), _bits(cs[m]))
            assert out["x"].validity_numpy().all()


def test_filter_on_sliced_columns(gpu):
    rng = np.random.default_rng(3)
    n = 5000
    x = rng.standard_normal(n)
    vx = rng.random(n) > 0.2
    full = pl.Series.from_numpy("x", x, vx)
    for off in (1, 7, 63, 64, 65, 1000):
        s = full.slice(off, 3000)
        df = pl.DataFrame([s])
        out = df.filter(pl.col("x") > 0.1)["x"]
        xs, vs = x[off: off + 3000], vx[off: off + 3000]
        m = vs & (xs > 0.1)
        assert np.array_equal(out.to_numpy(), xs[m])
        assert out.validity_numpy().all()


# --------------------------------------------------------------- group_by
def _ulp(a, b):
    return abs(int(np.array(a).view(np.int64)) - int(np.array(b).view(np.int64)))


def _check_group_by(cols, key, kvalid, aggs, pred_expr, pred_prog, pred_names, maintain_order, info=None,
                    kahan_cols=()):
    """Run on GPU and compare against the oracle (exact mode)."""
    n = key.shape[0]
    names = list(dict.fromkeys(pred_names + [c for _, c in aggs]))
    data = {"k": (key, kvalid)}
    data.update({k: cols[k] for k in names})
    df = _gpu_df(data)
    lf = df.lazy()
    if pred_expr is not None:
        lf = lf.filter(pred_expr)
    exprs = [getattr(pl.col(c), kind)().alias(f"{kind}_{c}") for kind, c in aggs]
    res = {}
    out = lf.group_by("k", maintain_order=maintain_order).agg(*exprs).collect(info=res)
    if info is not None:
        info.update(res)
    hc = _host_cols(cols, names)
    okeys, okvalid, oouts = O.group_by_agg(O.HostCol(key, kvalid), hc, pred_prog,
                                           [(kind, names.index(c)) for kind, c in aggs], n, O.SUM_EXACT)
    _, _, kahan = O.group_by_agg(O.HostCol(key, kvalid), hc, pred_prog,
                                 [(kind, names.index(c)) for kind, c in aggs], n, O.SUM_KAHAN)
    gk = out["k"].to_numpy().astype(np.int64)
    gkv = out["k"].validity_numpy()
    assert gk.shape[0] == okeys.shape[0]
    # canonical order: null group last, then by key
    def order(keys, valid):
        return np.lexsort((keys, ~valid))
    if maintain_order:
        go = np.arange(gk.shape[0])
        oo = np.arange(okeys.shape[0])
    else:
        go, oo = order(gk, gkv), order(okeys, okvalid)
    assert np.array_equal(gkv[go], okvalid[oo])
    assert np.array_equal(gk[go][gkv[go]], okeys[oo][okvalid[oo]])
    for (kind, c), (ov, ovalid), (kv, _) in zip(aggs, oouts, kahan):
        s = out[f"{kind}_{c}"]
        gv, gvalid = s.to_numpy(), s.validity_numpy()
        gv, gvalid, ov, ovalid, kv = gv[go], gvalid[go], ov[oo], ovalid[oo], kv[oo]
        assert np.array_equal(gvalid, ovalid), (kind, c)
        if ov.dtype == np.float64:
            gb, ob = _bits(gv)[ovalid], _bits(ov)[ovalid]
            nan_g, nan_o = np.isnan(gv[ovalid]), np.isnan(ov[ovalid])
            assert np.array_equal(nan_g, nan_o), (kind, c)
            assert np.array_equal(gb[~nan_g], ob[~nan_o]), (kind, c, gv[ovalid][~nan_g][:5], ov[ovalid][~nan_o][:5])
            if kind == "sum" and c in kahan_cols:   # same-sign data: Kahan is within 1 ULP
                fin = np.isfinite(ov[ovalid])
                for x, y in zip(gv[ovalid][fin], kv[ovalid][fin]):
                    assert _ulp(x, y) <= 1, (x, y)   # vs the reference's Kahan fold
        else:
            assert np.array_equal(gv[ovalid].astype(np.int64), ov[ovalid].astype(np.int64)), (kind, c)
    return out


ALL_AGGS = [("sum", "a"), ("mean", "a"), ("min", "a"), ("max", "a"), ("count", "a"), ("len", "a"),
            ("sum", "b"), ("mean", "b"), ("min", "b"), ("max", "b"), ("sum", "c"), ("min", "c"),
            ("max", "d"), ("sum", "d")]


@pytest.mark.parametrize("card", [1, 7, 100, 3000, 50000])
@pytest.mark.parametrize("maintain_order", [False, True])
def test_group_by_all_aggs_vs_oracle(gpu, card, maintain_order):
    rng = np.random.default_rng(card)
    n = 200_000
    cols = _rand_frame(rng, n)
    key = rng.integers(-card // 2, card - card // 2, n).astype(np.int64) * 1_000_003
    kvalid = rng.random(n) > 0.01
    info = {}
    for i in range(0, len(ALL_AGGS), 6):   # at most 6 distinct columns per call
        _check_group_by(cols, key, kvalid, ALL_AGGS[i:i + 6], None, None, [], maintain_order, info)


@pytest.mark.parametrize("pname", ["simple_f64", "simple_i64", "program", "nan_eq"])
def test_group_by_with_predicate_vs_oracle(gpu, pname):
    rng = np.random.default_rng(11)
    n = 300_000
    cols = _rand_frame(rng, n)
    key = rng.integers(0, 100, n).astype(np.int64)
    mk, names, prog = PREDICATES[pname]
    aggs = [("sum", "a"), ("mean", "d"), ("count", "b"), ("len", "a"), ("max", "b")]
    _check_group_by(cols, key, None, aggs, mk(), prog, names, False,
                    kahan_cols=("a",) if pname == "simple_f64" else ())


def _nonull_frame(rng, n, specials=False):
    a = rng.standard_normal(n) * 100
    if specials:
        a[rng.random(n) < 0.001] = np.nan
        a[rng.random(n) < 0.001] = np.inf
        a[rng.random(n) < 0.001] = -np.inf
        a[rng.random(n) < 0.01] = -0.0
    b = rng.integers(-10**12, 10**12, n).astype(np.int64)
    d = rng.uniform(1.0, 1000.0, n)
    return {"a": (a, None), "b": (b, None), "d": (d, None)}


FAST_AGGS = {
    "sumonly": [("sum", "a"), ("sum", "d"), ("mean", "a")],
    "mixed": [("sum", "a"), ("max", "d"), ("sum", "b"), ("count", "a"), ("len", "a"), ("min", "b")],
}


@pytest.mark.parametrize("n", [1, 1023, 1024, 1025, 4097, 300001])
@pytest.mark.parametrize("aggset", list(FAST_AGGS))
@pytest.mark.parametrize("pname", [None, "simple_f64", "simple_i64"])
def test_group_by_fast_path_vs_oracle(gpu, n, aggset, pname):
    """Null-free 8-byte columns take gb_fast_kernel (sum-only variant for
    `sumonly`); the tail rows beyond the last full tile take gb_kernel."""
    rng = np.random.default_rng(n + len(aggset))
    cols = _nonull_frame(rng, n, specials=(n % 2 == 1))
    key = rng.integers(0, 37, n).astype(np.int64) * 1_000_003 - 5
    key[rng.random(n) < 0.01] = np.iinfo(np.int64).min
    info = {}
    if pname is None:
        _check_group_by(cols, key, None, FAST_AGGS[aggset], None, None, [], False, info)
    else:
        mk, names, prog = PREDICATES[pname]
        _check_group_by(cols, key, None, FAST_AGGS[aggset], mk(), prog, names, False, info)
    if n >= 1024:
        assert info["path"] == (2 if aggset == "sumonly" else 1), info


@pytest.mark.parametrize("card", [5000, 60000, 300000])
@pytest.mark.parametrize("pname", [None, "simple_f64", "program"])
@pytest.mark.parametrize("maintain_order", [False, True])
def test_group_by_partitioned_vs_oracle(gpu, card, pname, maintain_order):
    """More groups than one LDS table: the selected rows are scattered into
    hash partitions whose groups fit LDS tables (info path 3)."""
    rng = np.random.default_rng(card + (pname is None))
    n = 1_500_001
    a = rng.standard_normal(n) * 100
    a[rng.random(n) < 0.001] = np.nan
    a[rng.random(n) < 0.001] = -0.0
    cols = {"a": (a, None), "b": (rng.integers(-10**12, 10**12, n).astype(np.int64), None),
            "c": (rng.integers(-50, 50, n).astype(np.int32), None), "d": (rng.uniform(-5, 5, n), None)}
    key = rng.integers(0, card, n).astype(np.int64) * 7919 - 3
    key[rng.random(n) < 0.001] = np.iinfo(np.int64).min
    aggs = [("sum", "a"), ("mean", "d"), ("min", "b"), ("max", "c"), ("sum", "c"), ("len", "a")]
    info = {}
    if pname is None:
        _check_group_by(cols, key, None, aggs, None, None, [], maintain_order, info)
    else:
        mk, names, prog = PREDICATES[pname]
        _check_group_by(cols, key, None, aggs, mk(), prog, names, maintain_order, info)
    assert info["path"] == 3, info


@pytest.mark.parametrize("naggcols", [1, 2, 3])
def test_group_by_partitioned_first_rows_few_columns(gpu, naggcols):
    """maintain_order on the partitioned path with fewer aggregated columns
    than the scatter keeps in registers (kPartRegAcc = 3): the row-id column
    of the partition buffers must hold row ids (it once took an unloaded
    register's value when nacc < 3, scrambling the first-occurrence order)."""
    rng = np.random.default_rng(17 + naggcols)
    n = 1_500_001
    cols = {"a": (rng.uniform(10, 500, n), None), "b": (rng.integers(-10**9, 10**9, n).astype(np.int64), None),
            "c": (rng.standard_normal(n), None)}
    key = rng.integers(0, 100_000, n).astype(np.int64) * 7919 - 3
    aggs = [("sum", "a"), ("max", "b"), ("min", "c")][:naggcols]
    info = {}
    _check_group_by(cols, key, None, aggs, None, None, [], True, info)
    assert info["path"] == 3, info


@pytest.mark.parametrize("card", [5000, 60000, 300000])
@pytest.mark.parametrize("data", ["prices", "specials", "tiny"])
def test_group_by_partitioned_sum_only(gpu, card, data):
    """Many groups with f64 sums / means only: the partition buffers are
    aggregated by the fast kernel's slim 2-limb table (gb_fast_kernel PART);
    a value below the 2-limb window ("tiny") reruns with 3 limbs."""
    rng = np.random.default_rng(card + len(data))
    n = 1_500_001
    # magnitudes within a few binades (the 2-limb window's condition)
    a = rng.uniform(10, 500, n)
    d = rng.uniform(1, 5, n) * rng.choice([-1.0, 1.0], n)
    if data == "specials":
        a[rng.random(n) < 0.001] = np.nan
        a[rng.random(n) < 0.0005] = np.inf
        d[rng.random(n) < 0.001] = -0.0
    if data == "tiny":
        # three rows the plan's 65,536-row sample almost surely misses
        d[rng.choice(n, 3, replace=False)] = 1e-30
    cols = {"a": (a, None), "d": (d, None)}
    key = rng.integers(0, card, n).astype(np.int64) * 7919 - 3
    key[rng.random(n) < 0.001] = np.iinfo(np.int64).min
    aggs = [("sum", "a"), ("sum", "d"), ("mean", "a")]
    info = {}
    mk, names, prog = PREDICATES["simple_f64"]
    _check_group_by(cols, key, None, aggs, mk(), prog, names, False, info)
    assert info["path"] == 3, info
    assert info["sum_limbs"] == (3 if data == "tiny" else 2), info


def test_group_by_special_keys_and_i32_key(gpu):
    rng = np.random.default_rng(5)
    n = 20000
    cols = _rand_frame(rng, n)
    key = rng.choice(np.array([np.iinfo(np.int64).min, -1, 0, 1, np.iinfo(np.int64).max]), n)
    kvalid = rng.random(n) > 0.3
    _check_group_by(cols, key, kvalid, [("sum", "a"), ("len", "a")], None, None, [], True)
    # Int32 key keeps its dtype
    k32 = rng.integers(-5, 5, n).astype(np.int32)
    df = pl.DataFrame({"k": pl.Series.from_numpy("k", k32), "v": pl.Series.from_numpy("v", cols["d"][0])})
    out = df.group_by("k").agg(pl.col("v").sum())
    assert out["k"].dtype == pl.Int32
    got = dict(zip(out["k"].to_list(), out["v"].to_list()))
    for kv in np.unique(k32):
        assert got[int(kv)] == math.fsum(cols["d"][0][k32 == kv])


def test_group_by_empty_and_all_filtered(gpu):
    df = pl.DataFrame({"k": pl.Series("k", [], pl.Int64), "v": pl.Series("v", [], pl.Float64)})
    out = df.group_by("k").agg(pl.col("v").sum())
    assert out.height == 0
    df = pl.DataFrame({"k": [1, 2, 3], "v": [1.0, 2.0, 3.0]})
    out = df.lazy().filter(pl.col("v") > 10.0).group_by("k").agg(pl.col("v").sum()).collect()
    assert out.height == 0


def test_group_by_golden(gpu):
    for case in load_golden("group_by_cases.json")["cases"]:
        data = {"key": pl.Series("key", case["key"], pl.Int64)}
        for name, spec in case["cols"].items():
            vals = unhex(spec["values"]) if spec["dtype"] == "f64" else spec["values"]
            data[name] = pl.Series(name, vals, pl.Float64 if spec["dtype"] == "f64" else pl.Int64)
        df = pl.DataFrame(data)
        exprs = [getattr(pl.col(a[1]), a[0])().alias(a[2] if len(a) > 2 else a[1]) for a in case["aggs"]]
        out = df.group_by("key", maintain_order=case["maintain_order"]).agg(*exprs)
        keys = out["key"].to_list()
        order = sorted(range(len(keys)), key=lambda i: keys[i]) if case.get("sort_by_key") else range(len(keys))
        assert [keys[i] for i in order] == case["expected"]["key"], case["name"]
        for a in case["aggs"]:
            nm = a[2] if len(a) > 2 else a[1]
            got = out[nm].to_list()
            got = [got[i] for i in order]
            exp = unhex(case["expected"][nm])
            for g, e in zip(got, exp):
                if e is None or g is None:
                    assert g is None and e is None, (case["name"], nm, got, exp)
                elif isinstance(e, float) and math.isnan(e):
                    assert math.isnan(g), (case["name"], nm, got, exp)
                else:
                    assert g == e, (case["name"], nm, got, exp)


def test_filter_golden(gpu):
    for case in load_golden("filter_cases.json")["cases"]:
        names = list(case["cols"])
        dt = pl.Int32 if "Int32" in case["name"] else pl.Int64
        df = pl.DataFrame({k: pl.Series(k, v, dt) for k, v in case["cols"].items()})
        pred = eval(case["predicate"], {"lit": pl.lit, "col": pl.col})
        if "expected_mask" in case:
            assert df.select(pred.alias("m"))["m"].to_list() == case["expected_mask"]
        else:
            out = df.filter(pred)
            assert [list(r) for r in out.rows()] == case["expected_rows"], case["name"]
            assert out.columns == names


# ------------------------------------------------- size-independent props
@pytest.mark.slow
def test_group_by_large_properties(gpu):
    """configs[1]-sized (1e8 rows) checks: permutation invariance (bitwise),
    exact linearity sum(2x) == 2 sum(x), and sum(len) == selected rows."""
    import torch

    n = 100_000_000
    g = torch.Generator(device="cuda").manual_seed(0)
    key = torch.randint(0, 100, (n,), device="cuda", generator=g, dtype=torch.int64)
    px = torch.rand(n, device="cuda", generator=g, dtype=torch.float64) * 1000.0
    perm = torch.randperm(n, device="cuda", generator=g)

    def run(k, x, scale=1.0):
        xs = x * scale
        df = pl.DataFrame([pl.Series.from_torch("k", k), pl.Series.from_torch("x", xs)])
        out = df.lazy().filter(pl.col("x") > 500.0 * scale).group_by("k").agg(
            pl.col("x").sum().alias("s"), pl.len()).collect()
        keys = out["k"].to_numpy()
        o = np.argsort(keys)
        return keys[o], out["s"].to_numpy()[o], out["len"].to_numpy()[o]

    k1, s1, l1 = run(key, px)
    k2, s2, l2 = run(key[perm].contiguous(), px[perm].contiguous())
    assert np.array_equal(k1, k2) and np.array_equal(_bits(s1), _bits(s2)) and np.array_equal(l1, l2)
    k3, s3, _ = run(key, px, 2.0)
    assert np.array_equal(_bits(s3), _bits(s1 * 2.0))
    assert int(l1.sum()) == int((px > 500.0).sum().item())


# ------------------------------------------------- sum window variants
def _sum_only_frame(n, seed):
    rng = np.random.default_rng(seed)
    d = rng.uniform(1.0, 1000.0, n)
    # |e| >= 0.5: the exponent span is narrow whichever rows the plan samples
    e = rng.uniform(0.5, 50.0, n) * rng.choice([-1.0, 1.0], n)
    key = rng.integers(0, 50, n).astype(np.int64) * 3 + 1
    return rng, key, d, e


@pytest.mark.parametrize("inject", [None, "tiny", "subnormal", "huge", "negzero"])
def test_sum_window_two_limbs_and_reruns(gpu, inject):
    """Narrow exponent spans take the 2-limb LDS window; values the sampled
    plan did not see (tiny / subnormal / huge, placed off the sample
    stride) force the 3-limb rerun or a window refit.  The result is the
    exact sum either way."""
    n = 300_001
    rng, key, d, e = _sum_only_frame(n, 17)
    # the plan samples 4096 clusters of 16 consecutive rows, cluster c at
    # row c * (n // 4096) (groupby.hip plan_row): inject outside them
    cstep = n // 4096
    rows = np.arange(n)
    unsampled = rows[(rows >= 4096 * cstep) | (rows % cstep >= 16)]
    pos = rng.choice(unsampled, 40, replace=False)
    if inject == "tiny":
        d[pos] = 1e-30
    elif inject == "subnormal":
        d[pos] = 5e-324
    elif inject == "huge":
        d[pos] = 1e300
    elif inject == "negzero":
        d[pos] = -0.0
    info = {}
    cols = {"d": (d, None), "e": (e, None)}
    _check_group_by(cols, key, None, [("sum", "d"), ("sum", "e"), ("mean", "d")], None, None, [], False, info)
    assert info["path"] == 2
    if inject in (None, "negzero"):
        assert info["sum_limbs"] == 2 and info["reruns"] == 0, info
    else:
        assert info["reruns"] >= 1, info


@pytest.mark.parametrize("nulls", [False, True])
def test_sum_wide_exponent_span_is_exact(gpu, nulls):
    """Values spanning far more binades than one fixed-point window (1e300,
    1, 1e-300, subnormals, cancellation) take the exact wide fallback; sums
    are still math.fsum of each group, bit for bit."""
    rng = np.random.default_rng(99)
    n = 200_000
    key = rng.integers(0, 40, n).astype(np.int64)
    d = rng.uniform(-1.0, 1.0, n)
    big = rng.random(n) < 0.01
    d[big] = rng.choice([1e300, -1e300, 3e299], big.sum())
    small = rng.random(n) < 0.01
    d[small] = rng.choice([1e-300, -2.5e-300, 5e-324, 1e-310], small.sum())
    # an exact cancellation: +1e300, -1e300 and 1.0 in group 41 only
    key[:3] = 41
    d[:3] = [1e300, 1.0, -1e300]
    valid = (rng.random(n) > 0.05) if nulls else None
    if valid is not None:
        valid[:3] = True
    info = {}
    cols = {"d": (d, valid), "e": (rng.uniform(1, 2, n), None)}
    out = _check_group_by(cols, key, None, [("sum", "d"), ("mean", "d"), ("sum", "e")], None, None, [], False, info)
    got = dict(zip(out["k"].to_list(), out["sum_d"].to_list()))
    assert got[41] == 1.0
    assert info["sum_inexact"] == 0


def test_sum_wide_with_program_predicate(gpu):
    rng = np.random.default_rng(5)
    n = 100_000
    cols = _rand_frame(rng, n)
    a = cols["a"][0].copy()
    a[rng.random(n) < 0.01] = 1e280
    a[rng.random(n) < 0.01] = 1e-280
    cols["a"] = (a, cols["a"][1])
    key = rng.integers(0, 30, n).astype(np.int64)
    mk, names, prog = PREDICATES["program"]
    _check_group_by(cols, key, None, [("sum", "a"), ("mean", "a"), ("len", "a")], mk(), prog, names, False)


@pytest.mark.parametrize("layout", ["sorted", "runs_forced_random", "sorted_specials", "sorted_part"])
def test_group_by_register_accumulators(gpu, layout, plgpu_option):
    """Sorted / clustered keys: the plan sees adjacent equal keys and the
    fused kernel's lanes sum rows of a group they already hold in a register
    accumulator (flushed into the LDS table on a group change and at the
    end); option runs=1 forces that variant on random keys, specials mix its
    rows with the per-row path, and "sorted_part" runs the partitioned
    kernel's 4-slot form on sorted many-groups keys.  Exact vs the oracle."""
    rng = np.random.default_rng(len(layout) + 77)
    n = 3_000_017
    card = 30_000 if layout == "sorted_part" else 100
    a = rng.uniform(10, 500, n)
    d = rng.uniform(1, 5, n) * rng.choice([-1.0, 1.0], n)
    if layout == "sorted_specials":
        a[rng.random(n) < 0.001] = np.nan
        a[rng.random(n) < 0.0005] = np.inf
        d[rng.random(n) < 0.001] = -0.0
    key = rng.integers(0, card, n).astype(np.int64) * 7919 - 3
    if layout == "runs_forced_random":
        plgpu_option("runs", 1)
    else:
        key = np.sort(key)
    if layout == "sorted_part":
        plgpu_option("local", 0)  # keep sorted many-groups keys on the partitioned path
    cols = {"a": (a, None), "d": (d, None)}
    aggs = [("sum", "a"), ("sum", "d"), ("mean", "a")]
    info = {}
    mk, names, prog = PREDICATES["simple_f64"]
    _check_group_by(cols, key, None, aggs, mk(), prog, names, False, info)
    assert info["sum_limbs"] == 2, info
    if layout == "sorted_part":
        assert info["path"] == 3, info


@pytest.mark.parametrize("card", [7, 3000, 200_000])
@pytest.mark.parametrize("nullable", [False, True])
def test_len_count_first_last_of_float_with_specials(gpu, card, nullable):
    """len / count / first / last of a Float64 column holding NaN / inf: such
    an acc has no flags field (no sum / min / max), and an inf / NaN row must
    not write one (round 2's out-of-table write, DESIGN.md "GPU fault
    audit"; the checked build's CK_FIELD bit guards it).  Fused (LDS), generic
    and global-table paths.  Exact vs the oracle."""
    rng = np.random.default_rng(card + nullable)
    n = 400_000
    a = rng.standard_normal(n)
    a[rng.random(n) < 0.05] = np.nan
    a[rng.random(n) < 0.05] = np.inf
    a[rng.random(n) < 0.05] = -np.inf
    d = rng.standard_normal(n)
    cols = {"a": (a, (rng.random(n) > 0.1) if nullable else None), "d": (d, None)}
    key = rng.integers(0, card, n).astype(np.int64)
    for aggs, mo in (([("len", "a"), ("sum", "d")], False), ([("count", "a"), ("len", "a")], False),
                     ([("first", "a"), ("last", "a"), ("sum", "d")], True)):
        _check_group_by(cols, key, None, aggs, None, None, [], mo)


@pytest.mark.parametrize("layout", ["sorted", "runs_forced_random", "sorted_specials", "sorted_maintain_order",
                                    "random_control"])
def test_group_by_register_runs_mixed_aggs(gpu, layout, plgpu_option):
    """Sorted keys with min / max / count / len / integer sums / first / last
    next to the f64 sums: the fused kernel's lanes keep one register run per
    group (every acc's state) and fold it into the LDS table on a group
    change; rows with inf / NaN take the per-row path.  Exact vs the oracle."""
    rng = np.random.default_rng(len(layout) + 901)
    n = 2_000_003
    a = rng.uniform(10, 500, n)
    d = rng.uniform(1, 5, n) * rng.choice([-1.0, 1.0], n)  # narrow exponent span: the 2-limb window
    b = rng.integers(-10**12, 10**12, n).astype(np.int64)
    c = rng.integers(-2**40, 2**40, n).astype(np.int64)  # the fused kernel takes 8-byte columns
    if layout == "sorted_specials":
        a[rng.random(n) < 0.001] = np.nan
        a[rng.random(n) < 0.0005] = -np.inf
        d[rng.random(n) < 0.001] = -0.0
        # a few values the plan's sample misses, below the 2-limb window:
        # straight into the LDS limb fields
        d[[17, 1_000_003, n - 5]] = [1e-310, 3e-30, -7e-20]
    key = rng.integers(0, 120, n).astype(np.int64) * 104729 - 7
    if layout == "runs_forced_random":
        plgpu_option("runs", 1)
    elif layout != "random_control":
        key = np.sort(key, kind="stable")
    cols = {"a": (a, None), "b": (b, None), "c": (c, None), "d": (d, None)}
    aggs = [("sum", "a"), ("min", "d"), ("max", "a"), ("count", "d"), ("len", "a"), ("sum", "b"),
            ("min", "c"), ("max", "b"), ("mean", "d"), ("sum", "c")]
    if layout == "sorted_maintain_order":
        aggs += [("first", "d"), ("last", "a")]
    info = {}
    mk, names, prog = PREDICATES["simple_f64"]
    _check_group_by(cols, key, None, aggs, mk(), prog, names, layout == "sorted_maintain_order", info)
    assert info["path"] == 1, info
    assert info["register_runs"] == (0 if layout == "random_control" else 1), info


@pytest.mark.parametrize("layout", ["day_ordered", "symbol_sorted", "clustered_blocks", "random_control"])
@pytest.mark.parametrize("aggs_kind", ["sums", "mixed"])
def test_group_by_range_local_kernel(gpu, layout, aggs_kind):
    """Keys clustered in row order (time-ordered (symbol, day) codes, a frame
    sorted by symbol, blocks of a few keys): the plan sees few keys per row
    range although the column holds many, and the fused kernel gives each
    workgroup one contiguous run of tiles with an LDS table sized for that
    range (keys it misses take the global table).  Random keys keep the
    partitioned path.  Exact vs the oracle."""
    rng = np.random.default_rng(len(layout) * 7 + len(aggs_kind))
    n = 4_500_001
    if layout == "day_ordered":
        day = (np.arange(n) * 200) // n
        key = (rng.integers(0, 150, n) + 1000 * day).astype(np.int64)  # 30k groups, 150 per day
    elif layout == "symbol_sorted":
        key = np.sort(rng.integers(0, 40_000, n)).astype(np.int64) * 13
    elif layout == "clustered_blocks":
        blk = np.arange(n) // 65536
        key = (rng.integers(0, 64, n) * 100_003 + blk * 7).astype(np.int64)
    else:
        key = rng.integers(0, 40_000, n).astype(np.int64)
    a = rng.uniform(10, 500, n)
    d = rng.standard_normal(n)
    cols = {"a": (a, None), "d": (d, None)}
    aggs = [("sum", "a"), ("sum", "d")] if aggs_kind == "sums" else \
        [("sum", "a"), ("min", "d"), ("max", "a"), ("count", "d"), ("len", "a")]
    info = {}
    mk, names, prog = PREDICATES["simple_f64"]
    _check_group_by(cols, key, None, aggs, mk(), prog, names, False, info)
    if layout == "random_control":
        assert info["local_range"] == 0, info
    else:
        assert info["local_range"] == 1 and info["path"] in (1, 2), info
