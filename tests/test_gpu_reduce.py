"""GPU parity of aggregations over computed inputs and of global reductions
(plgpu_group_by_agg_ex), against the oracle (oracle.group_by_agg_inputs) and
the reference's own cases (tests/golden/reduce_cases.json).

  * `x op y` of Float64 columns / literals under an aggregation runs in the
    fused kernel's registers (no extra pass); the tests check the path taken
    and bit-exact results against the oracle, which evaluates the same
    expression elementwise and sums exactly;
  * any other expression (integer arithmetic, casts, when/then, String
    comparisons) is evaluated once into a column first;
  * select(aggs) is the fused kernel with one group, one output row even
    when no row is selected.
"""

import math

import numpy as np
import pytest

import polaroid_amd as pl
from oracle import oracle as O
from polaroid_amd import _native as N
from polaroid_amd.expr import col, lit, lower, when

from conftest import load_golden, unhex
from test_reduce import CASES, NP, check, oracle_case

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.asarray(a, dtype=np.float64).view(np.uint64)


def gpu_frame(case):
    data = {}
    for nm, spec in case["cols"].items():
        vals = unhex(spec["values"])
        valid = np.array([v is not None for v in vals], bool)
        arr = np.array([0 if v is None else v for v in vals], dtype=NP[spec["dtype"]])
        data[nm] = pl.Series.from_numpy(nm, arr, None if valid.all() else valid)
    if case["key"] is not None:
        data["__k"] = pl.Series.from_numpy("__k", np.array(case["key"], np.int64))
    return pl.DataFrame(data)


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_reduce_cases_on_gpu(gpu, case):
    df = gpu_frame(case)
    exprs = [eval(t, {"pl": pl, "col": col, "lit": lit, "when": when}).alias(nm) for t, nm in case["aggs"]]
    if case["key"] is None:
        out = df.lazy().select(*exprs).collect()
        res = {"key": np.zeros(out.height, np.int64)}
    else:
        out = df.lazy().group_by("__k", maintain_order=True).agg(*exprs).collect()
        res = {"key": out["__k"].to_numpy().astype(np.int64)}
    for _, nm in case["aggs"]:
        res[nm] = (out[nm].to_numpy(), out[nm].validity_numpy())
    check(case, res)
    # and equal to the oracle
    ref = oracle_case(case)
    for _, nm in case["aggs"]:
        if nm in case.get("tol", {}):
            continue
        g, gv = res[nm]
        o, ov = ref[nm]
        assert np.array_equal(gv, ov), nm
        if o.dtype == np.float64:
            assert np.array_equal(_bits(g.astype(np.float64))[gv], _bits(o)[ov]), nm
        else:
            assert np.array_equal(g[gv].astype(np.int64), o[ov].astype(np.int64)), nm


def _frame(rng, n, nulls=False, nkeys=100):
    a = rng.standard_normal(n) * 100
    b = rng.uniform(0.5, 2.0, n)
    c = rng.uniform(10, 500, n)
    k = (rng.integers(0, nkeys, n) * 7919 + 11).astype(np.int64)
    q = rng.integers(-50, 50, n).astype(np.int64)
    va = (rng.random(n) > 0.05) if nulls else None
    df = pl.DataFrame({"k": pl.Series.from_numpy("k", k), "a": pl.Series.from_numpy("a", a, va),
                       "b": pl.Series.from_numpy("b", b), "c": pl.Series.from_numpy("c", c),
                       "q": pl.Series.from_numpy("q", q)})
    cols = {"k": (k, None), "a": (a, va), "b": (b, None), "c": (c, None), "q": (q, None)}
    return df, cols


# (name, expression, aggregation)
DERIVED = [
    ("ab_sum", lambda: (col("a") * col("b")).sum()),
    ("bc_sum", lambda: (col("b") + col("c")).sum()),
    ("c_minus_lit", lambda: (col("c") - 250.0).sum()),
    ("lit_div_b", lambda: (2.0 / col("b")).mean()),
    ("a_div_b", lambda: (col("a") / col("b")).sum()),
    ("a_scalar_div", lambda: (col("a") / 3.0).sum()),
    ("c_times_lit_max", lambda: (col("c") * 1.5).max()),
    ("ab_min", lambda: (col("a") * col("b")).min()),
]


def _oracle(cols, names, key, exprs_aggs, pred_expr, n):
    """Oracle result {out name: (values, valid)} (+ key) for aggregations
    over expressions, with the same lowering the executor uses."""
    hc = [O.HostCol(cols[nm][0], cols[nm][1]) for nm in names]
    idx = {nm: i for i, nm in enumerate(names)}
    schema = {nm: c.code for nm, c in zip(names, hc)}
    inputs, specs = [], []
    for kind, x in exprs_aggs:
        if x is None:
            specs.append(("len", 0))
        elif x.kind == "col":
            specs.append((kind, idx[x.value]))
        else:
            inputs.append(lower(x, idx, schema))
            specs.append((kind, len(hc) + len(inputs) - 1))
    prog = lower(pred_expr, idx, schema) if pred_expr is not None else None
    kc = None if key is None else O.HostCol(cols[key][0], cols[key][1])
    return O.group_by_agg_inputs(kc, hc, prog, inputs, specs, n)


def _compare(out, keyname, okeys, oouts, names):
    if keyname is None:
        order_g = np.arange(out.height)
        order_o = np.arange(okeys.shape[0])
    else:
        order_g = np.argsort(out[keyname].to_numpy(), kind="stable")
        order_o = np.argsort(okeys, kind="stable")
        assert np.array_equal(out[keyname].to_numpy()[order_g], okeys[order_o])
    assert out.height == okeys.shape[0]
    for nm, (ov, ovalid) in zip(names, oouts):
        gv, gvalid = out[nm].to_numpy()[order_g], out[nm].validity_numpy()[order_g]
        ov, ovalid = ov[order_o], ovalid[order_o]
        assert np.array_equal(gvalid, ovalid), nm
        if ov.dtype == np.float64:
            g, o = gv[ovalid].astype(np.float64), ov[ovalid]
            assert np.array_equal(np.isnan(g), np.isnan(o)), nm
            m = ~np.isnan(o)
            assert np.array_equal(_bits(g)[m], _bits(o)[m]), (nm, g[m][:3], o[m][:3])
        else:
            assert np.array_equal(gv[ovalid].astype(np.int64), ov[ovalid].astype(np.int64)), nm


@pytest.mark.parametrize("n", [1, 1000, 1023, 1025, 300_001])
@pytest.mark.parametrize("pred", [False, True])
def test_fused_derived_inputs_vs_oracle(gpu, n, pred):
    """x op y inputs in the fused kernel (every row: full tiles and the
    masked tail tile), with and without the fused predicate."""
    rng = np.random.default_rng(n + int(pred))
    df, cols = _frame(rng, n)
    p = col("c") > 250.0 if pred else None
    for part in (DERIVED[:4], DERIVED[4:]):  # at most 6 aggregated inputs per call
        exprs = [f().alias(nm) for nm, f in part]
        lf = df.lazy()
        if pred:
            lf = lf.filter(p)
        info = {}
        out = lf.group_by("k").agg(*exprs).collect(info=info)
        if n >= 1024:
            assert info["path"] in (1, 2), info  # the fused kernel
        names = ["k", "a", "b", "c"]
        ea = [(e.args[0].op, e.args[0].args[0]) for e in exprs]
        okeys, _, oouts = _oracle(cols, names, "k", ea, p, n)
        _compare(out, "k", okeys, oouts, [nm for nm, _ in part])


def test_fused_derived_sum_only_vwap(gpu):
    """The VWAP form: (close * volume).sum() / volume.sum() inputs, sum-only
    fused kernel (path 2), 2-limb and register-accumulator (sorted keys)
    variants."""
    rng = np.random.default_rng(9)
    n = 400_000
    close = rng.uniform(100, 200, n)
    vol = rng.uniform(1e3, 1e5, n)
    for sorted_keys in (False, True):
        k = rng.integers(0, 50, n).astype(np.int64)
        if sorted_keys:
            k = np.sort(k)
        df = pl.DataFrame({"k": pl.Series.from_numpy("k", k), "close": pl.Series.from_numpy("close", close),
                           "volume": pl.Series.from_numpy("volume", vol)})
        info = {}
        out = df.lazy().group_by("k").agg((col("close") * col("volume")).sum().alias("pv"),
                                          col("volume").sum().alias("v")).collect(info=info)
        assert info["path"] == 2, info
        cols = {"k": (k, None), "close": (close, None), "volume": (vol, None)}
        okeys, _, oouts = _oracle(cols, ["k", "close", "volume"], "k",
                                  [("sum", col("close") * col("volume")), ("sum", col("volume"))], None, n)
        _compare(out, "k", okeys, oouts, ["pv", "v"])


@pytest.mark.parametrize("n", [1025, 100_003, 1_000_001])
@pytest.mark.parametrize("form", ["one_acc", "vwap", "vwap_rev", "vwap_swap", "three_accs", "literal"])
@pytest.mark.parametrize("pred", ["none", "on_a", "on_b", "other"])
def test_derived_forms_over_two_columns(gpu, n, form, pred):
    """Sum / mean aggregations whose inputs are drawn from two Float64 columns
    a, b -- a op b, b op a, a op literal, a or b itself -- on the sum-only
    fused kernel (path 2) with the predicate on a, on b (the predicate reuses
    an operand's registers) or on a third column, across the masked tail
    tile; bit-exact against the oracle.  The vwap forms (a product and one of
    its operands, in either order, the operand first or second in the
    product) run the product-pair variant (gb_fast_kernel VAR 2 / 3)."""
    rng = np.random.default_rng(n + len(form) * 3 + len(pred))
    k = rng.integers(0, 64, n).astype(np.int64)
    a = rng.uniform(100, 200, n)
    b = rng.uniform(1e3, 1e5, n)
    c = rng.uniform(-1, 1, n)
    df = pl.DataFrame({"k": pl.Series.from_numpy("k", k), "a": pl.Series.from_numpy("a", a),
                       "b": pl.Series.from_numpy("b", b), "c": pl.Series.from_numpy("c", c)})
    forms = {
        "one_acc": [("sum", col("a") - col("b"))],
        "vwap": [("sum", col("a") * col("b")), ("sum", col("b"))],
        "vwap_rev": [("sum", col("b")), ("sum", col("a") * col("b"))],
        "vwap_swap": [("mean", col("b") * col("a")), ("sum", col("b"))],
        "three_accs": [("sum", col("b") / col("a")), ("mean", col("a")), ("sum", col("b") + col("a"))],
        "literal": [("sum", col("a") * 2.5), ("mean", col("b") - col("a"))],
    }[form]
    p = {"none": None, "on_a": col("a") > 150.0, "on_b": col("b") < 5e4, "other": col("c") > 0.0}[pred]
    lf = df.lazy()
    if p is not None:
        lf = lf.filter(p)
    names = [f"o{i}" for i in range(len(forms))]
    info = {}
    out = lf.group_by("k").agg(*[getattr(e, op)().alias(nm) for (op, e), nm in zip(forms, names)]).collect(info=info)
    assert info["path"] == 2, info
    cols = {"k": (k, None), "a": (a, None), "b": (b, None), "c": (c, None)}
    okeys, _, oouts = _oracle(cols, ["k", "a", "b", "c"], "k", forms, p, n)
    _compare(out, "k", okeys, oouts, names)


def test_derived_inputs_off_the_fused_path(gpu):
    """Nullable operands (generic kernel), many groups (partitioned path),
    several keys and a String key: the fused inputs are materialised there,
    with the same results."""
    rng = np.random.default_rng(11)
    n = 1_200_000
    df, cols = _frame(rng, n, nulls=True, nkeys=100)
    exprs = [(col("a") * col("b")).sum().alias("ab"), (col("b") + col("c")).mean().alias("bc")]
    ea = [("sum", col("a") * col("b")), ("mean", col("b") + col("c"))]
    out = df.lazy().group_by("k").agg(*exprs).collect()
    okeys, _, oouts = _oracle(cols, ["k", "a", "b", "c"], "k", ea, None, n)
    _compare(out, "k", okeys, oouts, ["ab", "bc"])
    # many groups: the partitioned path (null-free operands)
    df2, cols2 = _frame(rng, n, nulls=False, nkeys=200_000)
    info = {}
    exprs2 = [(col("b") * col("c")).sum().alias("bc"), col("b").sum().alias("b")]
    out2 = df2.lazy().group_by("k").agg(*exprs2).collect(info=info)
    okeys2, _, oouts2 = _oracle(cols2, ["k", "b", "c"], "k", [("sum", col("b") * col("c")), ("sum", col("b"))],
                                None, n)
    _compare(out2, "k", okeys2, oouts2, ["bc", "b"])
    # two keys (packed) and a String key
    s = np.array(["AAPL", "MSFT", "X", "BRK.B"])[rng.integers(0, 4, 5000)]
    q = rng.integers(0, 3, 5000).astype(np.int32)
    x = rng.standard_normal(5000)
    y = rng.standard_normal(5000)
    df3 = pl.DataFrame({"s": pl.Series.from_arrow("s", __import__("pyarrow").array(s.tolist())),
                        "q": pl.Series.from_numpy("q", q), "x": pl.Series.from_numpy("x", x),
                        "y": pl.Series.from_numpy("y", y)})
    for by in (("s",), ("s", "q")):
        out3 = df3.lazy().group_by(*by, maintain_order=True).agg((col("x") * col("y")).sum().alias("xy"))
        out3 = out3.collect()
        keys = [tuple(r) for r in zip(*[out3[b].to_list() for b in by])]
        for kk, v in zip(keys, out3["xy"].to_list()):
            m = np.ones(5000, bool)
            for b, kv in zip(by, kk):
                m &= (s == kv) if b == "s" else (q == kv)
            assert v == math.fsum(x[m] * y[m])


def test_materialised_inputs_vs_oracle(gpu):
    """Expressions outside the fused form: integer arithmetic, casts, a
    when/then/otherwise over a String comparison, a Boolean input."""
    import pyarrow as pa

    rng = np.random.default_rng(13)
    n = 100_000
    k = rng.integers(0, 20, n).astype(np.int64)
    qty = rng.integers(1, 1000, n).astype(np.int64)
    px = rng.uniform(1, 10, n)
    side = np.array(["B", "S"])[rng.integers(0, 2, n)]
    df = pl.DataFrame({"k": pl.Series.from_numpy("k", k), "qty": pl.Series.from_numpy("qty", qty),
                       "px": pl.Series.from_numpy("px", px), "side": pl.Series.from_arrow("side", pa.array(side))})
    out = df.lazy().group_by("k").agg(
        (col("qty") * 2).sum().alias("q2"),
        (col("qty").cast(pl.Float64) * col("px")).sum().alias("notional"),
        when(col("side") == "B").then(col("qty")).otherwise(0).sum().alias("bought"),
        (col("px") > 5.0).sum().alias("n_hi"),
        (col("px") > 5.0).mean().alias("f_hi"),
    ).collect()
    assert out["n_hi"].dtype == pl.UInt32
    got = {kk: i for i, kk in enumerate(out["k"].to_list())}
    for g in range(20):
        m = k == g
        i = got[g]
        assert out["q2"].to_list()[i] == int((qty[m] * 2).sum())
        assert out["notional"].to_list()[i] == math.fsum(qty[m].astype(np.float64) * px[m])
        assert out["bought"].to_list()[i] == int(qty[m & (side == "B")].sum())
        assert out["n_hi"].to_list()[i] == int((px[m] > 5.0).sum())
        assert out["f_hi"].to_list()[i] == float((px[m] > 5.0).sum()) / m.sum()


@pytest.mark.parametrize("n", [0, 1, 777, 1025, 250_000])
def test_global_reductions_vs_oracle(gpu, n):
    """select(aggs) with and without a predicate, over columns and computed
    inputs; no selected row gives the reference's empty reductions."""
    rng = np.random.default_rng(n + 3)
    df, cols = _frame(rng, n, nulls=True)
    names = ["a", "b", "c", "q"]
    aggs = [("sum", col("a")), ("mean", col("a")), ("min", col("a")), ("max", col("c")), ("count", col("a")),
            ("len", None), ("first", col("a")), ("last", col("c")), ("sum", col("q")),
            ("sum", col("b") * col("c")), ("mean", col("c") - 100.0)]
    outn = [f"o{i}" for i in range(len(aggs))]
    exprs = [(pl.len() if x is None else getattr(x, kind)()).alias(nm) for (kind, x), nm in zip(aggs, outn)]
    for pred in (None, col("c") > 400.0, col("c") > 1e9):
        lf = df.lazy()
        if pred is not None:
            lf = lf.filter(pred)
        out = lf.select(*exprs).collect()
        assert out.height == 1
        okeys, _, oouts = _oracle(cols, names, None, aggs, pred, n)
        _compare(out, None, okeys, oouts, outn)


def test_global_reduction_fast_paths(gpu):
    """Keyless sums on the fused sum-only kernel (one group, the sorted-key
    register accumulators) and mixed aggregations, at 2e7 rows, exact."""
    import torch

    n = 20_000_000
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    a = torch.rand(n, device="cuda", generator=g, dtype=torch.float64) * 100 + 1
    b = torch.rand(n, device="cuda", generator=g, dtype=torch.float64) + 0.5
    df = pl.DataFrame([pl.Series.from_torch("a", a), pl.Series.from_torch("b", b)])
    info = {}
    out = df.lazy().select(col("a").sum().alias("sa"), (col("a") * col("b")).sum().alias("sab")).collect(info=info)
    assert info["path"] == 2 and info["groups"] == 1
    ha, hb = a.cpu().numpy(), b.cpu().numpy()
    assert out["sa"].to_list()[0] == math.fsum(ha)
    assert out["sab"].to_list()[0] == math.fsum(ha * hb)
    out = df.lazy().filter(col("b") > 1.0).select(col("a").min().alias("mn"), col("a").max().alias("mx"),
                                                  pl.len().alias("n"), col("b").mean().alias("mb")).collect()
    sel = hb > 1.0
    assert out["mn"].to_list()[0] == ha[sel].min() and out["mx"].to_list()[0] == ha[sel].max()
    assert out["n"].to_list()[0] == int(sel.sum())
    assert out["mb"].to_list()[0] == math.fsum(hb[sel]) / sel.sum()


def test_var_std_of_expressions_and_global(gpu):
    rng = np.random.default_rng(17)
    n = 50_000
    df, cols = _frame(rng, n)
    out = df.lazy().group_by("k").agg((col("a") * col("b")).std().alias("s"), col("c").var(0).alias("v")).collect()
    a, b, c, k = cols["a"][0], cols["b"][0], cols["c"][0], cols["k"][0]
    for kk, s_, v_ in zip(out["k"].to_list(), out["s"].to_list(), out["v"].to_list()):
        m = k == kk
        x = a[m] * b[m]
        mean = math.fsum(x) / x.size
        assert math.isclose(s_, math.sqrt(math.fsum((x - mean) ** 2) / (x.size - 1)), rel_tol=1e-12)
        mc = math.fsum(c[m]) / m.sum()
        assert math.isclose(v_, math.fsum((c[m] - mc) ** 2) / m.sum(), rel_tol=1e-12)
    g = df.lazy().select(col("c").std().alias("s")).collect()["s"].to_list()[0]
    mc = math.fsum(c) / n
    assert math.isclose(g, math.sqrt(math.fsum((c - mc) ** 2) / (n - 1)), rel_tol=1e-12)
