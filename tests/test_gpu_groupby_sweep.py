"""Forced-path parity sweep of the group-by (round 5): every kernel path the
plan can take, crossed with the aggregated-column count (1-6), maintain_order,
the predicate form (none / fused simple / program) and nullable keys or
values, each result compared bit for bit with the oracle -- first-occurrence
order included under maintain_order.

Paths are forced with the library's test hooks (plgpu_set_option):
  gb_path 0  generic kernel on the global table
  gb_path 1  generic kernel with LDS tables
  gb_path 2  fused kernel (sum-only / mixed layouts by the aggregations)
  gb_path 2 + runs 1   the fused kernel's register-run variants
  gb_path 3  partitioned: one scatter pass (part_levels 1) / two (2)
  auto       the plan's own choice
Where the inputs rule a path out (nulls for the fused and partitioned paths,
4-byte columns and program predicates for the fused kernel), the plan takes
the next path that accepts them; `_expect_path` states which, so a path
refusing more than DESIGN.md "Group-by paths" lists is a failure too (since
round 6 no path refuses validity bitmaps).  The
derived-input (DERIV), variance-triple (VAR), keyless, packed multi-key
(PACK 1), String-key (PACK 2), sorted-key (RUNS), range-local (time-ordered
keys) and wide-sum variants are crossed with the same paths below.

This is the class of test that would have caught the partition scatter's
row-id bug of rounds 2-3 (DESIGN.md "Multi-key operators", round-4 fix).
Reference: polars-core/src/frame/group_by/aggregations/mod.rs:581,
polars-expr/src/reduce/*.
"""

import math

import numpy as np
import pytest

import polaroid_amd as pl
from oracle import oracle as O
from polaroid_amd.expr import col, lower

pytestmark = pytest.mark.gpu

I64_MIN = np.iinfo(np.int64).min

PATHS = {
    "auto": {},
    "generic_global": {"gb_path": 0},
    "generic_lds": {"gb_path": 1},
    "fused": {"gb_path": 2},
    "fused_runs": {"gb_path": 2, "runs": 1},
    "part1": {"gb_path": 3, "part_levels": 1, "part_bits": 6},
    "part2": {"gb_path": 3, "part_levels": 2, "part_bits": 10},
}

N = 200_003


def _bits(a):
    return np.asarray(a, dtype=np.float64).view(np.uint64)


def _data(seed, n=N, card=300, sorted_keys=False):
    rng = np.random.default_rng(seed)
    k = (rng.integers(0, card, n) * 7919 - 5).astype(np.int64)
    k[rng.random(n) < 0.002] = I64_MIN
    if sorted_keys:
        k = np.sort(k)
    kv = rng.random(n) > 0.02
    c = rng.uniform(10, 500, n)
    b = rng.uniform(0.5, 2.0, n)
    a = rng.standard_normal(n) * 100
    a[rng.random(n) < 0.001] = np.nan
    a[rng.random(n) < 0.0005] = np.inf
    a[rng.random(n) < 0.002] = -0.0
    d = rng.uniform(-5, 5, n)
    e = c * rng.uniform(0.99, 1.01, n)
    f = rng.uniform(1, 1000, n)
    q = rng.integers(-10**12, 10**12, n).astype(np.int64)
    i = rng.integers(-50, 50, n).astype(np.int32)
    an_valid = rng.random(n) > 0.05
    cols = {"k": (k, None), "kn": (k, kv), "c": (c, None), "b": (b, None), "a": (a, None), "d": (d, None),
            "e": (e, None), "f": (f, None), "q": (q, None), "i": (i, None), "an": (a, an_valid),
            "cn": (c, an_valid)}
    df = pl.DataFrame({nm: pl.Series.from_numpy(nm, v, m) for nm, (v, m) in cols.items()})
    return df, cols


# aggregated-column families: (kind, column) per distinct column
SUMONLY = [("sum", "c"), ("mean", "b"), ("sum", "e"), ("sum", "f"), ("mean", "d"), ("sum", "a")]
MIXED = [("sum", "c"), ("min", "q"), ("max", "a"), ("first", "b"), ("last", "d"), ("count", "f")]
MIXED_NULLS = [("sum", "cn"), ("min", "q"), ("max", "an"), ("first", "b"), ("last", "d"), ("count", "an")]
NARROW = [("sum", "i"), ("max", "c"), ("mean", "i"), ("min", "c"), ("len", "c"), ("sum", "q")]

PREDS = {
    "none": None,
    "simple": lambda: col("c") > 250.0,
    "program": lambda: ((col("b") * 2.0 + col("d")) > 3.0) & (col("q") > -(10**11)),
}


def _oracle(cols, key, specs, pred, n, names_extra=()):
    """Oracle result (keys, key_valid, [(values, valid)]) for aggregations
    (kind, input expr or None for len) under `pred` (an expr or None)."""
    names = list(dict.fromkeys(["c", "b", "d", "q"] + list(names_extra) +
                               [x.value for _, x in specs if x is not None and x.kind == "col"]))
    hc = [O.HostCol(cols[nm][0], cols[nm][1]) for nm in names]
    idx = {nm: i for i, nm in enumerate(names)}
    schema = {nm: c.code for nm, c in zip(names, hc)}
    inputs, aggs = [], []
    for kind, x in specs:
        if x is None:
            aggs.append(("len", 0))
        elif x.kind == "col":
            aggs.append((kind, idx[x.value]))
        else:
            inputs.append(lower(x, idx, schema))
            aggs.append((kind, len(hc) + len(inputs) - 1))
    prog = lower(pred, idx, schema) if pred is not None else None
    kc = None if key is None else O.HostCol(cols[key][0], cols[key][1])
    return O.group_by_agg_inputs(kc, hc, prog, inputs, aggs, n)


def _gpu(df, key, specs, pred, maintain):
    exprs = [(pl.len() if x is None else getattr(x, kind)()).alias(f"o{j}") for j, (kind, x) in enumerate(specs)]
    lf = df.lazy()
    if pred is not None:
        lf = lf.filter(pred)
    info = {}
    if key is None:
        out = lf.select(*exprs).collect(info=info)
    else:
        out = lf.group_by(key, maintain_order=maintain).agg(*exprs).collect(info=info)
    return out, info


def _compare(out, key, exp, nspecs, maintain, tag):
    okeys, okvalid, oouts = exp
    assert out.height == okeys.shape[0], tag
    if key is None:
        go = oo = np.arange(out.height)
    else:
        gk, gkv = out[key].to_numpy().astype(np.int64), out[key].validity_numpy()
        if maintain:
            go, oo = np.arange(gk.shape[0]), np.arange(okeys.shape[0])
        else:
            go, oo = np.lexsort((gk, ~gkv)), np.lexsort((okeys, ~okvalid))
        assert np.array_equal(gkv[go], okvalid[oo]), tag
        assert np.array_equal(gk[go][gkv[go]], okeys[oo][okvalid[oo]]), tag
    for j in range(nspecs):
        s = out[f"o{j}"]
        gv, gvalid = s.to_numpy()[go], s.validity_numpy()[go]
        ov, ovalid = oouts[j][0][oo], oouts[j][1][oo]
        assert np.array_equal(gvalid, ovalid), (tag, j)
        if ov.dtype == np.float64:
            g, o = gv[ovalid].astype(np.float64), ov[ovalid]
            assert np.array_equal(np.isnan(g), np.isnan(o)), (tag, j)
            m = ~np.isnan(o)
            assert np.array_equal(_bits(g)[m], _bits(o)[m]), (tag, j, g[m][:3], o[m][:3])
        else:
            assert np.array_equal(gv[ovalid].astype(np.int64), ov[ovalid].astype(np.int64)), (tag, j)


def _expect_path(path, key_nulls, val_nulls, narrow, pred, sum_only, maintain):
    """The info["path"] a forced path must report for these inputs (None:
    not asserted).  DESIGN.md "Group-by paths" lists the refusals."""
    opts = PATHS[path]
    gp = opts.get("gb_path", -1)
    if gp in (0, 1):
        return 0
    if gp == 2:
        if narrow or pred == "program":
            return 0                      # the fused kernel needs 8-byte columns and a simple predicate
        # (validity bitmaps: the NULLS variant, round 6)
        return 2 if sum_only and not maintain else 1   # maintain_order: the first-row field
    if gp == 3:
        return 3                          # null bits travel with the partitioned rows (round 6)
    return None


def _set(plgpu_option, path):
    for k, v in PATHS[path].items():
        plgpu_option(k, v)


@pytest.fixture(scope="module")
def frame():
    return _data(2024)


@pytest.mark.parametrize("path", list(PATHS))
def test_sweep_paths_x_columns_x_order_x_predicate(gpu, path, frame, plgpu_option):
    """Every path x 1-6 aggregated columns (sum-only, mixed, nullable,
    4-byte) x maintain_order x predicate x nullable key, bit-exact."""
    df, cols = frame
    _set(plgpu_option, path)
    families = {"sumonly": SUMONLY, "mixed": MIXED, "nulls": MIXED_NULLS, "narrow": NARROW}
    cache = {}
    for fam, pool in families.items():
        for ncol in range(1, 7):
            specs = [(kind, col(c)) for kind, c in pool[:ncol]]
            if fam == "narrow" and ncol >= 5:
                specs[4] = ("len", None)
            for pname, pf in PREDS.items():
                for key in ("k", "kn"):
                    if fam in ("nulls", "narrow") and key == "kn" and pname == "program":
                        continue  # covered by the other families' nullable-key cases
                    ck = (fam, ncol, pname, key)
                    if ck not in cache:
                        cache.clear()
                        cache[ck] = _oracle(cols, key, specs, pf() if pf else None, N)
                    for maintain in (False, True):
                        out, info = _gpu(df, key, specs, pf() if pf else None, maintain)
                        tag = (path, fam, ncol, pname, key, maintain, info.get("path"))
                        _compare(out, key, cache[ck], len(specs), maintain, tag)
                        sum_only = all(kind in ("sum", "mean") and cols[c][0].dtype == np.float64
                                       for kind, c in pool[:ncol]) and fam != "narrow"
                        want = _expect_path(path, key == "kn", fam == "nulls", fam == "narrow", pname,
                                            sum_only, maintain)
                        if want is not None:
                            assert info["path"] == want or (want == 2 and info["path"] == 4), tag


DERIVED = [
    ("sum", lambda: col("c") * col("b")),
    ("sum", lambda: col("b")),
    ("mean", lambda: col("a") / col("b")),
    ("sum", lambda: col("c") - 250.0),
    ("max", lambda: col("d") * 1.5),
    ("sum", lambda: col("e") + col("f")),
]


@pytest.mark.parametrize("path", list(PATHS))
def test_sweep_derived_inputs(gpu, path, frame, plgpu_option):
    """Aggregations over x op y (the fused kernel's DERIV variant; the other
    paths take them materialised) x 1-6 inputs x maintain_order x predicate."""
    df, cols = frame
    _set(plgpu_option, path)
    for ncol in (1, 2, 4, 6):
        specs = [(kind, f()) for kind, f in DERIVED[:ncol]]
        for pname, pf in PREDS.items():
            exp = _oracle(cols, "k", specs, pf() if pf else None, N, names_extra=("a", "e", "f"))
            for maintain in (False, True):
                out, info = _gpu(df, "k", specs, pf() if pf else None, maintain)
                _compare(out, "k", exp, len(specs), maintain, (path, ncol, pname, maintain, info.get("path")))


@pytest.mark.parametrize("path", list(PATHS))
def test_sweep_keyless(gpu, path, frame, plgpu_option):
    """select(aggs): the keyless form of every path (one group)."""
    df, cols = frame
    _set(plgpu_option, path)
    for specs in ([("sum", col("c"))], [(k, col(c)) for k, c in SUMONLY], [(k, col(c)) for k, c in MIXED_NULLS],
                  [("len", None), ("sum", col("c") * col("b"))]):
        for pname, pf in PREDS.items():
            exp = _oracle(cols, None, specs, pf() if pf else None, N, names_extra=("a", "e", "f", "an", "cn"))
            out, info = _gpu(df, None, specs, pf() if pf else None, False)
            _compare(out, None, exp, len(specs), False, (path, len(specs), pname, info.get("path")))


@pytest.mark.parametrize("path", list(PATHS))
def test_sweep_sorted_keys(gpu, path, plgpu_option):
    """Symbol-sorted rows (every wave sees one or two groups: the register
    runs) with sum-only and mixed aggregations."""
    df, cols = _data(77, sorted_keys=True)
    _set(plgpu_option, path)
    for pool in (SUMONLY, MIXED):
        for ncol in (1, 3, 6):
            specs = [(kind, col(c)) for kind, c in pool[:ncol]]
            for pname in ("none", "simple"):
                pf = PREDS[pname]
                exp = _oracle(cols, "k", specs, pf() if pf else None, N)
                for maintain in (False, True):
                    out, info = _gpu(df, "k", specs, pf() if pf else None, maintain)
                    _compare(out, "k", exp, len(specs), maintain, (path, ncol, pname, maintain, info.get("path")))


@pytest.mark.parametrize("path", ["auto", "generic_global", "part2"])
def test_sweep_range_local(gpu, path, plgpu_option):
    """Time-ordered keys (the range-local fused table: each workgroup one
    contiguous run of tiles, its LDS table sized for that range's keys) x
    1-6 aggregated columns (sum-only and mixed) x maintain_order x predicate,
    and the same frame forced onto the global table and the partitioned
    path.  Exact vs the oracle, first-occurrence order included."""
    rng = np.random.default_rng(31)
    n = 4_500_001
    day = (np.arange(n) * 200) // n
    k = (rng.integers(0, 150, n) + 1000 * day).astype(np.int64)  # 30k groups, 150 per row range
    c = rng.uniform(10, 500, n)
    cols = {"k": (k, None), "c": (c, None), "b": (rng.uniform(0.5, 2.0, n), None),
            "a": (rng.standard_normal(n) * 100, None), "d": (rng.uniform(-5, 5, n), None),
            "e": (c * rng.uniform(0.99, 1.01, n), None), "f": (rng.uniform(1, 1000, n), None),
            "q": (rng.integers(-10**12, 10**12, n).astype(np.int64), None)}
    df = pl.DataFrame({nm: pl.Series.from_numpy(nm, v, m) for nm, (v, m) in cols.items()})
    _set(plgpu_option, path)
    saw_local = False
    for pool in (SUMONLY, MIXED[:3] + [("max", "e"), ("count", "f"), ("sum", "q")]):
        for ncol in (1, 2, 4, 6):
            specs = [(kind, col(c_)) for kind, c_ in pool[:ncol]]
            for pname in ("none", "simple", "program"):
                pf = PREDS[pname]
                exp = _oracle(cols, "k", specs, pf() if pf else None, n)
                for maintain in (False, True):
                    out, info = _gpu(df, "k", specs, pf() if pf else None, maintain)
                    tag = (path, ncol, pname, maintain, info.get("path"), info.get("local_range"))
                    _compare(out, "k", exp, len(specs), maintain, tag)
                    if info["local_range"]:
                        saw_local = True
                        assert info["path"] in (1, 2), tag
                    if path != "auto" or pname == "program":
                        assert info["local_range"] == 0, tag  # the fused kernel only
    # (the plan takes the range-local table while a range's keys fit one LDS
    # table in the full layout: the narrower column counts here)
    assert saw_local == (path == "auto")


def _var_check(out, cols, key, xname, ddof, pred_mask, maintain, tag):
    k = cols[key][0]
    x = cols[xname][0]
    sel = pred_mask
    first = {}
    groups = {}
    for r in np.nonzero(sel)[0]:
        kk = int(k[r])
        groups.setdefault(kk, []).append(x[r])
        first.setdefault(kk, r)
    keys = out[key].to_list()
    assert len(keys) == len(groups), tag
    if maintain:
        assert keys == sorted(groups, key=lambda g: first[g]), tag
    vals = out["v"].to_list()
    for kk, v in zip(keys, vals):
        xs = groups[kk]
        if len(xs) <= ddof:
            assert v is None, tag
            continue
        if any(not math.isfinite(t) for t in xs):
            assert v is not None and math.isnan(v), tag
            continue
        m = math.fsum(xs) / len(xs)
        ref = math.fsum((t - m) ** 2 for t in xs) / (len(xs) - ddof)
        assert v is not None and abs(v - ref) <= 1e-12 * max(abs(ref), 1e-300), (tag, kk, v, ref)


@pytest.mark.parametrize("path", list(PATHS))
def test_sweep_var_std(gpu, path, plgpu_option):
    """var / std (the variance-triple kernel on the fused path; exact
    sums of x, x * x and its error elsewhere) x maintain_order x predicate."""
    df, cols = _data(91, n=60_001, card=40)
    _set(plgpu_option, path)
    for xname in ("c", "a"):
        for ddof in (0, 1):
            for pname in ("none", "simple"):
                pf = PREDS[pname]
                mask = np.ones(60_001, bool) if pf is None else cols["c"][0] > 250.0
                for maintain in (False, True):
                    lf = df.lazy()
                    if pf is not None:
                        lf = lf.filter(pf())
                    out = lf.group_by("k", maintain_order=maintain).agg(col(xname).var(ddof=ddof).alias("v")).collect()
                    _var_check(out, cols, "k", xname, ddof, mask, maintain, (path, xname, ddof, pname, maintain))


@pytest.mark.parametrize("path", list(PATHS))
def test_sweep_multi_key_and_string_key(gpu, path, frame, plgpu_option):
    """Packed integer key pairs (PACK 1: the codes formed in the fused
    kernel) and a short String key (PACK 2), exact vs the oracle's row
    encoding, under every path."""
    df, cols = frame
    _set(plgpu_option, path)
    n = N
    rng = np.random.default_rng(5)
    day = rng.integers(0, 20, n).astype(np.int32)
    syms = np.array([f"S{j:03d}" for j in range(60)])
    sidx = rng.integers(0, 60, n)
    df2 = pl.DataFrame({"sym": pl.Series.from_numpy("sym", cols["k"][0]), "day": pl.Series.from_numpy("day", day),
                        "ticker": pl.Series("ticker", syms[sidx].tolist(), pl.String),
                        "c": pl.Series.from_numpy("c", cols["c"][0]), "b": pl.Series.from_numpy("b", cols["b"][0]),
                        "q": pl.Series.from_numpy("q", cols["q"][0])})
    hc = [O.HostCol(cols["c"][0]), O.HostCol(cols["b"][0]), O.HostCol(cols["q"][0])]
    prog = [(1, 0, 0), (2, 0, 250.0), (24, 0, 0)]
    for keys, kcols in ((("sym", "day"), [(cols["k"][0], None), (day, None)]),
                        (("ticker",), [(sidx.astype(np.int64), None)])):
        for aggs in ([("sum", 0), ("sum", 1)], [("sum", 0), ("min", 2), ("max", 1), ("len", 0)]):
            for pred in (False, True):
                okeys, oouts = O.group_by_agg_multi(kcols, hc, prog if pred else None, aggs, n)
                for maintain in (False, True):
                    lf = df2.lazy()
                    if pred:
                        lf = lf.filter(col("c") > 250.0)
                    out = lf.group_by(*keys, maintain_order=maintain).agg(
                        *[getattr(col(["c", "b", "q"][ci]), kind)().alias(f"o{j}")
                          for j, (kind, ci) in enumerate(aggs)]).collect()
                    tag = (path, keys, len(aggs), pred, maintain)
                    assert out.height == okeys[0][0].shape[0], tag
                    if keys == ("ticker",):
                        gk = [[int(np.nonzero(syms == t)[0][0]) for t in out["ticker"].to_list()]]
                    else:
                        gk = [out[k].to_numpy().astype(np.int64) for k in keys]
                    ok = [ov.astype(np.int64) for ov, _ in okeys]
                    if maintain:
                        go = oo = np.arange(out.height)
                    else:
                        go, oo = np.lexsort(tuple(gk[::-1])), np.lexsort(tuple(ok[::-1]))
                    for g, o in zip(gk, ok):
                        assert np.array_equal(np.asarray(g)[go], o[oo]), tag
                    for j, (kind, ci) in enumerate(aggs):
                        gv = out[f"o{j}"].to_numpy()[go]
                        ov = oouts[j][0][oo]
                        if ov.dtype == np.float64:
                            assert np.array_equal(_bits(gv), _bits(ov)), (tag, j)
                        else:
                            assert np.array_equal(gv.astype(np.int64), ov.astype(np.int64)), (tag, j)


@pytest.mark.parametrize("path", list(PATHS))
def test_sweep_wide_sums(gpu, path, plgpu_option):
    """A column whose values span more binades than one fixed-point window
    (1e300 next to 1e-300): the exact wide fallback under every path."""
    rng = np.random.default_rng(13)
    n = 100_003
    k = (rng.integers(0, 50, n) * 31).astype(np.int64)
    w = rng.standard_normal(n) * 1e-300
    w[rng.random(n) < 0.01] = 1e300
    w[rng.random(n) < 0.01] = -1e300
    c = rng.uniform(10, 500, n)
    cols = {"k": (k, None), "w": (w, None), "c": (c, None), "b": (c, None), "d": (c, None), "q": (k, None)}
    df = pl.DataFrame({"k": pl.Series.from_numpy("k", k), "w": pl.Series.from_numpy("w", w),
                       "c": pl.Series.from_numpy("c", c), "b": pl.Series.from_numpy("b", c),
                       "d": pl.Series.from_numpy("d", c), "q": pl.Series.from_numpy("q", k)})
    _set(plgpu_option, path)
    specs = [("sum", col("w")), ("sum", col("c")), ("mean", col("w"))]
    for pname in ("none", "simple"):
        pf = PREDS[pname]
        exp = _oracle(cols, "k", specs, pf() if pf else None, n, names_extra=("w",))
        for maintain in (False, True):
            out, info = _gpu(df, "k", specs, pf() if pf else None, maintain)
            _compare(out, "k", exp, len(specs), maintain, (path, pname, maintain, info.get("path")))


def test_partition_launchers_refuse_a_keyless_reduction(gpu, frame, plgpu_option):
    """gb_path 5 skips the plan's input checks and forces the partitioned
    path: the partition launchers' own precondition (groupby.hip
    gb_partition) must turn a keyless reduction -- round 5's r05c fault, a
    null key column read by gbp_count_kernel -- into InvalidOperationError,
    never a device access; a nullable key is taken (its null bits travel
    with the rows) and stays exact."""
    df, cols = frame
    plgpu_option("gb_path", 5)
    with pytest.raises(pl.InvalidOperationError, match="partitioned group-by"):
        df.lazy().select(col("c").sum().alias("o0")).collect()
    specs = [("sum", col("cn")), ("min", col("an")), ("count", col("an"))]
    exp = _oracle(cols, "kn", specs, None, N, names_extra=("an", "cn"))
    out, info = _gpu(df, "kn", specs, None, False)
    assert info["path"] == 3
    _compare(out, "kn", exp, len(specs), False, ("gb_path 5", info.get("path")))
