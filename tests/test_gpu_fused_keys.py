"""Fused key packing and Categorical keys (round 4).

* Several integer keys (and one Int32 / UInt32 key) of a large input are
  packed into the exact Int64 tuple code (mk_plan_pack's layout) inside the
  fused group-by kernel's registers: no code column is written or read
  (info["key_pack"] = the number of key columns packed in the kernel).
  Checked bit-exact against the oracle's row-encoding restatement
  (oracle.group_by_agg_multi, polars-core/src/chunked_array/ops/
  row_encode.rs), against the code-column path (option fuse_keys = 0) on the
  same data, through the sampled plan's repack (an outlier row) and through
  the fallbacks (many groups, derived inputs).
* A Categorical column (an Arrow dictionary array: polars' export) groups
  by its UInt32 codes (polars-core/src/frame/group_by/into_groups.rs:132-139
  groups a Categorical by its physical codes); the strings are gathered only
  for the output keys (info["categorical_codes"]).  Pinned by the fixtures of
  tests/golden/categorical_cases.json (test_group_by.py:903-957 with nulls
  and maintain_order, test_categorical.py:104-118 two chunks, an empty key).
"""

import math

import numpy as np
import pyarrow as pa
import pytest

import polaroid_amd as pl
from conftest import load_golden
from oracle import oracle as O
from test_gpu_groupby_multi import _check
from test_gpu_parity import _rand_frame

pytestmark = pytest.mark.gpu

N = 1_500_003  # above the sampled-plan / fused-packing threshold (2^20 rows)


def _dense(rng, n):
    """_rand_frame's columns without validity (the fused kernel's inputs are
    null-free; NaN / inf / -0.0 stay)."""
    return {k: (v, None) for k, (v, _) in _rand_frame(rng, n).items()}


@pytest.mark.parametrize("layout", ["day_ordered", "random"])
@pytest.mark.parametrize("aggs", ["sums", "mixed"])
@pytest.mark.parametrize("pred", [None, "simple_f64"])
def test_fused_two_keys_vs_oracle(gpu, layout, aggs, pred):
    """(symbol: Int64, day: Int32) packed in the fused kernel, exact vs the
    oracle: time-ordered days (range-local table) and random tuples."""
    rng = np.random.default_rng(len(layout) + 3 * len(aggs) + (pred is None))
    # day-ordered: 25,000 groups, ~100 per row range (the range-local table,
    # which needs >= 2^22 rows); random: 120 groups (one LDS table: the
    # mixed aggregations' table layout holds 256 slots at load 1/2)
    n = 4_500_001 if layout == "day_ordered" else N
    nsym = 100 if layout == "day_ordered" else 30
    sym = (rng.integers(0, nsym, n) * 7919 + 1_000_000).astype(np.int64)
    day = ((np.arange(n) * 250) // n).astype(np.int32) if layout == "day_ordered" else \
        rng.integers(0, 4, n).astype(np.int32)
    cols = _dense(rng, n)
    ag = [("sum", "a"), ("sum", "d")] if aggs == "sums" else \
        [("sum", "a"), ("min", "d"), ("max", "b"), ("count", "d"), ("len", "a"), ("mean", "d")]
    info = {}
    _check({"sym": (sym, None), "day": (day, None)}, cols, ag, False, pred, info=info)
    assert info["key_pack"] == 2, info


@pytest.mark.parametrize("dtype", [np.int32, np.uint32])
@pytest.mark.parametrize("maintain_order", [False, True])
def test_fused_single_narrow_key(gpu, dtype, maintain_order):
    """One null-free Int32 / UInt32 key (dates, Categorical codes): the fused
    kernel reads the 4-byte key and packs it (was: the generic kernel)."""
    rng = np.random.default_rng(int(maintain_order) + (dtype == np.uint32) * 2)
    lo = 0 if dtype == np.uint32 else -(1 << 30)
    k = (rng.integers(0, 300, N) * 1_000_003 % (1 << 30) + lo).astype(dtype)
    # the type's extremes and -1 (all-ones in 32 bits) as keys too
    info_ = np.iinfo(dtype)
    k[rng.integers(0, N, 50)] = info_.min
    k[rng.integers(0, N, 50)] = info_.max
    if dtype == np.int32:
        k[rng.integers(0, N, 50)] = -1
    cols = _dense(rng, N)
    info = {}
    _check({"k": (k, None)}, cols, [("sum", "a"), ("len", "b"), ("max", "d")], maintain_order, info=info)
    assert info["key_pack"] == 1, info


def test_fused_matches_code_column_path(gpu, plgpu_option):
    """fuse_keys = 0 (the packed code column) gives the same frame."""
    rng = np.random.default_rng(5)
    sym = rng.integers(0, 100, N).astype(np.int64)
    day = rng.integers(0, 5, N).astype(np.int32)  # 500 groups: one LDS table
    a = rng.uniform(10, 500, N)
    df = pl.DataFrame({"sym": pl.Series.from_numpy("sym", sym), "day": pl.Series.from_numpy("day", day),
                       "a": pl.Series.from_numpy("a", a)})
    q = df.lazy().filter(pl.col("a") > 250.0).group_by("sym", "day", maintain_order=True).agg(
        pl.col("a").sum(), pl.len())
    i1, i0 = {}, {}
    fused = q.collect(info=i1)
    plgpu_option("fuse_keys", 0)
    plain = q.collect(info=i0)
    assert i1["key_pack"] == 2 and i0["key_pack"] == 0
    for c in ("sym", "day", "len"):
        assert fused[c].to_list() == plain[c].to_list()
    assert np.array_equal(fused["a"].to_numpy().view(np.uint64), plain["a"].to_numpy().view(np.uint64))


@pytest.mark.parametrize("outlier", ["i64_high", "i32_low", "i32_high", "i32_negative_base"])
def test_fused_outlier_repacks(gpu, outlier):
    """A row outside the sampled packing plan (far from every sampled key)
    is caught in the fused kernel (ST_KPACK): the group-by repacks with the
    exact ranges and runs fused again, exact.  The Int32 cases take the
    32-bit field test (KeyPack mode 1), below and above the sampled range."""
    rng = np.random.default_rng(9)
    k1 = (rng.integers(0, 40, N) * 3 - 500).astype(np.int64)
    k2 = rng.integers(0, 10, N).astype(np.int32)  # ~400 groups: one LDS table
    if outlier == "i32_negative_base":
        k2 = (k2 - 1_000_000).astype(np.int32)
    r = N // 2 + 7
    if outlier == "i64_high":
        k1[r] = 1 << 40
    elif outlier == "i32_low":
        k2[r] = np.iinfo(np.int32).min + 3
    elif outlier == "i32_high":
        k2[r] = np.iinfo(np.int32).max
    else:
        k2[r] = 2_000_000_000
    cols = _dense(rng, N)
    info = {}
    _check({"k1": (k1, None), "k2": (k2, None)}, cols, [("sum", "a"), ("len", "b")], False, info=info)
    assert info["key_pack"] == 2, info


def test_fused_fallbacks(gpu):
    """Off the fused kernel the code column is used, with the same result:
    many groups (the partitioned / global path) and derived inputs."""
    rng = np.random.default_rng(11)
    n = 2_000_000
    k1 = rng.integers(0, 1000, n).astype(np.int64)
    k2 = rng.integers(0, 1000, n).astype(np.int32)
    cols = {"a": (rng.standard_normal(n), None), "b": (rng.integers(-9, 9, n).astype(np.int64), None)}
    info = {}
    _check({"k1": (k1, None), "k2": (k2, None)}, cols, [("sum", "a"), ("len", "a")], False, info=info)
    assert info["key_pack"] == 0 and info["groups"] > 600_000
    # (a * b).sum(): a derived input fused in registers is not a PACK variant
    df = pl.DataFrame({"k1": pl.Series.from_numpy("k1", k1 % 10), "k2": pl.Series.from_numpy("k2", k2 % 10),
                       "a": pl.Series.from_numpy("a", cols["a"][0]),
                       "b": pl.Series.from_numpy("b", cols["a"][0] * 2.0)})
    info = {}
    out = df.lazy().group_by("k1", "k2").agg((pl.col("a") * pl.col("b")).sum().alias("ab")).collect(info=info)
    assert info["key_pack"] == 0
    got = dict(zip(zip(out["k1"].to_list(), out["k2"].to_list()), out["ab"].to_list()))
    a, b = cols["a"][0], cols["a"][0] * 2.0
    for key in list(got)[:10]:
        m = ((k1 % 10) == key[0]) & ((k2 % 10) == key[1])
        assert got[key] == math.fsum(a[m] * b[m])


def _cat_frame(strings, vals=None, chunks=None):
    """A frame with a Categorical column "c" built as polars exports it: an
    Arrow dictionary array (one chunk, or several with their own dictionaries)."""
    if chunks is None:
        chunks = [strings]
    arrs = [pa.array(ch, pa.string()).dictionary_encode() for ch in chunks]
    s = pl.Series.from_arrow("c", pa.chunked_array(arrs) if len(arrs) > 1 else arrs[0])
    cols = [s]
    if vals is not None:
        cols.append(pl.Series.from_numpy("v", np.asarray(vals)))
    return pl.DataFrame(cols)


def test_categorical_golden(gpu):
    for case in load_golden("categorical_cases.json")["cases"]:
        if "chunks" in case:
            df = _cat_frame(None, case["vals"], case["chunks"])
        else:
            df = _cat_frame(case["key"], np.arange(len(case["key"]), dtype=np.int64))
        info = {}
        out = df.lazy().group_by("c", maintain_order=case["maintain_order"]).agg(pl.len()).collect(info=info)
        got = list(zip(out["c"].to_list(), out["len"].to_list()))
        want = list(zip(case["groups"], case["len"]))
        if not case["maintain_order"]:
            got, want = sorted(got, key=str), sorted(want, key=str)
        assert got == want, case["name"]
        if len(case["groups"]):
            assert info.get("categorical_codes") == 1, (case["name"], info)


@pytest.mark.parametrize("nulls", [False, True])
@pytest.mark.parametrize("maintain_order", [False, True])
def test_categorical_headline_vs_strings(gpu, nulls, maintain_order):
    """The headline query on a Categorical symbol: grouped by the codes
    (fused 4-byte key when null-free) and identical to the same query on the
    String column."""
    rng = np.random.default_rng(int(nulls) * 2 + maintain_order)
    syms = np.array([f"SYM{i:03d}" for i in range(100)], dtype=object)
    k = rng.integers(0, 100, N)
    strs = syms[k].tolist()
    if nulls:
        for i in rng.integers(0, N, 1000):
            strs[i] = None
    close = rng.uniform(10, 490, N)
    df = _cat_frame(strs, close)
    info = {}
    q = df.lazy().filter(pl.col("v") > 250.0).group_by("c", maintain_order=maintain_order).agg(
        pl.col("v").sum().alias("s"), pl.len())
    out = q.collect(info=info)
    assert info["categorical_codes"] == 1
    assert info["key_pack"] == (0 if nulls else 1), info
    sdf = pl.DataFrame([pl.Series("c", strs, pl.String), pl.Series.from_numpy("v", close)])
    ref = sdf.lazy().filter(pl.col("v") > 250.0).group_by("c", maintain_order=maintain_order).agg(
        pl.col("v").sum().alias("s"), pl.len()).collect()
    a = sorted(zip(out["c"].to_list(), out["s"].to_list(), out["len"].to_list()), key=str)
    b = sorted(zip(ref["c"].to_list(), ref["s"].to_list(), ref["len"].to_list()), key=str)
    assert a == b
    if maintain_order:
        assert out["c"].to_list() == ref["c"].to_list()
    # the output keys stay codes over the dictionary until exported
    arr = out["c"].to_arrow()
    assert pa.types.is_dictionary(arr.type) and arr.to_pylist() == out["c"].to_list()


def test_categorical_key_also_used_elsewhere(gpu):
    """A Categorical key that the predicate or an aggregation also reads
    keeps its strings for those (and still groups correctly)."""
    rng = np.random.default_rng(2)
    n = 200_000
    strs = np.array(["AAPL", "MSFT", "GOOG", "AMZN"], dtype=object)[rng.integers(0, 4, n)].tolist()
    v = rng.uniform(0, 1, n)
    df = _cat_frame(strs, v)
    out = df.lazy().filter(pl.col("c") != "MSFT").group_by("c").agg(pl.col("v").sum().alias("s")).collect()
    got = dict(zip(out["c"].to_list(), out["s"].to_list()))
    sa = np.array(strs, dtype=object)
    assert set(got) == {"AAPL", "GOOG", "AMZN"}
    for key, val in got.items():
        assert val == math.fsum(v[sa == key])
    # the column's strings are gathered for other uses (a filter of the frame)
    f = df.filter(pl.col("c") == "GOOG")
    assert f["c"].to_list() == [s for s in strs if s == "GOOG"]


def _string_frame(keys_list, vals):
    return pl.DataFrame([pl.Series("s", keys_list, pl.String), pl.Series.from_numpy("v", vals)])


@pytest.mark.parametrize("case", ["short", "long_selected", "long_unselected", "empty_strings"])
def test_fused_string_key(gpu, case):
    """One null-free String key of a large input: its exact short-string
    codes are formed inside the fused kernel from the offsets and data words
    (no code column); a selected string longer than 7 bytes sends the
    query to the hashed long-string path (key_pack 0), one in an unselected
    row does not.  Same groups and exact sums as Python on the strings."""
    rng = np.random.default_rng(len(case))
    n = 1_200_001
    pool = np.array([f"S{i}" for i in range(150)] + ["", "abcdefg"], dtype=object)
    if case == "empty_strings":
        pool[:20] = ""
    idx = rng.integers(0, len(pool), n)
    strs = pool[idx].astype(object)
    v = rng.uniform(0, 100, n)
    if case == "long_selected":
        strs[n // 3] = "a-much-longer-symbol"
        v[n // 3] = 99.0
    if case == "long_unselected":
        strs[n // 3] = "a-much-longer-symbol"
        v[n // 3] = 1.0
    df = _string_frame(strs.tolist(), v)
    info = {}
    out = df.lazy().filter(pl.col("v") > 50.0).group_by("s").agg(pl.col("v").sum().alias("sv"), pl.len()).collect(
        info=info)
    assert info["key_pack"] == (0 if case == "long_selected" else 1), info
    sel = v > 50.0
    want = {}
    for sv, x in zip(strs[sel].tolist(), v[sel].tolist()):
        want.setdefault(sv, []).append(x)
    got = dict(zip(out["s"].to_list(), zip(out["sv"].to_list(), out["len"].to_list())))
    assert set(got) == set(want)
    for key, xs in want.items():
        assert got[key] == (math.fsum(xs), len(xs)), key



_NONNEG_PREDS = {  # name -> (expr, the oracle's program over column 0 = close)
    "gt0": (lambda: pl.col("close") > 0.0, [(1, 0, 0), (2, 0, 0.0), (24, 0, 0)]),
    "ge0": (lambda: pl.col("close") >= 0.0, [(1, 0, 0), (2, 0, 0.0), (25, 0, 0)]),
    "gt250": (lambda: pl.col("close") > 250.0, [(1, 0, 0), (2, 0, 250.0), (24, 0, 0)]),
    "eq0": (lambda: pl.col("close") == 0.0, [(1, 0, 0), (2, 0, 0.0), (20, 0, 0)]),
    "eq": (lambda: pl.col("close") == 3.5, [(1, 0, 0), (2, 0, 3.5), (20, 0, 0)]),
    "gtneg": (lambda: pl.col("close") > -1.0, [(1, 0, 0), (2, 0, -1.0), (24, 0, 0)]),
}


@pytest.mark.parametrize("pname", list(_NONNEG_PREDS))
@pytest.mark.parametrize("keys", ["int64", "sym_day", "runs", "int64_nulls"])
@pytest.mark.parametrize("order", ["close_last", "close_first"])
def test_nonneg_predicate_column_sum(gpu, plgpu_option, pname, keys, order):
    """Four sums whose last column is the fused predicate's and keeps no
    value below a literal >= 0 (the headline's close.sum() under
    close > 250) run the variant whose last limbs carry no sign
    (gb_fast_kernel VAR 5, option sum_pos).  Checked bit-exact against the
    oracle (or_group_by_agg, SUM_EXACT) with the option on and off, on data
    with negatives, zeros, -0.0, NaN, +inf and exact hits of the literal;
    keys: an Int64 key, (Int64, Int32) packed in the kernel, and a sorted
    key (the RUNS layout), and an Int64 key over value columns with ~2 %
    nulls (the NULLS variant; a null close drops its row, so VAR 5 still
    holds).  close_first puts the predicate's column in the
    first acc: var_x_nonneg's pred_acc is then 0 and the signed kernel runs
    (gtneg: a negative literal, never the unsigned variant)."""
    rng = np.random.default_rng(len(pname) + len(keys) + len(order))
    n = 400_003
    sym = rng.integers(0, 100, n).astype(np.int64)
    if keys == "runs":
        sym = np.sort(sym)
    day = (np.arange(n) // 5000).astype(np.int32)
    names = ["open", "high", "low", "close"] if order == "close_last" else ["close", "open", "high", "low"]
    cols = {c: rng.uniform(-500, 500, n) for c in names}
    x = cols["close"]
    x[rng.random(n) < 0.05] = 0.0
    x[rng.random(n) < 0.05] = -0.0
    x[rng.random(n) < 0.02] = 3.5
    x[rng.integers(0, n, 3)] = np.nan
    x[rng.integers(0, n, 2)] = np.inf
    x[rng.integers(0, n, 2)] = -np.inf
    valid = {c: (rng.random(n) > 0.02 if keys == "int64_nulls" else None) for c in names}
    df = pl.DataFrame({"sym": pl.Series.from_numpy("sym", sym), "day": pl.Series.from_numpy("day", day),
                       **{c: pl.Series.from_numpy(c, v, valid[c]) for c, v in cols.items()}})
    mk, prog = _NONNEG_PREDS[pname]
    by = ["sym", "day"] if keys == "sym_day" else ["sym"]
    hk = [(sym, None)] + ([(day, None)] if keys == "sym_day" else [])
    hc = [O.HostCol(cols[c], valid[c]) for c in ["close"] + [c for c in names if c != "close"]]
    oidx = {c: i for i, c in enumerate(["close"] + [c for c in names if c != "close"])}
    okeys, oouts = O.group_by_agg_multi(hk, hc, prog, [("sum", oidx[c]) for c in names], n)
    want = {tuple(int(k[0][i]) for k in okeys): [o[0][i] for o in oouts] for i in range(len(okeys[0][0]))}
    for on in (1, 0):
        plgpu_option("sum_pos", on)
        info = {}
        out = df.lazy().filter(mk()).group_by(*by).agg(*[pl.col(c).sum() for c in names]).collect(info=info)
        assert out.height == len(want), (pname, on)
        if keys != "sym_day":  # (8,001 (sym, day) groups over 4e5 rows: the plan's choice)
            assert info["path"] == 2, info
        kc = [out[k].to_numpy() for k in by]
        vc = [out[c].to_numpy() for c in names]
        for i in range(out.height):
            w = want[tuple(int(k[i]) for k in kc)]
            got = np.array([v[i] for v in vc])
            assert np.array_equal(got.view(np.int64), np.array(w).view(np.int64)), (pname, keys, order, on, i)
