"""GPU parity of the multi-key group-by (plgpu_group_by_agg_multi) against
the oracle's row-encoding restatement (oracle.group_by_agg_multi), which
follows polars-core/src/frame/group_by/mod.rs:91 (keys row-encoded by
chunked_array/ops/row_encode.rs:11, groups = distinct encoded tuples).

Bar: key tuples, group order (maintain_order) and every aggregation
bit-exact; f64 sums are the correctly rounded exact sums on both sides.
"""

import math
import os

import numpy as np
import pytest

import polaroid_amd as pl
from conftest import load_golden, unhex
from oracle import oracle as O
from test_gpu_parity import PREDICATES, _bits, _gpu_df, _host_cols, _rand_frame

pytestmark = pytest.mark.gpu


def _canon(v, m):
    """Key tuple element in comparable form (None / TotalOrd f64)."""
    if not m:
        return None
    if isinstance(v, float):
        return "nan" if math.isnan(v) else v + 0.0
    return v


def _check(keys, cols, aggs, maintain_order, pred=None, info=None):
    """keys: {name: (values, valid)}; cols: {name: (values, valid)}."""
    n = next(iter(keys.values()))[0].shape[0]
    pred_expr, pred_names, pred_prog = (None, [], None) if pred is None else (PREDICATES[pred][0](),
                                                                           PREDICATES[pred][1],
                                                                           PREDICATES[pred][2])
    names = list(dict.fromkeys(pred_names + [c for _, c in aggs]))
    data = dict(keys)
    data.update({k: cols[k] for k in names})
    lf = _gpu_df(data).lazy()
    if pred_expr is not None:
        lf = lf.filter(pred_expr)
    exprs = [getattr(pl.col(c), kind)().alias(f"{kind}_{c}") for kind, c in aggs]
    res = {}
    out = lf.group_by(*keys, maintain_order=maintain_order).agg(*exprs).collect(info=res)
    if info is not None:
        info.update(res)
    okeys, oouts = O.group_by_agg_multi(list(keys.values()), _host_cols(cols, names), pred_prog,
                                        [(kind, names.index(c)) for kind, c in aggs], n)
    g = len(okeys[0][0])
    assert out.height == g
    assert out.columns[:len(keys)] == list(keys)
    gcols = [(out[k].to_numpy().tolist(), out[k].validity_numpy().tolist()) for k in keys]
    gt = [tuple(_canon(gcols[j][0][i], gcols[j][1][i]) for j in range(len(keys))) for i in range(g)]
    ocols = [(v.tolist(), m.tolist()) for v, m in okeys]
    ot = [tuple(_canon(ocols[j][0][i], ocols[j][1][i]) for j in range(len(keys))) for i in range(g)]
    assert len(set(gt)) == g  # distinct tuples
    if maintain_order:
        go = np.arange(g)
        oo = np.arange(g)
        assert gt == ot
    else:
        pos = {t: i for i, t in enumerate(ot)}
        assert set(gt) == set(ot)
        go = np.arange(g)
        oo = np.array([pos[t] for t in gt], dtype=np.int64)
    # key values are the group's first selected row (bitwise for f64 keys)
    for j, k in enumerate(keys):
        if keys[k][0].dtype == np.float64:
            gv, ov = out[k].to_numpy(), okeys[j][0]
            m = okeys[j][1][oo]
            assert np.array_equal(_bits(gv[go])[m], _bits(ov[oo])[m]), k
    for (kind, c), (ov, ovalid) in zip(aggs, oouts):
        s = out[f"{kind}_{c}"]
        gv, gvalid = s.to_numpy()[go], s.validity_numpy()[go]
        ov, ovalid = ov[oo], ovalid[oo]
        assert np.array_equal(gvalid, ovalid), (kind, c)
        if ov.dtype == np.float64:
            nan_g, nan_o = np.isnan(gv[ovalid]), np.isnan(ov[ovalid])
            assert np.array_equal(nan_g, nan_o), (kind, c)
            assert np.array_equal(_bits(gv[ovalid])[~nan_g], _bits(ov[ovalid])[~nan_o]), (kind, c)
        else:
            assert np.array_equal(gv[ovalid].astype(np.int64), ov[ovalid].astype(np.int64)), (kind, c)
    return out


AGGS = [("sum", "a"), ("mean", "d"), ("min", "b"), ("max", "a"), ("count", "d"), ("len", "b")]


@pytest.mark.parametrize("card", [1, 5, 300, 20000])
@pytest.mark.parametrize("maintain_order", [False, True])
@pytest.mark.parametrize("pack", [True, False])
def test_two_int_keys_vs_oracle(gpu, card, maintain_order, pack, plgpu_option):
    """Integer keys go through the exact packed Int64 key; PLGPU_NO_PACK
    forces the hash + verify path on the same data."""
    if not pack:
        plgpu_option("no_pack", 1)
    rng = np.random.default_rng(card + 7)
    n = 150_000
    cols = _rand_frame(rng, n)
    k1 = rng.integers(0, card, n).astype(np.int64)
    k2 = rng.integers(-3, 3, n).astype(np.int32)
    k1v = rng.random(n) > 0.05
    _check({"k1": (k1, k1v), "k2": (k2, None)}, cols, AGGS, maintain_order)


@pytest.mark.parametrize("pred", [None, "simple_f64", "program"])
def test_mixed_dtype_keys_with_predicate(gpu, pred):
    """Int64 / UInt32 / Float64 (-0.0, NaN) / Boolean keys, nullable."""
    rng = np.random.default_rng(21)
    n = 100_003
    cols = _rand_frame(rng, n)
    ki = rng.integers(-(1 << 62), 1 << 62, 40)[rng.integers(0, 40, n)].astype(np.int64)
    ku = rng.integers(0, 1 << 32, 7, dtype=np.uint64)[rng.integers(0, 7, n)].astype(np.uint32)
    kf = np.array([0.0, -0.0, np.nan, -np.nan, 1.5, np.inf])[rng.integers(0, 6, n)]
    kb = rng.random(n) < 0.3
    keys = {"ki": (ki, rng.random(n) > 0.1), "ku": (ku, None), "kf": (kf, rng.random(n) > 0.05),
            "kb": (kb, rng.random(n) > 0.2)}
    _check(keys, cols, [("sum", "a"), ("len", "b"), ("min", "d")], True, pred)


@pytest.mark.parametrize("nkeys", [1, 3, 8])
def test_key_count_and_single_non_int_key(gpu, nkeys):
    """One Float64 key (goes through the multi-key path), and 3 / 8 keys."""
    rng = np.random.default_rng(nkeys)
    n = 50_000
    cols = _rand_frame(rng, n)
    keys = {}
    for i in range(nkeys):
        if i % 2:
            keys[f"k{i}"] = (rng.integers(0, 3, n).astype(np.int64), rng.random(n) > 0.1)
        else:
            keys[f"k{i}"] = (rng.choice(np.array([-0.0, 0.0, 2.5, np.nan]), n), None)
    _check(keys, cols, [("sum", "d"), ("len", "a")], nkeys != 3)


@pytest.mark.parametrize("pack", [True, False])
def test_many_groups_and_special_hashes(gpu, pack, plgpu_option):
    """~1e6 distinct tuples over 2e6 rows (global-table path)."""
    if not pack:
        plgpu_option("no_pack", 1)
    rng = np.random.default_rng(99)
    n = 2_000_000
    cols = {"a": (rng.standard_normal(n), None), "b": (rng.integers(-9, 9, n).astype(np.int64), None)}
    k1 = rng.integers(0, 1000, n).astype(np.int64)
    k2 = rng.integers(0, 1000, n).astype(np.int64)
    info = {}
    _check({"k1": (k1, None), "k2": (k2, None)}, cols, [("sum", "a"), ("max", "b"), ("len", "a")], False,
           info=info)
    assert info["groups"] > 600_000


def test_collision_triggers_reseed(gpu, plgpu_option):
    """A forced 3-bit first hash merges distinct tuples; the verify pass
    must catch it and the re-seeded run must be exact."""
    plgpu_option("mk_collide", 1)
    plgpu_option("no_pack", 1)  # integer keys would be packed exactly
    rng = np.random.default_rng(4)
    n = 30_000
    cols = _rand_frame(rng, n)
    k1 = rng.integers(0, 50, n).astype(np.int64)
    k2 = rng.integers(0, 3, n).astype(np.int64)
    info = {}
    _check({"k1": (k1, None), "k2": (k2, None)}, cols, AGGS, True, info=info)
    assert info["reruns"] >= 1


def test_empty_all_filtered_and_errors(gpu):
    df = pl.DataFrame({"a": pl.Series("a", [], pl.Int64), "b": pl.Series("b", [], pl.Int64),
                       "v": pl.Series("v", [], pl.Float64)})
    out = df.group_by("a", "b").agg(pl.col("v").sum())
    assert out.height == 0 and out.columns == ["a", "b", "v"]
    df = pl.DataFrame({"a": [1, 2, 3], "b": [1, 1, 1], "v": [1.0, 2.0, 3.0]})
    out = df.lazy().filter(pl.col("v") > 10.0).group_by("a", "b").agg(pl.col("v").sum()).collect()
    assert out.height == 0
    with pytest.raises(pl.DuplicateError):
        df.group_by("a", "a")
    with pytest.raises(pl.InvalidOperationError):
        df.group_by(*[f"k{i}" for i in range(9)])


def test_group_by_multi_golden(gpu):
    for case in load_golden("group_by_multi_cases.json")["cases"]:
        data = {}
        for name, spec in list(case["keys"].items()) + list(case["cols"].items()):
            if name in data:
                continue
            vals = unhex(spec["values"]) if spec["dtype"] == "f64" else spec["values"]
            data[name] = pl.Series(name, vals, pl.Float64 if spec["dtype"] == "f64" else pl.Int64)
        df = pl.DataFrame(data)
        exprs = [getattr(pl.col(a[1]), a[0])().alias(a[2]) for a in case["aggs"]]
        out = df.group_by(*case["keys"], maintain_order=case["maintain_order"]).agg(*exprs)
        order = list(range(out.height))
        if "sort_by" in case:
            sk = out[case["sort_by"]].to_list()
            order = sorted(order, key=lambda i: sk[i])
        for nm, exp in case["expected"].items():
            got = out[nm].to_list()
            got = [got[i] for i in order]
            exp = unhex(exp)
            for g, e in zip(got, exp):
                if e is None or g is None:
                    assert g is None and e is None, (case["name"], nm, got, exp)
                elif isinstance(e, float) and math.isnan(e):
                    assert math.isnan(g), (case["name"], nm, got, exp)
                else:
                    assert g == e, (case["name"], nm, got, exp)
        assert len(got) == len(exp)


def test_packed_key_ranges_extremes(gpu):
    """Packing at the edges: full-range Int32 / UInt32 keys, negative Int64
    ranges, an all-null key, Boolean keys; and a pair whose ranges need more
    than 63 bits (hash path)."""
    rng = np.random.default_rng(17)
    n = 60_000
    cols = _rand_frame(rng, n)
    i32 = rng.choice(np.array([-2**31, 2**31 - 1, 0, -1], dtype=np.int32), n)
    u32 = rng.choice(np.array([0, 2**32 - 1, 7], dtype=np.uint32), n)
    neg = rng.integers(-10**15, -10**15 + 50, n).astype(np.int64)
    alln = (np.zeros(n, np.int64), np.zeros(n, bool))
    b = rng.random(n) < 0.5
    _check({"i32": (i32, rng.random(n) > 0.1), "u32": (u32, None), "neg": (neg, None), "z": alln,
            "bk": (b, rng.random(n) > 0.3)}, cols, [("sum", "a"), ("len", "b")], True)
    wide = rng.choice(np.array([np.iinfo(np.int64).min, np.iinfo(np.int64).max, 0]), n)
    _check({"w1": (wide, None), "w2": (wide[::-1].copy(), None)}, cols, [("sum", "d"), ("len", "a")], False)


@pytest.mark.parametrize("case", ["in_sample_range", "outlier_row", "null_in_unsampled_row", "narrow_dtypes"])
def test_sampled_packing_plan(gpu, case):
    """Above 2^20 rows the packing plan comes from a sample of the key
    columns (widened by the sampled span, a null code reserved per key); a
    row outside it (an outlier the sample missed) sends the group-by to the
    exact range pass and a repack, with the same result."""
    rng = np.random.default_rng(len(case))
    n = 1_500_003
    k1 = rng.integers(0, 1000, n).astype(np.int64) * 3 - 500
    k2 = rng.integers(0, 50, n).astype(np.int32)
    v1 = None
    if case == "outlier_row":
        k1[n // 2 + 7] = 1 << 40  # far outside any widened sampled range
    if case == "null_in_unsampled_row":
        v1 = np.ones(n, bool)
        v1[n // 2 + 7] = False
    if case == "narrow_dtypes":
        k1 = (k1 % 120).astype(np.int8)
        k2 = k2.astype(np.uint16)
    cols = _rand_frame(rng, n)
    _check({"k1": (k1, v1), "k2": (k2, None)}, cols, [("sum", "a"), ("len", "b"), ("max", "d")], False)


def test_hashed_tuples_between_one_table_and_a_million(gpu, plgpu_option):
    """~3e5 hashed tuples over 2e6 rows (option no_pack): more groups than
    one LDS table, fewer than the generic path's million, so the hashes go
    through the partitioned path with two aggregated columns; the verify
    pass reads every group's first row (the partition buffers' row ids)."""
    plgpu_option("no_pack", 1)
    rng = np.random.default_rng(123)
    n = 2_000_000
    cols = {"a": (rng.standard_normal(n), None), "b": (rng.integers(-9, 9, n).astype(np.int64), None)}
    k1 = rng.integers(0, 548, n).astype(np.int64)
    k2 = rng.integers(0, 548, n).astype(np.int64)
    info = {}
    _check({"k1": (k1, None), "k2": (k2, None)}, cols, [("sum", "a"), ("max", "b"), ("len", "a")], False,
           info=info)
    assert 200_000 < info["groups"] < 400_000
