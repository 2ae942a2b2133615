"""Many groups (round 5): the partitioned group-by over 2^B hash partitions,
one scatter pass (B <= 8) or two (level 1 over the input, level 2 within
each level-1 partition), exact against the oracle: keys, first-occurrence
order under maintain_order, and every aggregate bit for bit.

* 1e6 and 1e7 random groups, 1-4 aggregated columns, with and without the
  predicate and maintain_order (the sizes the plan sends to two passes);
* the partition bits and pass count forced (options gb_path = 3, part_bits,
  part_levels) over the same frame, every form bitwise equal to the oracle;
* program predicates and 4-byte key / value columns (the scatter's generic
  loads), Int64 extremes as keys.

Reference: polars-stream/src/nodes/group_by.rs:75 flush_evictions, :85
add_pre_agg (hash-partitioned pre-aggregation), polars-utils/src/
hashing.rs:72 HashPartitioner.
"""

import numpy as np
import pytest

import polaroid_amd as pl
from oracle import oracle as O

pytestmark = pytest.mark.gpu

I64_MIN = np.iinfo(np.int64).min
I64_MAX = np.iinfo(np.int64).max


def _bits(a):
    return np.asarray(a, dtype=np.float64).view(np.uint64)


def _ohlc(rng, n):
    close = rng.uniform(10.0, 500.0, n)
    return {
        "open": close * rng.uniform(0.99, 1.01, n),
        "high": close * rng.uniform(1.0, 1.02, n),
        "low": close * rng.uniform(0.98, 1.0, n),
        "close": close,
    }


# (1, col, 0) load column, (2, 0, x) f64 literal, (24, 0, 0) greater-than
def _gt_prog(ci, x):
    return [(1, ci, 0), (2, 0, x), (24, 0, 0)]


def _expected(cols, key, aggs, prog_names, prog):
    names = list(dict.fromkeys([c for _, c in aggs] + list(prog_names)))
    hc = [O.HostCol(cols[c], None) for c in names]
    p = prog(names) if prog else None
    return O.group_by_agg(O.HostCol(key, None), hc, p, [(kind, names.index(c)) for kind, c in aggs], key.shape[0],
                          O.SUM_EXACT)


def _gpu(cols, key, aggs, pred, maintain):
    data = {"k": pl.Series.from_numpy("k", key)}
    for c, v in cols.items():
        data[c] = pl.Series.from_numpy(c, v)
    lf = pl.DataFrame(data).lazy()
    if pred is not None:
        lf = lf.filter(pred)
    info = {}
    out = lf.group_by("k", maintain_order=maintain).agg(
        *[getattr(pl.col(c), kind)().alias(f"{kind}_{c}") for kind, c in aggs]).collect(info=info)
    return out, info


def _compare(out, exp, aggs, maintain):
    okeys, okvalid, oouts = exp
    gk = out["k"].to_numpy().astype(np.int64)
    assert gk.shape[0] == okeys.shape[0]
    assert out["k"].validity_numpy().all() and okvalid.all()
    if maintain:
        go = oo = slice(None)
    else:
        go, oo = np.argsort(gk, kind="stable"), np.argsort(okeys, kind="stable")
    assert np.array_equal(gk[go], okeys[oo])
    for (kind, c), (ov, ovalid) in zip(aggs, oouts):
        s = out[f"{kind}_{c}"]
        gv, gvalid = s.to_numpy()[go], s.validity_numpy()[go]
        ov, ovalid = ov[oo], ovalid[oo]
        assert np.array_equal(gvalid, ovalid), (kind, c)
        if ov.dtype == np.float64:
            assert np.array_equal(_bits(gv)[ovalid], _bits(ov)[ovalid]), (kind, c)
        else:
            assert np.array_equal(gv[ovalid].astype(np.int64), ov[ovalid].astype(np.int64)), (kind, c)


MANY = [
    # groups, aggregated columns, fused predicate, maintain_order
    (1_000_000, [("sum", "close")], False, True),
    (1_000_000, [("sum", "open"), ("sum", "high"), ("sum", "low"), ("sum", "close")], True, False),
    (1_000_000, [("sum", "close"), ("min", "low"), ("max", "high"), ("len", "close")], True, True),
    (10_000_000, [("sum", "open"), ("mean", "close")], True, True),
    (10_000_000, [("sum", "open"), ("sum", "high"), ("sum", "low"), ("sum", "close")], True, False),
]


@pytest.mark.slow
@pytest.mark.parametrize("case", range(len(MANY)))
def test_many_groups_exact(gpu, case):
    groups, aggs, pred, maintain = MANY[case]
    rng = np.random.default_rng(100 + case)
    n = 3 * groups
    # random keys: ~0.95 of the key space occurs at 3 rows per key
    key = rng.integers(0, groups, n).astype(np.int64) * 7919 - 3 * groups
    cols = _ohlc(rng, n)
    exp = _expected(cols, key, aggs, ["close"] if pred else [],
                    (lambda names: _gt_prog(names.index("close"), 250.0)) if pred else None)
    out, info = _gpu(cols, key, aggs, (pl.col("close") > 250.0) if pred else None, maintain)
    assert info["path"] == 3, info
    assert info["part_layout"] >> 8 == 2, info   # two scatter passes
    _compare(out, exp, aggs, maintain)


FORCED = [(0, 1), (1, 1), (6, 1), (8, 1), (4, 2), (9, 2), (12, 2), (16, 2)]


@pytest.mark.parametrize("card", [300, 20_000, 200_000])
@pytest.mark.parametrize("maintain", [False, True])
def test_partition_bits_and_passes_forced(gpu, card, maintain, plgpu_option):
    """The same frame through every forced partition layout (bits, passes),
    with sum-only and mixed aggregations, each bitwise equal to the oracle."""
    rng = np.random.default_rng(card + maintain)
    n = 1_500_001
    key = rng.integers(0, card, n).astype(np.int64) * 1_000_003 - 7
    key[rng.random(n) < 0.001] = I64_MIN
    key[rng.random(n) < 0.001] = I64_MAX
    cols = _ohlc(rng, n)
    cols["vol"] = rng.integers(-10**12, 10**12, n).astype(np.int64)
    cols["close"][rng.random(n) < 0.0005] = np.nan
    cols["open"][rng.random(n) < 0.0005] = -np.inf
    agg_sets = [
        [("sum", "open"), ("sum", "high"), ("mean", "close")],
        [("sum", "close"), ("min", "low"), ("max", "vol"), ("sum", "vol"), ("count", "high"), ("len", "open")],
    ]
    for aggs in agg_sets:
        exp = _expected(cols, key, aggs, ["close"], lambda names: _gt_prog(names.index("close"), 250.0))
        for bits, levels in FORCED:
            plgpu_option("gb_path", 3)
            plgpu_option("part_bits", bits)
            plgpu_option("part_levels", levels)
            out, info = _gpu(cols, key, aggs, pl.col("close") > 250.0, maintain)
            assert info["path"] == 3, (bits, levels, info)
            got_bits, got_levels = info["part_layout"] & 0xFF, info["part_layout"] >> 8
            assert got_bits >= bits and got_levels == (2 if (levels == 2 or got_bits > 8) and got_bits >= 2 else 1), \
                (bits, levels, info)
            _compare(out, exp, aggs, maintain)


@pytest.mark.parametrize("levels", [1, 2])
def test_partitioned_program_predicate_and_narrow_columns(gpu, levels, plgpu_option):
    """A program predicate (evaluated per row in the count and scatter
    passes) and 4-byte key / value columns (the scatter's generic loads)."""
    rng = np.random.default_rng(7 + levels)
    n = 1_200_003
    key = rng.integers(-40_000, 40_000, n).astype(np.int32)
    cols = {"a": rng.standard_normal(n) * 100, "b": rng.integers(-50, 50, n).astype(np.int32),
            "d": rng.uniform(-5, 5, n)}
    aggs = [("sum", "a"), ("max", "b"), ("sum", "b"), ("min", "d"), ("len", "a")]
    # ((a * 2 + b) > d): the oracle's program over names [a, b, d]
    prog = [(1, 0, 0), (3, 0, 2), (12, 0, 0), (1, 1, 0), (10, 0, 0), (1, 2, 0), (24, 0, 0)]
    names = ["a", "b", "d"]
    hc = [O.HostCol(cols[c], None) for c in names]
    exp = O.group_by_agg(O.HostCol(key, None), hc, prog, [(kind, names.index(c)) for kind, c in aggs], n,
                         O.SUM_EXACT)
    plgpu_option("gb_path", 3)
    plgpu_option("part_bits", 10 if levels == 2 else 7)
    plgpu_option("part_levels", levels)
    for maintain in (False, True):
        out, info = _gpu(cols, key, aggs, (pl.col("a") * 2 + pl.col("b")) > pl.col("d"), maintain)
        assert info["path"] == 3 and info["part_layout"] >> 8 == levels, info
        assert out["k"].dtype == pl.Int32
        okeys, okvalid, oouts = exp
        _compare(out, (okeys.astype(np.int64), okvalid, oouts), aggs, maintain)


@pytest.mark.parametrize("compact", [1, 0])
@pytest.mark.parametrize("nullable", [False, True])
def test_compact_regions(gpu, compact, nullable, plgpu_option):
    """Compact regions (option part_compact): each partition's workgroup
    writes its groups densely from its region's first slot and the finalize
    reads only those prefixes plus the two special groups (the null key and
    the key equal to the table's empty marker, Int64 extremes here).  Bitwise
    equal to the oracle with the option on and off, with NaN / inf values,
    null keys and null values (the NULLS partition kernel)."""
    rng = np.random.default_rng(31 + compact + 2 * nullable)
    n = 2_000_003
    key = rng.integers(0, 400_000, n).astype(np.int64) * 104_729 + 11
    key[rng.random(n) < 0.001] = I64_MIN
    key[rng.random(n) < 0.001] = I64_MAX
    cols = _ohlc(rng, n)
    cols["close"][rng.random(n) < 0.0005] = np.nan
    cols["open"][rng.random(n) < 0.0005] = np.inf
    kvalid = (rng.random(n) > 0.01) if nullable else None
    vvalid = {c: ((rng.random(n) > 0.02) if nullable and c != "close" else None) for c in cols}
    aggs = [("sum", "open"), ("sum", "high"), ("sum", "low"), ("sum", "close")]
    plgpu_option("part_compact", compact)
    plgpu_option("gb_path", 3)
    data = {"k": pl.Series.from_numpy("k", key, kvalid)}
    for c, v in cols.items():
        data[c] = pl.Series.from_numpy(c, v, vvalid[c])
    info = {}
    out = pl.DataFrame(data).lazy().filter(pl.col("close") > 100.0).group_by("k").agg(
        *[pl.col(c).sum().alias(f"sum_{c}") for _, c in aggs]).collect(info=info)
    assert info["path"] == 3, info
    names = [c for _, c in aggs]
    hc = [O.HostCol(cols[c], vvalid[c]) for c in names]
    okeys, okvalid, oouts = O.group_by_agg(O.HostCol(key, kvalid), hc, _gt_prog(names.index("close"), 100.0),
                                           [(kind, names.index(c)) for kind, c in aggs], n, O.SUM_EXACT)
    gk, gkv = out["k"].to_numpy().astype(np.int64), out["k"].validity_numpy()
    assert gk.shape[0] == okeys.shape[0]
    assert gkv.sum() == okvalid.sum() and (~gkv).sum() == (~okvalid).sum() <= 1
    tg = [("n", 0) if not v else ("k", int(k_)) for k_, v in zip(gk, gkv)]
    to = [("n", 0) if not v else ("k", int(k_)) for k_, v in zip(okeys, okvalid)]
    pos = {t: i for i, t in enumerate(to)}
    oo = np.array([pos[t] for t in tg], dtype=np.int64)
    for (kind, c), (ov, ovalid) in zip(aggs, oouts):
        s = out[f"{kind}_{c}"]
        assert np.array_equal(s.validity_numpy(), ovalid[oo]), c
        assert np.array_equal(_bits(s.to_numpy()), _bits(ov[oo])), c


def test_compact_regions_rerun_on_stale_plan(gpu):
    """A plan whose group estimate is stale (the cached statistics of columns
    rewritten in place, six times the groups) sizes partitions too small:
    rows miss their partition's LDS table, the compact run is redone on the
    probed regions, and the result stays exact."""
    import torch

    n = 3_000_001
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    k = torch.randint(0, 200_000, (n,), device="cuda", generator=g, dtype=torch.int64)
    x = torch.rand(n, device="cuda", generator=g, dtype=torch.float64) * 100.0
    df = pl.DataFrame([pl.Series.from_torch("k", k), pl.Series.from_torch("x", x)])
    q = df.lazy().group_by("k").agg(pl.col("x").sum().alias("s"))
    info = {}
    q.collect(info=info)
    k.copy_(torch.randint(0, 1_200_000, (n,), device="cuda", generator=g, dtype=torch.int64))
    torch.cuda.synchronize()
    info = {}
    out = q.collect(info=info)
    kh, xh = k.cpu().numpy(), x.cpu().numpy()
    okeys, _, oouts = O.group_by_agg(O.HostCol(kh, None), [O.HostCol(xh, None)], None, [("sum", 0)], n, O.SUM_EXACT)
    go, oo = np.argsort(out["k"].to_numpy()), np.argsort(okeys)
    assert np.array_equal(out["k"].to_numpy()[go], okeys[oo])
    assert np.array_equal(_bits(out["s"].to_numpy()[go]), _bits(oouts[0][0][oo]))


@pytest.mark.parametrize("compact", [1, 0])
def test_compact_regions_sorted_keys(gpu, compact, plgpu_option):
    """Sorted (clustered) keys take the partition kernel's register
    accumulators (part_racc) before the compact flush: bitwise equal to the
    oracle with compact regions on and off."""
    rng = np.random.default_rng(77 + compact)
    n = 2_000_003
    key = np.sort(rng.integers(0, 300_000, n)).astype(np.int64) * 13 - 5
    cols = _ohlc(rng, n)
    aggs = [("sum", "open"), ("sum", "close")]
    plgpu_option("part_compact", compact)
    plgpu_option("gb_path", 3)
    out, info = _gpu(cols, key, aggs, pl.col("close") > 100.0, False)
    assert info["path"] == 3, info
    exp = _expected(cols, key, aggs, ["close"], lambda names: _gt_prog(names.index("close"), 100.0))
    _compare(out, exp, aggs, False)


@pytest.mark.parametrize("extremes", ["none", "max", "max_and_min"])
@pytest.mark.parametrize("sentinel", [1, 0])
def test_null_key_sentinel(gpu, plgpu_option, extremes, sentinel):
    """A sum-only partitioned run over a nullable Int64 key writes each null
    key as a value outside the non-null keys' range (above the maximum, else
    below the minimum, never INT64_MIN, which has a special slot of its own)
    instead of carrying a null-bits column (option part_null_sentinel).  Keys
    holding INT64_MAX (sentinel below the range) or INT64_MAX and INT64_MIN + 1
    (no sentinel: the null-bits column) with the option on and off, bitwise
    equal to the oracle, INT64_MIN keys and the null group included."""
    rng = np.random.default_rng(3 + sentinel + len(extremes))
    n = 1_500_007
    key = rng.integers(-200_000, 200_000, n).astype(np.int64)
    if extremes in ("max", "max_and_min"):
        key[rng.random(n) < 0.001] = I64_MAX
    if extremes == "max_and_min":
        key[rng.random(n) < 0.001] = I64_MIN + 1
    key[rng.random(n) < 0.001] = I64_MIN
    kvalid = rng.random(n) > 0.02
    cols = _ohlc(rng, n)
    vvalid = rng.random(n) > 0.01
    aggs = [("sum", "open"), ("sum", "close")]
    plgpu_option("part_null_sentinel", sentinel)
    plgpu_option("gb_path", 3)
    data = {"k": pl.Series.from_numpy("k", key, kvalid), "open": pl.Series.from_numpy("open", cols["open"], vvalid),
            "close": pl.Series.from_numpy("close", cols["close"])}
    info = {}
    out = pl.DataFrame(data).lazy().filter(pl.col("close") > 100.0).group_by("k").agg(
        *[pl.col(c).sum().alias(f"sum_{c}") for _, c in aggs]).collect(info=info)
    assert info["path"] == 3, info
    names = ["open", "close"]
    okeys, okvalid, oouts = O.group_by_agg(O.HostCol(key, kvalid), [O.HostCol(cols["open"], vvalid),
                                                                     O.HostCol(cols["close"])],
                                           _gt_prog(1, 100.0), [("sum", 0), ("sum", 1)], n, O.SUM_EXACT)
    gk, gkv = out["k"].to_numpy().astype(np.int64), out["k"].validity_numpy()
    tg = [("n", 0) if not v else ("k", int(k_)) for k_, v in zip(gk, gkv)]
    to = [("n", 0) if not v else ("k", int(k_)) for k_, v in zip(okeys, okvalid)]
    assert len(tg) == len(to) and set(tg) == set(to)
    pos = {t: i for i, t in enumerate(to)}
    oo = np.array([pos[t] for t in tg], dtype=np.int64)
    for (kind, c), (ov, ovalid) in zip(aggs, oouts):
        s = out[f"{kind}_{c}"]
        assert np.array_equal(_bits(s.to_numpy()), _bits(ov[oo])), c
