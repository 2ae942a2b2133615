"""The group-by at BASELINE's own sizes, checked exactly (no properties in
between):

  metric / configs[1] query at 1e9 rows  filter(close > 250).group_by(symbol)
        .agg(open/high/low/close.sum()) over bench.py's own OHLCV data,
        against an exact reference computed here: every value of that data
        lies in [8, 1024), so it is an integer multiple of 2^-49 below 2^59;
        the multiples are split into 30-bit halves and summed per group with
        int64 scatter-adds (no overflow at 1e9 rows), joined as Python
        integers and rounded once by float(int) -- the correctly rounded sum.
        Every group's every sum must be bit-identical.
  configs[4] per-rank shard  one rank's 1.25e9-row shard of the 1e10-row
        8-GPU job, through the partitioned path exactly as a rank runs it at
        world 8 (plgpu_gb_partial_begin -> plgpu_gb_partial_export into 8
        destinations -> plgpu_gb_merge_sources of each destination's bucket),
        on one GPU: the union of the 8 partitions must equal the single-GPU
        group_by of the same shard bit for bit, each group on one rank.
  multi-key (packed) at 1e9 rows  group_by(symbol, day) whose tuples pack
        into one Int64 code (plgpu_key_ranges / plgpu_key_pack, the plan every
        rank agrees on), partitioned 8 ways, merged, unpacked
        (plgpu_key_unpack): equal to the single-GPU multi-key group_by.
"""
import ctypes as C
import os
import sys

import numpy as np
import pytest

import polaroid_amd as pl
from polaroid_amd import _native as N
from polaroid_amd import distributed as D
from polaroid_amd.frame import DataFrame, Series, _col_array, _gb_lower

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (the bench's own data generator)

THRESHOLD = bench.THRESHOLD
COLS = ("open", "high", "low", "close")
SCALE = 49  # values in [8, 1024) are multiples of 2^-49


def _frame(torch, n, seed):
    sym, cols = bench.make_data(torch, n, 100, seed)
    df = pl.DataFrame([pl.Series.from_torch("symbol", sym)] + [pl.Series.from_torch(k, v) for k, v in cols.items()])
    return df, sym, cols


def _exact_sums(torch, sym, cols):
    """{symbol: (len, [exact sums of open, high, low, close] as floats)}."""
    sel = cols["close"] > THRESHOLD
    gid = ((sym - 1_000_000) // 7919).masked_fill(~sel, 100)  # bin 100: unselected rows
    lens = torch.bincount(gid, minlength=101)[:100].tolist()
    out = {}
    sums = []
    for c in COLS:
        x = cols[c]
        assert bool((x >= 8).all()) and bool((x < 1024).all()), "data outside the exactness range of this check"
        q = (x * 2.0 ** SCALE).to(torch.int64)  # power-of-two scaling: exact
        assert torch.equal(q.to(torch.float64) * 2.0 ** -SCALE, x)
        lo = torch.zeros(101, dtype=torch.int64, device=x.device)
        hi = torch.zeros(101, dtype=torch.int64, device=x.device)
        lo.scatter_add_(0, gid, q & ((1 << 30) - 1))
        hi.scatter_add_(0, gid, q >> 30)
        del q
        sums.append([float((h << 30) + l) * 2.0 ** -SCALE for h, l in zip(hi.tolist()[:100], lo.tolist()[:100])])
    for g in range(100):
        if lens[g]:
            out[g * 7919 + 1_000_000] = (lens[g], [s[g] for s in sums])
    return out


def _bits(v):
    return np.asarray(v, dtype=np.float64).view(np.uint64)


def test_headline_query_1e9_rows_exact(gpu):
    import torch

    n = 1_000_000_000
    df, sym, cols = _frame(torch, n, seed=1234)
    aggs = [pl.col(c).sum() for c in COLS]  # the bench's query, exactly
    info = {}
    out = df.lazy().filter(pl.col("close") > THRESHOLD).group_by("symbol").agg(*aggs).collect(info=info)
    assert info["path"] == 2  # the fused sum-only kernel, as in the bench
    ref = _exact_sums(torch, sym, cols)
    keys = out["symbol"].to_numpy().tolist()
    assert sorted(keys) == sorted(ref)
    for c_i, c in enumerate(COLS):
        got = _bits(out[c].to_numpy())
        want = _bits([ref[k][1][c_i] for k in keys])
        assert np.array_equal(got, want), (c, int((got != want).sum()))
    assert sum(v[0] for v in ref.values()) == info["rows_selected"]
    del df, sym, cols, out
    torch.cuda.empty_cache()


def _partition_world8(g, world=8):
    """One rank's partial stage at `world`, then every destination's merge of
    its bucket (this rank as its only source): the 8 partitions."""
    part = D.GpuPartial(g, world)
    bottoms = part.begin()
    send, counts = part.export()
    rw = part.record_words
    frames = []
    off = 0
    for dest in range(world):
        seg = send[off * rw:(off + counts[dest]) * rw].contiguous()
        off += counts[dest]
        out, _ = D.GpuPartial(g, world).merge(seg, [counts[dest]], [bottoms])
        frames.append(out)
    return frames, counts


def _assert_same_groups(frames, ref, key_cols, val_cols):
    """Union of the partitions == ref, bit for bit, each group once."""
    def table(f):
        ks = [f[k].to_numpy().astype(np.int64) for k in key_cols]
        order = np.lexsort(ks[::-1])
        return [k[order] for k in ks], [f[v].to_numpy()[order] for v in val_cols]

    u = {nm: np.concatenate([f[nm].to_numpy() for f in frames]) for nm in list(key_cols) + list(val_cols)}
    uk = [u[k].astype(np.int64) for k in key_cols]
    order = np.lexsort(uk[::-1])
    rk, rv = table(ref)
    for a, b in zip([k[order] for k in uk], rk):
        assert np.array_equal(a, b)
    for v, b in zip(val_cols, rv):
        a = u[v][order]
        if a.dtype == np.float64:
            assert np.array_equal(_bits(a), _bits(b)), v
        else:
            assert np.array_equal(a, b), v


def test_configs4_rank_shard_1_25e9_world8_routing(gpu):
    import torch

    n = 1_250_000_000
    df, sym, cols = _frame(torch, n, seed=1234 + 5)
    aggs = [pl.col(c).sum().alias(c) for c in COLS] + [pl.col("close").mean().alias("m"), pl.len().alias("len")]
    pred = pl.col("close") > THRESHOLD
    ref = df.lazy().filter(pred).group_by("symbol").agg(*aggs).collect()
    frames, counts = _partition_world8(_gb_lower(df, "symbol", aggs, pred))
    assert sum(counts) == ref.height and sum(1 for c in counts if c) > 1
    _assert_same_groups(frames, ref, ["symbol"], list(COLS) + ["m", "len"])
    del df, sym, cols
    torch.cuda.empty_cache()


def test_multi_key_packed_1e9_world8_routing(gpu):
    import torch

    n = 1_000_000_000
    dev = torch.device("cuda")
    gen = torch.Generator(device=dev)
    gen.manual_seed(77)
    sym = torch.randint(0, 100, (n,), device=dev, generator=gen, dtype=torch.int64) * 7919
    day = (torch.arange(n, device=dev, dtype=torch.int64) * 250) // n + 19000  # time-ordered days
    a = torch.rand(n, device=dev, generator=gen, dtype=torch.float64) * 100
    b = torch.randn(n, device=dev, generator=gen, dtype=torch.float64)
    df = pl.DataFrame([pl.Series.from_torch("sym", sym), pl.Series.from_torch("day", day.to(torch.int32)),
                       pl.Series.from_torch("a", a), pl.Series.from_torch("b", b)])
    aggs = [pl.col("a").sum().alias("sa"), pl.col("b").sum().alias("sb"), pl.col("b").max().alias("mx"),
            pl.len().alias("len")]
    ref = df.group_by("sym", "day").agg(*aggs)
    assert ref.height == 100 * 250
    # the code column every rank would pack with the agreed ranges
    keys = ["sym", "day"]
    kcols = _col_array([df[k] for k in keys])
    r = (C.c_int64 * 6)()
    N.check(N.lib().plgpu_key_ranges(kcols, 2, r, None))
    codes, ok = N.Column(), C.c_int32(0)
    N.check(N.lib().plgpu_key_pack(kcols, 2, r, C.byref(codes), C.byref(ok), None))
    assert ok.value
    dfc = DataFrame(list(df._cols.values()) + [Series._from_native("__key", codes)])
    frames, counts = _partition_world8(_gb_lower(dfc, "__key", aggs, None))
    plan = (keys, [df[k]._col.dtype for k in keys], [df[k]._logical_dtype() for k in keys], r)
    frames = [D._unpack_keys(f, "__key", plan, ["sa", "sb", "mx", "len"]) for f in frames]
    _assert_same_groups(frames, ref, keys, ["sa", "sb", "mx", "len"])
    del df, dfc, sym, day, a, b
    torch.cuda.empty_cache()
