"""GPU parity of the hash-partitioned group-by (partial -> export -> merge)
through the C-ABI, against the oracle's exact leg on the concatenated data.

A W-way partitioned run is simulated in one process on one GPU: W shards are
pre-aggregated by plgpu_gb_partial_begin, each with its own fixed-point
windows, exported with plgpu_gb_partial_export, the records for each
destination are concatenated the way all_to_all_single lays them out, and
each destination merges them with plgpu_gb_merge_sources given every
source's record count and windows.  The union
of the W partitions must equal the single-pass result bit for bit (exact
f64 sums are associative, so sharding cannot change them).  The real
torch.distributed path is exercised at world_size 1 over RCCL.
"""

import math
import os
import socket

import numpy as np
import pytest

import polaroid_amd as pl
from polaroid_amd import distributed as D
from polaroid_amd.frame import _gb_lower
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.asarray(a, dtype=np.float64).view(np.uint64)


def _frame(rng, n, scale=100.0, nulls=True):
    a = rng.standard_normal(n) * scale
    a[rng.random(n) < 0.01] = np.nan
    a[rng.random(n) < 0.005] = np.inf
    a[rng.random(n) < 0.01] = -0.0
    b = rng.integers(-10**12, 10**12, n).astype(np.int64)
    d = rng.uniform(-5, 5, n)
    va = (rng.random(n) > 0.05) if nulls else None
    vd = (rng.random(n) > 0.05) if nulls else None
    return {"a": (a, va), "b": (b, None), "d": (d, vd)}


AGGS = [("sum", "a"), ("mean", "a"), ("min", "a"), ("max", "d"), ("count", "a"), ("len", "a"),
        ("sum", "b"), ("sum", "d")]


def _simulate(shards, world, aggs, pred):
    """Run the partitioned protocol over `shards` (list of GPU DataFrames)."""
    import torch

    exprs = [getattr(pl.col(c), k)().alias(f"{k}_{c}") for k, c in aggs]
    parts = [D.GpuPartial(_gb_lower(df, "k", exprs, pred), world) for df in shards]
    windows = [p.begin() for p in parts]
    rw = parts[0].record_words
    exported = [p.export() for p in parts]
    frames = []
    for dest in range(world):
        segs, cnts = [], []
        for send, counts in exported:
            off = sum(counts[:dest]) * rw
            segs.append(send[off: off + counts[dest] * rw])
            cnts.append(counts[dest])
        recv = torch.cat(segs) if segs else torch.empty(0, dtype=torch.int64, device="cuda")
        out, _ = parts[dest].merge(recv.contiguous(), cnts, windows)
        frames.append(out)
    return frames, windows


def _simulate_wide(shards, world, aggs, pred):
    """_simulate with the wide-sum agreement of run_partitioned (agree_wide:
    wide on any shard, the union of the exponent ranges)."""
    import torch

    exprs = [getattr(pl.col(c), k)().alias(f"{k}_{c}") for k, c in aggs]
    parts = [D.GpuPartial(_gb_lower(df, "k", exprs, pred), world) for df in shards]
    windows = [p.begin() for p in parts]
    reps = [p.wide_info() for p in parts]
    A = len(reps[0][0])
    wide = [max(r[0][a] for r in reps) for a in range(A)]
    lo = [min(r[1][a] for r in reps) for a in range(A)]
    hi = [max(r[2][a] for r in reps) for a in range(A)]
    if any(wide):
        for p in parts:
            p.set_wide(wide, lo, hi)
    rw = parts[0].record_words
    assert all(p.record_words == rw for p in parts)
    exported = [p.export() for p in parts]
    frames = []
    for dest in range(world):
        segs, cnts = [], []
        for send, counts in exported:
            off = sum(counts[:dest]) * rw
            segs.append(send[off: off + counts[dest] * rw])
            cnts.append(counts[dest])
        recv = torch.cat(segs) if segs else torch.empty(0, dtype=torch.int64, device="cuda")
        out, _ = parts[dest].merge(recv.contiguous(), cnts, windows)
        frames.append(out)
    return frames, wide, rw


@pytest.mark.parametrize("layout", ["one_wide", "all_wide", "none_wide"])
@pytest.mark.parametrize("world", [2, 3])
def test_wide_sum_partial_states_bit_identical(gpu, world, layout):
    """An f64 sum whose values span more binades than one window on some
    shards (1e300 / 1e-300 / subnormal values, signs mixed, cancelling
    groups, NaN / inf and nulls) crosses the partial-state protocol as digit
    records over the union of the shards' exponent ranges: the union of the
    partitions equals the oracle's exact group-by bit for bit (the
    single-GPU wide sum's result)."""
    rng = np.random.default_rng(world * 7 + len(layout))
    n = 40_000
    shards_np = []
    for s in range(world):
        x = rng.standard_normal(n) * 10.0 ** (s * 3)
        wide_here = layout == "all_wide" or (layout == "one_wide" and s == world - 1)
        if wide_here:
            x[rng.random(n) < 0.2] *= 1e300 / 10.0 ** (s * 3)
            x[rng.random(n) < 0.2] *= 1e-300
            x[rng.random(n) < 0.01] = 5e-324 * rng.integers(1, 100)
        x[rng.random(n) < 0.002] = np.nan
        x[rng.random(n) < 0.001] = -np.inf
        b = rng.integers(-10**12, 10**12, n).astype(np.int64)
        xv = rng.random(n) > 0.03
        shards_np.append((x, xv, b))
    key = rng.integers(0, 300, world * n).astype(np.int64) * 7919 - 11
    # a cancelling group: +1e300 and -1e300 and a tiny value on a wide
    # shard (+-1e3 otherwise)
    key[:6] = 42
    big, tiny = (1e300, 3e-310) if layout == "all_wide" else (1e3, 0.125)
    shards_np[0][0][:6] = [big, -big, tiny, big, -big, 2.5]
    shards_np[0][1][:6] = True
    aggs = [("sum", "x"), ("mean", "x"), ("sum", "b"), ("count", "x"), ("len", "x")]
    shards = []
    for s in range(world):
        x, xv, b = shards_np[s]
        sl = slice(s * n, (s + 1) * n)
        shards.append(pl.DataFrame({"k": pl.Series.from_numpy("k", key[sl]), "x": pl.Series.from_numpy("x", x, xv),
                                    "b": pl.Series.from_numpy("b", b)}))
    frames, wide, rw = _simulate_wide(shards, world, aggs, None)
    assert bool(wide[0]) == (layout != "none_wide")
    cols = {"x": (np.concatenate([t[0] for t in shards_np]), np.concatenate([t[1] for t in shards_np])),
            "b": (np.concatenate([t[2] for t in shards_np]), None)}
    _check(frames, cols, key, None, aggs, None, ["x", "b"])


def _check(frames, cols, key, kvalid, aggs, pred_prog, names):
    n = key.shape[0]
    hc = [O.HostCol(cols[c][0], cols[c][1]) for c in names]
    okeys, okvalid, oouts = O.group_by_agg(O.HostCol(key, kvalid), hc, pred_prog,
                                           [(k, names.index(c)) for k, c in aggs], n, O.SUM_EXACT)
    gk = np.concatenate([f["k"].to_numpy().astype(np.int64) for f in frames])
    gkv = np.concatenate([f["k"].validity_numpy() for f in frames])
    # each group on exactly one rank
    assert gk.shape[0] == okeys.shape[0]
    assert len(set(gk[gkv].tolist())) == int(gkv.sum())
    assert int((~gkv).sum()) <= 1
    go, oo = np.lexsort((gk, ~gkv)), np.lexsort((okeys, ~okvalid))
    assert np.array_equal(gkv[go], okvalid[oo])
    assert np.array_equal(gk[go][gkv[go]], okeys[oo][okvalid[oo]])
    for (kind, c), (ov, ovalid) in zip(aggs, oouts):
        gv = np.concatenate([f[f"{kind}_{c}"].to_numpy() for f in frames])[go]
        gvalid = np.concatenate([f[f"{kind}_{c}"].validity_numpy() for f in frames])[go]
        ov, ovalid = ov[oo], ovalid[oo]
        assert np.array_equal(gvalid, ovalid), (kind, c)
        if ov.dtype == np.float64:
            g, o = gv[ovalid], ov[ovalid]
            assert np.array_equal(np.isnan(g), np.isnan(o)), (kind, c)
            m = ~np.isnan(o)
            assert np.array_equal(_bits(g)[m], _bits(o)[m]), (kind, c, g[m][:4], o[m][:4])
        else:
            assert np.array_equal(gv[ovalid].astype(np.int64), ov[ovalid].astype(np.int64)), (kind, c)


def _run_case(world, nshards, n, card, pred=None, pred_prog=None, pred_names=(), scales=None, nulls=True,
              specials=True):
    rng = np.random.default_rng(world * 1000 + n + card)
    parts = []
    for s in range(nshards):
        sc = scales[s] if scales else 100.0
        parts.append(_frame(rng, n, sc, nulls))
    cols = {c: (np.concatenate([p[c][0] for p in parts]),
                None if parts[0][c][1] is None else np.concatenate([p[c][1] for p in parts]))
            for c in parts[0]}
    N = n * nshards
    key = rng.integers(0, card, N).astype(np.int64) * 1_000_003 - 77
    kvalid = None
    if specials:
        key[rng.random(N) < 0.01] = np.iinfo(np.int64).min
        kvalid = rng.random(N) > 0.01
    names = list(dict.fromkeys(list(pred_names) + [c for _, c in AGGS]))
    shards = []
    for s in range(nshards):
        sl = slice(s * n, (s + 1) * n)
        data = {"k": pl.Series.from_numpy("k", key[sl], None if kvalid is None else kvalid[sl])}
        for c in names:
            v, m = cols[c]
            data[c] = pl.Series.from_numpy(c, v[sl], None if m is None else m[sl])
        shards.append(pl.DataFrame(data))
    frames, agreed = _simulate(shards, world, AGGS, pred)
    _check(frames, cols, key, kvalid, AGGS, pred_prog, names)
    return frames, agreed


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("card", [1, 100, 20000])
def test_partitioned_vs_oracle(gpu, world, card):
    _run_case(world, world, 30000, card)


def test_partitioned_with_predicate(gpu):
    prog = [(1, 0, 0), (2, 0, 0.5), (24, 0, 0)]   # d > 0.5
    _run_case(4, 4, 50000, 500, pred=pl.col("d") > 0.5, pred_prog=prog, pred_names=["d"])


def test_partitioned_window_agreement(gpu):
    """Shards of very different magnitude sample different windows; the
    merge shifts every source's exact states onto the lowest window, which
    must reproduce the exact sum of all shards."""
    frames, windows = _run_case(2, 2, 40000, 50, scales=[1e-3, 1e12], nulls=False, specials=False)
    assert windows[0][0] < windows[1][0] - 40


def test_partitioned_windows_too_far_apart(gpu):
    """Sums whose windows differ by more than one 192-bit state spans are
    refused (PLGPU_ERR_CAPACITY -> ComputeError), never wrong."""
    with pytest.raises(pl.ComputeError, match="192-bit"):
        _run_case(2, 2, 20000, 10, scales=[1e-40, 1e40], nulls=False, specials=False)


def test_partitioned_fast_path_shards(gpu):
    """Null-free 8-byte shards take the fast kernel in the partial stage."""
    _run_case(2, 2, 262144, 100, nulls=False, specials=False)


def test_partitioned_empty_shard(gpu):
    _run_case(2, 3, 0, 10)


def test_group_by_agg_world1_rccl(gpu):
    """The torch.distributed path itself (nccl = RCCL), one rank."""
    import torch
    import torch.distributed as dist

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        rng = np.random.default_rng(3)
        n = 100_000
        cols = _frame(rng, n)
        key = rng.integers(0, 300, n).astype(np.int64)
        df = pl.DataFrame({"k": pl.Series.from_numpy("k", key), "a": pl.Series.from_numpy("a", *cols["a"]),
                           "d": pl.Series.from_numpy("d", *cols["d"])})
        info = {}
        out = D.group_by_agg(df, "k", [pl.col("a").sum().alias("sum_a"), pl.col("d").mean().alias("mean_d")],
                             pl.col("d") > 0.0, info=info)
        ref = df.lazy().filter(pl.col("d") > 0.0).group_by("k").agg(
            pl.col("a").sum().alias("sum_a"), pl.col("d").mean().alias("mean_d")).collect()
        go, ro = np.argsort(out["k"].to_numpy()), np.argsort(ref["k"].to_numpy())
        assert np.array_equal(out["k"].to_numpy()[go], ref["k"].to_numpy()[ro])
        for c in ("sum_a", "mean_d"):
            g, r = out[c].to_numpy()[go], ref[c].to_numpy()[ro]
            assert np.array_equal(out[c].validity_numpy()[go], ref[c].validity_numpy()[ro])
            assert np.array_equal(np.isnan(g), np.isnan(r))
            m = ~np.isnan(r)
            assert np.array_equal(_bits(g)[m], _bits(r)[m])
        assert info["groups"] == ref.height
    finally:
        dist.destroy_process_group()


def test_group_by_agg_world1_rccl_string_key(gpu):
    """The multi-GPU group-by with a String symbol key (<= 7 bytes: exact
    Int64 codes through the partial-state exchange), one RCCL rank, against
    the single-GPU group-by; a longer key takes the row shuffle."""
    import torch.distributed as dist

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        rng = np.random.default_rng(4)
        n = 200_000
        pool = np.array(["AAPL", "MSFT", "", "BRK.B", "日本", "x"] + [f"S{i:04d}" for i in range(200)], dtype=object)
        sym = pool[rng.integers(0, pool.size, n)]
        sv = rng.random(n) > 0.02
        v = rng.standard_normal(n)
        df = pl.DataFrame({"sym": pl.Series.from_numpy("sym", sym, sv), "v": pl.Series.from_numpy("v", v)})
        out = D.group_by_agg(df, "sym", [pl.col("v").sum().alias("s"), pl.len()], pl.col("v") > -1.0)
        ref = df.lazy().filter(pl.col("v") > -1.0).group_by("sym").agg(pl.col("v").sum().alias("s"),
                                                                        pl.len()).collect()
        assert out["sym"].dtype == pl.String
        got = sorted(zip(out["sym"].to_list(), out["s"].to_list(), out["len"].to_list()), key=str)
        exp = sorted(zip(ref["sym"].to_list(), ref["s"].to_list(), ref["len"].to_list()), key=str)
        assert got == exp
        # a predicate on the String key itself (lowered before the key becomes codes)
        pred = (pl.col("sym") == "AAPL") | pl.col("sym").str.starts_with("S00")
        out = D.group_by_agg(df, "sym", [pl.col("v").sum().alias("s"), pl.len()], pred)
        ref = df.lazy().filter(pred).group_by("sym").agg(pl.col("v").sum().alias("s"), pl.len()).collect()
        got = sorted(zip(out["sym"].to_list(), out["s"].to_list(), out["len"].to_list()), key=str)
        exp = sorted(zip(ref["sym"].to_list(), ref["s"].to_list(), ref["len"].to_list()), key=str)
        assert got == exp and len(got) == 1 + 100
        # a longer key takes the row-shuffle protocol
        long_df = pl.DataFrame({"sym": pl.Series("sym", ["AAPL", "TOOLONGKEY", "AAPL"]),
                                "v": pl.Series("v", [1.0, 2.0, 4.0])})
        info = {}
        out = D.group_by_agg(long_df, "sym", [pl.col("v").sum()], info=info)
        assert sorted(zip(out["sym"].to_list(), out["v"].to_list())) == [("AAPL", 5.0), ("TOOLONGKEY", 2.0)]
        assert info["protocol"] == "row_shuffle"
    finally:
        dist.destroy_process_group()


def _fl_simulate(shards, world, key, exprs, pred):
    """run_first_last over `shards` in one process: each shard's local
    first / last frame is routed by plgpu_gb_route, every destination
    receives the sources' rows in source-rank order (as all_to_all lays them
    out) and combines them."""
    import torch

    from polaroid_amd.frame import _group_by

    ops = D.GpuFirstLastOps(key, exprs)
    sent = []
    for df in shards:
        local = _group_by(df, key, exprs, False, pred, None)
        perm, counts = ops.route(local, world)
        sent.append((ops.to_wire(local, perm), counts))
    frames = []
    for dest in range(world):
        cols = []
        n = sum(c[dest] for _, c in sent)
        for j in range(len(sent[0][0])):
            # a column is sent with a validity mask if any source holds nulls in it (_wire_spec)
            nullable = any(w[j].valid is not None for w, _ in sent)
            vals, valid = [], []
            for wire, counts in sent:
                off = sum(counts[:dest])
                vals.append(wire[j].values[off: off + counts[dest]])
                if nullable:
                    valid.append(wire[j].valid[off: off + counts[dest]] if wire[j].valid is not None else
                                 torch.ones(counts[dest], dtype=torch.uint8, device="cuda"))
            proto = sent[0][0][j]
            cols.append(D.WireColumn(proto.name, proto.dtype, torch.cat(vals).contiguous(),
                                     torch.cat(valid).contiguous() if nullable else None))
        frames.append(ops.combine(ops.from_wire(cols, n)))
    return frames


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_first_last_across_ranks(gpu, world):
    """first() / last() over W shards (rank order = row order): the union of
    the W owners' results equals the single-GPU group-by of the concatenated
    rows, values and nulls included, and each group lands on the rank that
    owns its partial states (plgpu_gb_route = the records' partition)."""
    rng = np.random.default_rng(40 + world)
    n = 20_000
    N_ = n * world
    key = rng.integers(0, 500, N_).astype(np.int64) * 7 - 1000
    key[rng.random(N_) < 0.01] = np.iinfo(np.int64).min
    kvalid = rng.random(N_) > 0.01
    a = rng.standard_normal(N_)
    va = rng.random(N_) > 0.1
    b = rng.integers(-50, 50, N_).astype(np.int32)
    full = pl.DataFrame({"k": pl.Series.from_numpy("k", key, kvalid), "a": pl.Series.from_numpy("a", a, va),
                         "b": pl.Series.from_numpy("b", b)})
    shards = [pl.DataFrame({"k": pl.Series.from_numpy("k", key[s * n:(s + 1) * n], kvalid[s * n:(s + 1) * n]),
                            "a": pl.Series.from_numpy("a", a[s * n:(s + 1) * n], va[s * n:(s + 1) * n]),
                            "b": pl.Series.from_numpy("b", b[s * n:(s + 1) * n])}) for s in range(world)]
    exprs = [pl.col("a").first().alias("fa"), pl.col("a").last().alias("la"), pl.col("b").first().alias("fb"),
             pl.col("b").last().alias("lb")]
    pred = pl.col("b") > -30
    frames = _fl_simulate(shards, world, "k", exprs, pred)
    ref = full.lazy().filter(pred).group_by("k").agg(*exprs).collect()

    def rows(f):
        ks = f["k"].to_numpy().astype(np.int64)
        kv = f["k"].validity_numpy()
        out = {}
        for i in range(f.height):
            vals = []
            for c in ("fa", "la", "fb", "lb"):
                v = f[c].validity_numpy()[i]
                vals.append(f[c].to_numpy()[i].item() if v else None)
            out[(bool(kv[i]), int(ks[i]) if kv[i] else 0)] = tuple(vals)
        return out

    got = {}
    for dest, f in enumerate(frames):
        r = rows(f)
        # ownership: a group's rows were routed to `dest` by the records' partition function
        perm, counts = D.GpuFirstLastOps("k", exprs).route(f, world)
        assert counts[dest] == f.height
        assert not (set(r) & set(got))
        got.update(r)
    assert got == rows(ref)


def test_group_by_agg_world1_rccl_first_last(gpu):
    """group_by_agg with first() / last() next to exact sums, over RCCL at
    world 1 (states + values exchanged, joined on the owner), against the
    single-GPU group-by; first / last alone skip the partial states."""
    import torch.distributed as dist

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        rng = np.random.default_rng(5)
        n = 100_000
        cols = _frame(rng, n)
        key = rng.integers(0, 300, n).astype(np.int32)
        kv = rng.random(n) > 0.02
        df = pl.DataFrame({"k": pl.Series.from_numpy("k", key, kv), "a": pl.Series.from_numpy("a", *cols["a"]),
                           "d": pl.Series.from_numpy("d", *cols["d"])})
        for exprs in ([pl.col("a").sum().alias("s"), pl.col("d").first().alias("f"), pl.len(),
                       pl.col("a").last().alias("l")],
                      [pl.col("d").last().alias("l"), pl.col("a").first().alias("f")]):
            info = {}
            out = D.group_by_agg(df, "k", exprs, pl.col("d") > 0.0, info=info)
            ref = df.lazy().filter(pl.col("d") > 0.0).group_by("k").agg(*exprs).collect()
            assert out.columns == ref.columns and out["k"].dtype == pl.Int32
            assert info["groups"] == ref.height and "first_last_ms" in info

            def table(f):
                return sorted(zip(*[[(v if not (isinstance(v, float) and v != v) else "nan") for v in f[c].to_list()]
                                    for c in f.columns]), key=repr)

            assert table(out) == table(ref)
    finally:
        dist.destroy_process_group()


def _ranges(cols):
    import ctypes as C

    from polaroid_amd import _native as N
    from polaroid_amd.frame import _col_array

    r = (C.c_int64 * (3 * len(cols)))()
    N.check(N.lib().plgpu_key_ranges(_col_array(cols), len(cols), r, None))
    return list(r)


def test_key_pack_agreed_across_shards(gpu):
    """plgpu_key_ranges per shard, reduced (min / max / or) as the ranks do,
    then plgpu_key_pack on each shard: equal tuples get equal codes on every
    shard, distinct tuples distinct codes (nulls are values), and
    plgpu_key_unpack restores the tuples; an empty shard reduces neutrally."""
    import ctypes as C

    from polaroid_amd import _native as N
    from polaroid_amd.frame import _col_array

    rng = np.random.default_rng(9)
    shards = []
    for s, n in enumerate([30_000, 0, 17_000]):
        k1 = rng.integers(-5, 40 + 100 * s, n).astype(np.int64)
        k2 = rng.integers(0, 3, n).astype(np.int32)
        kb = rng.random(n) < 0.5
        shards.append([pl.Series.from_numpy("k1", k1, rng.random(n) > 0.1), pl.Series.from_numpy("k2", k2),
                       pl.Series.from_numpy("kb", kb, rng.random(n) > 0.2)])
    rs = [_ranges(c) for c in shards]
    assert rs[1][0] > rs[1][1]  # empty shard: min > max
    agreed = []
    for i in range(3):
        agreed += [min(r[3 * i] for r in rs), max(r[3 * i + 1] for r in rs), max(r[3 * i + 2] for r in rs)]
    ranges = (C.c_int64 * 9)(*agreed)
    seen = {}
    for cols in shards:
        codes = N.Column()
        ok = C.c_int32(0)
        N.check(N.lib().plgpu_key_pack(_col_array(cols), 3, ranges, C.byref(codes), C.byref(ok), None))
        assert ok.value == 1
        cs = pl.Series._from_native("c", codes)
        got = cs.to_numpy().astype(np.int64)
        tuples = list(zip(*[[(None if not v else x) for x, v in zip(c.to_numpy().tolist(), c.validity_numpy())]
                            for c in cols]))
        for t, c in zip(tuples, got.tolist()):
            assert seen.setdefault(t, c) == c
        out = (N.Column * 3)()
        N.check(N.lib().plgpu_key_unpack(C.byref(cs._col), (C.c_int32 * 3)(*[c._col.dtype for c in cols]), 3,
                                         ranges, out, None))
        back = [pl.Series._from_native(c.name, out[i]) for i, c in enumerate(cols)]
        assert list(zip(*[b.to_list() for b in back])) == [tuple(x if x is None else (bool(x) if i == 2 else int(x))
                                                                 for i, x in enumerate(t)) for t in tuples]
    assert len(set(seen.values())) == len(seen)


def test_group_by_agg_world1_rccl_multi_key(gpu):
    """The multi-GPU group-by on (Int64, Int32, Boolean) keys with nulls:
    packed codes agreed over the ranks, then the single-key protocol; against
    the single-GPU multi-key group-by.  A Float key in the tuple takes the
    row shuffle."""
    import torch.distributed as dist

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        rng = np.random.default_rng(6)
        n = 120_000
        cols = _frame(rng, n)
        df = pl.DataFrame({"k1": pl.Series.from_numpy("k1", rng.integers(-50, 50, n).astype(np.int64) * 1000,
                                                      rng.random(n) > 0.05),
                           "k2": pl.Series.from_numpy("k2", rng.integers(0, 7, n).astype(np.int32)),
                           "kb": pl.Series.from_numpy("kb", rng.random(n) < 0.3, rng.random(n) > 0.1),
                           "a": pl.Series.from_numpy("a", *cols["a"]), "d": pl.Series.from_numpy("d", *cols["d"])})
        exprs = [pl.col("a").sum().alias("s"), pl.col("d").max().alias("m"), pl.len(), pl.col("d").first().alias("f")]
        out = D.group_by_agg(df, ("k1", "k2", "kb"), exprs, pl.col("d") > -2.0)
        ref = df.lazy().filter(pl.col("d") > -2.0).group_by("k1", "k2", "kb").agg(*exprs).collect()
        assert out.columns == ref.columns
        assert [out[c].dtype for c in out.columns] == [ref[c].dtype for c in ref.columns]

        def table(f):
            return sorted(zip(*[[(v if not (isinstance(v, float) and v != v) else "nan") for v in f[c].to_list()]
                                for c in f.columns]), key=repr)

        assert table(out) == table(ref)
        fdf = pl.DataFrame({"k": pl.Series.from_numpy("k", np.array([1.0, 2.0])),
                            "j": pl.Series.from_numpy("j", np.array([1, 2], dtype=np.int64))})
        info = {}
        out = D.group_by_agg(fdf, ("k", "j"), [pl.len()], info=info)  # a Float in the tuple: row shuffle
        assert info["protocol"] == "row_shuffle" and sorted(out["len"].to_list()) == [1, 1]
    finally:
        dist.destroy_process_group()


def test_group_by_agg_world1_rccl_var_std(gpu):
    """var / std(ddof) across ranks (means all-gathered, squared deviations
    summed exactly by a second partitioned pass, aligned on the key), one
    RCCL rank, against the single-GPU var / std (itself pinned against the
    exact variance in test_gpu_var_std.py) to 1e-12; single and two keys,
    with nulls, a predicate and groups of one row (ddof=1 -> null)."""
    import torch.distributed as dist

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        rng = np.random.default_rng(8)
        n = 80_000
        cols = _frame(rng, n)
        k = rng.integers(0, 400, n).astype(np.int64)
        k[:5] = [10_000, 10_001, 10_002, 10_003, 10_004]  # one-row groups
        df = pl.DataFrame({"k": pl.Series.from_numpy("k", k, rng.random(n) > 0.03),
                           "j": pl.Series.from_numpy("j", rng.integers(0, 3, n).astype(np.int32)),
                           "b": pl.Series.from_numpy("b", rng.integers(-1000, 1000, n).astype(np.int64)),
                           "d": pl.Series.from_numpy("d", *cols["d"])})
        exprs = [pl.col("d").var().alias("vd"), pl.col("b").std().alias("sb"), pl.col("d").sum().alias("s"),
                 pl.col("b").var(ddof=0).alias("vb0")]
        sym = np.array(["AAPL", "MSFT", "", "BRK.B", "x"], dtype=object)[rng.integers(0, 5, n)]
        df = pl.DataFrame([df[c] for c in df.columns] + [pl.Series.from_numpy("sym", sym, rng.random(n) > 0.02)])
        for key in ("k", ("k", "j"), "sym"):
            by = (key,) if isinstance(key, str) else key
            out = D.group_by_agg(df, key, exprs, pl.col("d") > -4.0)
            ref = df.lazy().filter(pl.col("d") > -4.0).group_by(*by).agg(*exprs).collect()
            assert out.columns == ref.columns

            def table(f):
                return sorted(zip(*[[(v if not (isinstance(v, float) and v != v) else "nan") for v in f[c].to_list()]
                                    for c in f.columns]), key=lambda r: repr(r[:len(by)]))

            # the multi-GPU var / std composes exact passes around a rounded
            # mean; the single-GPU one combines exact states (rounded once):
            # both within 1e-12 of the exact variance, sums bit-identical
            to, tr = table(out), table(ref)
            assert len(to) == len(tr)
            for ro, rr in zip(to, tr):
                assert ro[:len(by)] == rr[:len(by)]
                for c, a, b in zip(out.columns[len(by):], ro[len(by):], rr[len(by):]):
                    if c == "s" or a is None or b is None or isinstance(a, str):
                        assert a == b, (c, a, b)
                    else:
                        assert math.isclose(a, b, rel_tol=1e-12, abs_tol=1e-300), (c, a, b)
    finally:
        dist.destroy_process_group()


def test_group_by_agg_world1_rccl_float_and_narrow_keys(gpu):
    """One Float64 key (canonical-bit codes: -0.0 with 0.0, NaNs together,
    a null group), one Float32, UInt16 and Boolean key (packed codes), over
    RCCL at world 1, against the single-GPU group-by."""
    import torch.distributed as dist

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        rng = np.random.default_rng(12)
        n = 60_000
        cols = _frame(rng, n)
        kf = np.array([0.0, -0.0, np.nan, -np.nan, 1.5, -2.25, np.inf, -np.inf, 1e300])[rng.integers(0, 9, n)]
        kv = rng.random(n) > 0.05
        df = pl.DataFrame({"kf": pl.Series.from_numpy("kf", kf, kv),
                           "kf32": pl.Series.from_numpy("kf32", kf.astype(np.float32), kv),
                           "ku": pl.Series.from_numpy("ku", rng.integers(0, 60000, n).astype(np.uint16)),
                           "kb": pl.Series.from_numpy("kb", rng.random(n) < 0.4, rng.random(n) > 0.1),
                           "a": pl.Series.from_numpy("a", *cols["a"]), "d": pl.Series.from_numpy("d", *cols["d"])})
        exprs = [pl.col("a").sum().alias("s"), pl.col("d").min().alias("m"), pl.len(), pl.col("d").last().alias("l")]

        def table(f):
            return sorted(zip(*[[(v if not (isinstance(v, float) and v != v) else "nan") for v in f[c].to_list()]
                                for c in f.columns]), key=repr)

        for key in ("kf", "kf32", "ku", "kb"):
            out = D.group_by_agg(df, key, exprs, pl.col("d") > -3.0)
            ref = df.lazy().filter(pl.col("d") > -3.0).group_by(key).agg(*exprs).collect()
            assert out.columns == ref.columns and out[key].dtype == ref[key].dtype, key
            assert table(out) == table(ref), key
    finally:
        dist.destroy_process_group()


def test_merge_sources_sum_guard_bits(gpu):
    """Several sources' 192-bit sum states fold into one cell: each shifted
    state must leave ceil(log2 sources) sign bits to spare, so states that
    each fit cannot wrap the cell when added (refused, never wrong).
    Records are built by hand: [kind, key, len, w0, w1, w2, flags]."""
    import torch

    a = pl.Series.from_numpy("a", np.zeros(1))
    df = pl.DataFrame({"k": pl.Series.from_numpy("k", np.zeros(1, np.int64)), "a": a})
    g = _gb_lower(df, "k", [pl.col("a").sum().alias("s")], None)
    part = D.GpuPartial(g, 3)
    assert part.record_words == 7
    base = -100

    def run(big_w1):
        rec = [[0, 5, 1, 1, 0, 0, 0],          # source 0: state 1 at bottom `base`
               [0, 5, 1, 0, big_w1, 0, 0],     # sources 1, 2: state big_w1 * 2^64 at bottom base + 78
               [0, 5, 1, 0, big_w1, 0, 0]]
        t = torch.tensor(rec, dtype=torch.int64, device="cuda").flatten()
        bottoms = [[base] + [0] * 5, [base + 78] + [0] * 5, [base + 78] + [0] * 5]
        return part.merge(t, [1, 1, 1], bottoms)[0]

    # 2^112 shifted by 78 is 2^190: alone it fits 192 bits, two of them wrap
    with pytest.raises(pl.ComputeError, match="192-bit"):
        run(1 << 48)
    # 2^100 shifted: 2^178 each, the exact sum is representable
    out = run(1 << 36)
    want = math.ldexp(1.0, base) + 2 * math.ldexp(1.0, 100 + base + 78)
    assert out["s"].to_list() == [want]


# ------------------------------------------------- row-shuffle protocol
def _canon(v):
    if isinstance(v, float):
        return ("f", "nan" if math.isnan(v) else v.hex())
    return v


def _rows_of(df, names):
    cols = [df[c].to_list() for c in names]
    return sorted((tuple(_canon(v) for v in r) for r in zip(*cols)), key=repr)


def _shuffle_simulate(shards, world, key, aggs, pred):
    """run_shuffled over `shards` in one process: each shard's selected rows
    are partitioned and put on the wire, every destination receives the
    sources' segments in source-rank order (as exchange_columns lays them
    out, String bytes included) and aggregates them."""
    import torch

    ops = D.GpuShuffleOps
    keys = [key] if isinstance(key, str) else list(key)
    names = list(dict.fromkeys(keys + [c for e in aggs for c in e.meta_root_names()]))
    sent, logical = [], None
    for df in shards:
        sub = ops.select(df, pred, names)
        logical = ops.logical(sub, names)
        perm, counts = ops.partition(sub, keys, world, True)
        sent.append((ops.to_wire(sub, perm), counts))
    frames = []
    for dest in range(world):
        n = sum(c[dest] for _, c in sent)
        cols = []
        for j in range(len(names)):
            nullable = any(w[j].valid is not None for w, _ in sent)
            vals, valid, data = [], [], []
            for wire, counts in sent:
                off = sum(counts[:dest])
                vals.append(wire[j].values[off: off + counts[dest]])
                if nullable:
                    valid.append(wire[j].valid[off: off + counts[dest]] if wire[j].valid is not None else
                                 torch.ones(counts[dest], dtype=torch.uint8, device="cuda"))
                if wire[j].data is not None:
                    sb = D._segment_sums(wire[j].values, counts)
                    b0 = sum(sb[:dest])
                    data.append(wire[j].data[b0: b0 + sb[dest]])
            proto = sent[0][0][j]
            cols.append(D.WireColumn(proto.name, proto.dtype, torch.cat(vals).contiguous(),
                                     torch.cat(valid).contiguous() if nullable else None,
                                     torch.cat(data).contiguous() if data else None))
        rows = ops.restore(ops.from_wire(cols, n), names, logical)
        frames.append(ops.local_group_by(rows, keys[0] if len(keys) == 1 else tuple(keys), aggs))
    return frames


def _shuffle_case_frame(rng, n, case):
    """(columns dict of Series inputs, key, aggs, predicate) for one of the
    inputs the partial-state records cannot carry."""
    pool = np.array(["AAPL.NASDAQ", "MSFT", "", "BRK.B-CLASS", "日本語の銘柄", "x" * 40] +
                    [f"SYMBOL-{i:05d}" for i in range(300)], dtype=object)
    v = rng.standard_normal(n) * 100
    v[rng.random(n) < 0.01] = np.nan
    w = rng.uniform(1, 5, n)
    i = rng.integers(-50, 50, n).astype(np.int64)
    cols = {"v": (v, rng.random(n) > 0.05), "w": (w, None), "i": (i, None)}
    if case == "long_string_key":
        cols["s"] = (pool[rng.integers(0, pool.size, n)], rng.random(n) > 0.02)
        key = "s"
        aggs = [pl.col("v").sum().alias("sum_v"), pl.col("v").mean().alias("mean_v"), pl.col("w").min().alias("mn"),
                pl.col("w").max().alias("mx"), pl.col("v").count().alias("cnt"), pl.len(),
                pl.col("w").first().alias("fw"), pl.col("i").last().alias("li")]
    elif case == "float_string_tuple":
        f = rng.choice(np.array([-0.0, 0.0, 1.5, np.nan, -2.25]), n)
        cols["f"] = (f, rng.random(n) > 0.03)
        cols["s"] = (pool[rng.integers(0, 20, n)], None)
        key = ("f", "s", "i")
        aggs = [pl.col("w").sum().alias("sw"), pl.len(), pl.col("v").max().alias("mv")]
    elif case == "wide_sum":
        x = rng.standard_normal(n)
        x[rng.random(n) < 0.3] *= 1e300
        x[rng.random(n) < 0.3] *= 1e-300
        cols["x"] = (x, None)
        key = "i"
        aggs = [pl.col("x").sum().alias("sx"), pl.col("x").mean().alias("mx"), pl.col("w").sum().alias("sw")]
    elif case == "wide_int_tuple":
        # two full-range Int64 keys: the tuple needs more than 63 bits
        cols["k1"] = (rng.integers(-2**62, 2**62, n).astype(np.int64) // 997 * 997, None)
        cols["k2"] = (rng.choice(np.array([-2**63, 2**63 - 1, 0, 5], dtype=np.int64), n), rng.random(n) > 0.05)
        key = ("k1", "k2")
        aggs = [pl.col("w").sum().alias("sw"), pl.col("i").first().alias("fi"), pl.col("v").last().alias("lv")]
    else:  # var / std with a String key in a tuple
        cols["s"] = (pool[rng.integers(0, 10, n)], None)
        key = ("s", "i")
        aggs = [pl.col("w").var().alias("var_w"), pl.col("v").std().alias("std_v"), pl.len()]
    return cols, key, aggs, pl.col("w") > 1.5


SHUFFLE_CASES = ["long_string_key", "float_string_tuple", "wide_sum", "wide_int_tuple", "var_std_tuple"]


@pytest.mark.parametrize("case", SHUFFLE_CASES)
@pytest.mark.parametrize("world", [1, 2, 3])
def test_row_shuffle_group_by_vs_single_gpu(gpu, world, case):
    """The row-shuffle protocol (inputs no fixed-size partial record
    carries), simulated over W shards in one process: the union of the W
    partitions equals the single-GPU group-by of the concatenated shards row
    for row (exact sums; first / last in global row order; every group on
    exactly one rank)."""
    rng = np.random.default_rng(world * 31 + len(case))
    n = 60_000
    cols, key, aggs, pred = _shuffle_case_frame(rng, n, case)
    full = pl.DataFrame({k: pl.Series.from_numpy(k, a, m) for k, (a, m) in cols.items()})
    cuts = np.linspace(0, n, world + 1).astype(int)
    shards = [pl.DataFrame({k: pl.Series.from_numpy(k, a[cuts[r]:cuts[r + 1]],
                                                    None if m is None else m[cuts[r]:cuts[r + 1]])
                            for k, (a, m) in cols.items()}) for r in range(world)]
    frames = _shuffle_simulate(shards, world, key, aggs, pred)
    ref = full.lazy().filter(pred).group_by(key).agg(*aggs).collect()
    names = ref.columns
    got = [r for f in frames for r in _rows_of(f, names)]
    assert sorted(got, key=repr) == _rows_of(ref, names)
    keys = [key] if isinstance(key, str) else list(key)
    seen = [tuple(_canon(v) for v in r) for f in frames for r in zip(*[f[k].to_list() for k in keys])]
    assert len(seen) == len(set(seen))  # each group on exactly one rank


def test_group_by_agg_world1_rccl_row_shuffle(gpu):
    """The row-shuffle protocol through torch.distributed (nccl = RCCL), one
    rank: every input the partial records cannot carry is accepted, reported
    as info["protocol"] == "row_shuffle", and equals the single-GPU group-by;
    the common keys keep the partial-state protocol, and so does a wide f64
    sum (digit records, round 5)."""
    import torch.distributed as dist

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        for case in SHUFFLE_CASES:
            rng = np.random.default_rng(len(case))
            cols, key, aggs, pred = _shuffle_case_frame(rng, 50_000, case)
            df = pl.DataFrame({k: pl.Series.from_numpy(k, a, m) for k, (a, m) in cols.items()})
            info = {}
            out = D.group_by_agg(df, key, aggs, pred, info=info)
            ref = df.lazy().filter(pred).group_by(key).agg(*aggs).collect()
            assert _rows_of(out, ref.columns) == _rows_of(ref, ref.columns), case
            if case == "wide_sum":
                # (round 5) a wide f64 sum stays on the partial states as digits
                assert "protocol" not in info and info["wide_accs"] == 1, (case, info)
            else:
                assert info.get("protocol") == "row_shuffle", (case, info)
        info = {}
        df = pl.DataFrame({"k": pl.Series("k", [1, 2, 1]), "v": pl.Series("v", [1.0, 2.0, 3.0])})
        D.group_by_agg(df, "k", [pl.col("v").sum()], info=info)
        assert "protocol" not in info
    finally:
        dist.destroy_process_group()


def test_join_world1_rccl_string_key_and_payload(gpu):
    """The multi-GPU join's wire carries String columns (per-row lengths +
    bytes): a String-keyed shuffle join with String payloads, one RCCL rank,
    against the single-GPU join."""
    import torch.distributed as dist

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        rng = np.random.default_rng(8)
        pool = np.array([f"instrument-{i:04d}" for i in range(500)] + ["", "é"], dtype=object)
        left = pl.DataFrame({"k": pl.Series.from_numpy("k", pool[rng.integers(0, pool.size, 20_000)],
                                                       rng.random(20_000) > 0.05),
                             "x": pl.Series.from_numpy("x", rng.standard_normal(20_000))})
        right = pl.DataFrame({"k": pl.Series.from_numpy("k", pool[:400]),
                              "name": pl.Series.from_numpy("name", np.array([f"n{i}" * (i % 5) for i in range(400)],
                                                                            dtype=object))})
        for strategy in ("shuffle", "broadcast"):
            info = {}
            out = D.join(left, right, on="k", strategy=strategy, info=info)
            ref = left.join(right, on="k")
            assert info["strategy"] == strategy
            assert _rows_of(out, ref.columns) == _rows_of(ref, ref.columns)
    finally:
        dist.destroy_process_group()
