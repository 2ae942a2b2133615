"""GPU parity of the multi-GPU join's device operations through the C-ABI:
plgpu_hash_partition (exact destinations against a numpy restatement of the
routing hash, stable partition-major order, equal keys co-located),
plgpu_gather_rows / plgpu_pack_bits (bit-exact round trip of values,
Booleans and validity), and a W-way shuffle join and broadcast join simulated
in one process on one GPU (the per-destination segments concatenated the
way all_to_all_single / all_gather lay them out), whose union must equal the
oracle's inner join (oracle.join_inner_multi, after polars-ops/src/frame/
join/mod.rs:625) as a multiset of row pairs.  The torch.distributed path
itself runs at world_size 1 over RCCL.
"""

import os
import socket

import numpy as np
import pytest

import polaroid_amd as pl
from polaroid_amd import _native as N
from polaroid_amd import distributed as D
from oracle import oracle as O

pytestmark = pytest.mark.gpu

M64 = (1 << 64) - 1
SEED = 0x5851F42D4C957F2D  # shuffle.hip kShSeed


def _fmix(x):
    x = np.asarray(x, dtype=np.uint64)
    x = x ^ (x >> np.uint64(33))
    x = x * np.uint64(0xFF51AFD7ED558CCD)
    x = x ^ (x >> np.uint64(33))
    x = x * np.uint64(0xC4CEB9FE1A85EC53)
    return x ^ (x >> np.uint64(33))


def _word(v):
    """shuffle.hip / tuplehash.hpp mk_word: the 64-bit key word."""
    if v.dtype == np.float64:
        b = v.view(np.uint64).copy()
        mag = b & np.uint64(0x7FFFFFFFFFFFFFFF)
        b[mag == 0] = 0
        b[mag > np.uint64(0x7FF0000000000000)] = np.uint64(0x7FF8000000000000)
        return b
    if v.dtype == np.int32:
        return v.astype(np.int64).view(np.uint64)
    if v.dtype == np.uint32:
        return v.astype(np.uint64)
    if v.dtype == np.bool_:
        return v.astype(np.uint64)
    return v.view(np.uint64)


def _mulhi(a, b):
    a_lo, a_hi = a & np.uint64(0xFFFFFFFF), a >> np.uint64(32)
    lo_lo = a_lo * np.uint64(b)
    hi_lo = a_hi * np.uint64(b)
    return (hi_lo + (lo_lo >> np.uint64(32))) >> np.uint64(32)


def _dest(keys, nparts, nulls_equal):
    """Restatement of sh_dest: fixed-seed tuple hash, multiply-high routing
    (polars-utils/src/hashing.rs:101), null tuples dropped or to partition 0."""
    n = keys[0][0].shape[0]
    h = np.full(n, SEED, dtype=np.uint64)
    anynull = np.zeros(n, bool)
    with np.errstate(over="ignore"):
        for i, (v, m) in enumerate(keys):
            valid = np.ones(n, bool) if m is None else m
            anynull |= ~valid
            w = np.where(valid, _fmix(_word(v) ^ np.uint64(SEED)), np.uint64(0x6A09E667F3BCC909 + i))
            h = _fmix(h * np.uint64(0x9E3779B97F4A7C15) + w + np.uint64(i))
    d = _mulhi(h, nparts).astype(np.int64)  # nparts < 2^32 keeps the split product exact
    d[anynull] = -1 if not nulls_equal else 0
    return d


def _keys(rng, n, kinds):
    out = []
    for k in kinds:
        if k == "i64":
            out.append((rng.integers(-50, 50, n).astype(np.int64) * 1_000_000_007, None))
        elif k == "i64n":
            out.append((rng.integers(0, 1000, n).astype(np.int64), rng.random(n) > 0.1))
        elif k == "i32":
            out.append((rng.integers(-3, 3, n).astype(np.int32), rng.random(n) > 0.05))
        elif k == "u32":
            out.append((rng.integers(0, 2**32 - 1, n, dtype=np.uint64).astype(np.uint32) % np.uint32(97), None))
        elif k == "f64":
            out.append((np.array([0.0, -0.0, np.nan, -np.nan, 1.5, -2.25])[rng.integers(0, 6, n)], None))
        elif k == "bool":
            out.append((rng.random(n) < 0.5, rng.random(n) > 0.1))
    return out


def _series(name, v, m):
    return pl.Series.from_numpy(name, v, m)


@pytest.mark.parametrize("nparts", [1, 2, 3, 8, 1000])
@pytest.mark.parametrize("kinds", [["i64"], ["i64n"], ["i32", "f64"], ["u32", "bool", "i64n"]])
@pytest.mark.parametrize("nulls_equal", [False, True])
def test_hash_partition_exact(gpu, nparts, kinds, nulls_equal):
    rng = np.random.default_rng(nparts * 7 + len(kinds))
    n = 70_001
    keys = _keys(rng, n, kinds)
    df = pl.DataFrame([_series(f"k{i}", v, m) for i, (v, m) in enumerate(keys)])
    perm, counts = D.GpuJoinOps.partition(df, df.columns, nparts, nulls_equal)
    p = perm.to_numpy().astype(np.int64)
    d = _dest(keys, nparts, nulls_equal)
    live = np.nonzero(d >= 0)[0]
    expect = live[np.argsort(d[live], kind="stable")]
    assert counts == [int((d == r).sum()) for r in range(nparts)]
    assert np.array_equal(p, expect)


def test_hash_partition_empty_and_errors(gpu):
    df = pl.DataFrame([pl.Series.from_numpy("k", np.zeros(0, np.int64))])
    perm, counts = D.GpuJoinOps.partition(df, ["k"], 4, False)
    assert perm.len() == 0 and counts == [0, 0, 0, 0]
    df = pl.DataFrame([pl.Series.from_numpy("k", np.arange(10, dtype=np.int64))])
    with pytest.raises(pl.InvalidOperationError):
        D.GpuJoinOps.partition(df, ["k"], 0, False)
    with pytest.raises(pl.InvalidOperationError):
        D.GpuJoinOps.partition(df, ["k"], 1025, False)


@pytest.mark.parametrize("n", [0, 1, 63, 64, 65, 100_003])
def test_wire_round_trip(gpu, n):
    """to_wire (plgpu_gather_rows) -> from_wire (plgpu_pack_bits) is the
    identity on values, Booleans and validity, with and without a perm."""
    rng = np.random.default_rng(n)
    cols = {
        "a": (rng.integers(-2**62, 2**62, n).astype(np.int64), rng.random(n) > 0.3),
        "b": (rng.standard_normal(n), None),
        "c": (rng.integers(-2**31, 2**31 - 1, n).astype(np.int32), None),
        "d": (rng.integers(0, 2**32 - 1, n, dtype=np.uint64).astype(np.uint32), rng.random(n) > 0.5),
        "e": (rng.random(n) < 0.5, rng.random(n) > 0.2),
    }
    df = pl.DataFrame([_series(k, v, m) for k, (v, m) in cols.items()])
    for use_perm in (False, True):
        perm = None
        idx = np.arange(n)
        if use_perm:
            idx = rng.permutation(n)
            perm = pl.Series.from_numpy("p", idx.astype(np.uint32))
        wire = D.GpuJoinOps.to_wire(df, perm)
        back = D.GpuJoinOps.from_wire(wire, n)
        assert back.columns == df.columns
        for k, (v, m) in cols.items():
            s = back[k]
            assert s.dtype is df[k].dtype
            exp_m = np.ones(n, bool) if m is None else m[idx]
            assert np.array_equal(s.validity_numpy(), exp_m), k
            assert s.null_count() == int((~exp_m).sum())
            got = s.to_numpy()
            assert np.array_equal(got[exp_m].view(np.uint8), v[idx][exp_m].view(np.uint8)), k


def _pairs_frame(keys, names, rowname, base):
    n = keys[0][0].shape[0]
    s = [_series(nm, v, m) for nm, (v, m) in zip(names, keys)]
    s.append(pl.Series.from_numpy(rowname, np.arange(base, base + n, dtype=np.int64)))
    return pl.DataFrame(s)


def _simulate_shuffle(lshards, rshards, names, world, nulls_equal, how="inner"):
    import torch

    ops = D.GpuJoinOps
    sides = []
    keep_nulls = (how in ("left", "anti", "full"), how in ("right", "full"))  # as run_join routes them
    for si, shards in enumerate((lshards, rshards)):
        wires = []
        for df in shards:
            perm, counts = ops.partition(df, names, world, nulls_equal or keep_nulls[si])
            wires.append((ops.to_wire(df, perm), counts))
        frames = []
        for dest in range(world):
            cols = []
            n = 0
            for ci in range(len(wires[0][0])):
                vals, valids = [], []
                for w, counts in wires:
                    off, k = sum(counts[:dest]), counts[dest]
                    c = w[ci]
                    vals.append(c.values[off:off + k])
                    if c.valid is not None:
                        valids.append(c.valid[off:off + k])
                c0 = wires[0][0][ci]
                cols.append(D.WireColumn(c0.name, c0.dtype, torch.cat(vals).contiguous(),
                                         torch.cat(valids).contiguous() if valids else None))
            n = sum(counts[dest] for _, counts in wires)
            frames.append(ops.from_wire(cols, n))
        sides.append(frames)
    lk = names[0] if len(names) == 1 else tuple(names)
    return [ops.local_join(l, r, lk, lk, "_right", nulls_equal, how) for l, r in zip(*sides)]


def _check_union(outs, lkeys, rkeys, nulls_equal):
    ol, orr = O.join_inner_multi(lkeys, rkeys, nulls_equal)
    gl = np.concatenate([o["li"].to_numpy() for o in outs]).astype(np.int64)
    gr = np.concatenate([o["ri"].to_numpy() for o in outs]).astype(np.int64)
    assert gl.shape == ol.shape
    a, b = np.lexsort((gr, gl)), np.lexsort((orr, ol))
    assert np.array_equal(gl[a], ol[b]) and np.array_equal(gr[a], orr[b])


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("kinds", [["i64"], ["i64n"], ["i32", "f64", "bool"]])
@pytest.mark.parametrize("nulls_equal", [False, True])
def test_shuffle_join_simulated(gpu, world, kinds, nulls_equal):
    rng = np.random.default_rng(world * 31 + len(kinds))
    names = [f"k{i}" for i in range(len(kinds))]
    nl, nr = [5000, 0, 7001, 3000][:world] + [4000] * max(0, world - 4), [2000, 1500, 0, 999][:world] + \
        [800] * max(0, world - 4)
    lk_sh = [_keys(rng, n, kinds) for n in nl]
    rk_sh = [_keys(rng, n, kinds) for n in nr]
    lsh = [_pairs_frame(k, names, "li", sum(nl[:i])) for i, k in enumerate(lk_sh)]
    rsh = [_pairs_frame(k, names, "ri", sum(nr[:i])) for i, k in enumerate(rk_sh)]
    outs = _simulate_shuffle(lsh, rsh, names, world, nulls_equal)
    cat = lambda sh, j: (np.concatenate([s[j][0] for s in sh]),  # noqa: E731
                         None if sh[0][j][1] is None else np.concatenate([s[j][1] for s in sh]))
    lkeys = [cat(lk_sh, j) for j in range(len(kinds))]
    rkeys = [cat(rk_sh, j) for j in range(len(kinds))]
    _check_union(outs, lkeys, rkeys, nulls_equal)
    for o in outs:
        assert o.columns == names + ["li", "ri"]


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("how", ["left", "right", "full", "semi", "anti"])
@pytest.mark.parametrize("nulls_equal", [False, True])
def test_shuffle_join_types_simulated(gpu, world, how, nulls_equal):
    """Every join type through the shuffle (partition, wire round trip,
    per-destination join) simulated on one GPU: the union of the ranks'
    (left, right) index pairs equals the single-process join's."""
    rng = np.random.default_rng(world * 7 + len(how) + nulls_equal)
    nl = [3000, 0, 4001][:world] + [1500] * max(0, world - 3)
    nr = [1200, 900, 0][:world] + [600] * max(0, world - 3)
    lk_sh = [_keys(rng, n, ["i64n"]) for n in nl]
    rk_sh = [_keys(rng, n, ["i64n"]) for n in nr]
    lsh = [_pairs_frame(k, ["k"], "li", sum(nl[:i])) for i, k in enumerate(lk_sh)]
    rsh = [_pairs_frame(k, ["k"], "ri", sum(nr[:i])) for i, k in enumerate(rk_sh)]
    outs = _simulate_shuffle(lsh, rsh, ["k"], world, nulls_equal, how)
    cat = lambda sh: (np.concatenate([s[0][0] for s in sh]), np.concatenate([s[0][1] for s in sh]))  # noqa: E731
    lv, lm = cat(lk_sh)
    rv, rm = cat(rk_sh)
    ol, orr = O.join(O.HostCol(lv, lm), O.HostCol(rv, rm), how, nulls_equal)

    def idx(o, name):
        s = o[name]
        return np.where(s.validity_numpy(), s.to_numpy().astype(np.int64), -1)

    gl = np.concatenate([idx(o, "li") for o in outs])
    if how in ("semi", "anti"):
        assert np.array_equal(np.sort(gl), np.sort(ol))
        return
    gr = np.concatenate([idx(o, "ri") for o in outs])
    a, b = np.lexsort((gr, gl)), np.lexsort((orr, ol))
    assert np.array_equal(gl[a], ol[b]) and np.array_equal(gr[a], orr[b])


def test_join_world1_rccl(gpu):
    """distributed.join over torch.distributed (nccl = RCCL), one rank, both
    strategies, against the single-GPU join."""
    import torch.distributed as dist

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        rng = np.random.default_rng(9)
        lk, rk = _keys(rng, 200_000, ["i64n"]), _keys(rng, 30_000, ["i64n"])
        left = _pairs_frame(lk, ["k"], "li", 0)
        right = _pairs_frame(rk, ["k"], "ri", 0)
        right = pl.DataFrame([right["k"], right["ri"],
                              pl.Series.from_numpy("flag", rng.random(30_000) < 0.5, rng.random(30_000) > 0.1)])
        for strategy in ("shuffle", "broadcast", "auto"):
            info = {}
            out = D.join(left, right, on="k", strategy=strategy, info=info)
            assert info["strategy"] == (strategy if strategy != "auto" else "broadcast")
            _check_union([out], lk, rk, False)
            ref = left.join(right, on="k")
            a = np.lexsort((out["ri"].to_numpy(), out["li"].to_numpy()))
            b = np.lexsort((ref["ri"].to_numpy(), ref["li"].to_numpy()))
            assert out.columns == ref.columns
            assert np.array_equal(out["flag"].to_numpy()[a], ref["flag"].to_numpy()[b])
            assert np.array_equal(out["flag"].validity_numpy()[a], ref["flag"].validity_numpy()[b])
        for how in ("left", "right", "full", "semi", "anti"):
            for strategy in ("shuffle", "auto"):
                info = {}
                out = D.join(left, right, on="k", how=how, strategy=strategy, info=info)
                ref = left.join(right, on="k", how=how)
                assert out.columns == ref.columns and out.height == ref.height, (how, strategy)
                key = [c for c in ("li", "ri") if c in ref.columns]
                got = sorted(zip(*[out[c].to_list() for c in key]), key=str)
                exp = sorted(zip(*[ref[c].to_list() for c in key]), key=str)
                assert got == exp, (how, strategy)
        # large enough that reading a receive buffer before RCCL finished
        # writing it would show (the buffers are host-waited on)
        import torch

        g = torch.Generator(device="cuda")
        g.manual_seed(1)
        pk = torch.randint(0, 4_000_000, (40_000_000,), device="cuda", generator=g)
        bk = torch.randperm(4_000_000, device="cuda", generator=g)[:2_000_000].contiguous()
        big_l = pl.DataFrame([pl.Series.from_torch("k", pk)])
        big_r = pl.DataFrame([pl.Series.from_torch("k", bk), pl.Series.from_torch("p", bk * 3 + 1)])
        member = torch.zeros(4_000_000, dtype=torch.bool, device="cuda")
        member[bk] = True
        expect = int(member[pk].sum().item())
        for strategy in ("shuffle", "broadcast"):
            out = D.join(big_l, big_r, on="k", strategy=strategy)
            assert out.height == expect, strategy
            k = torch.from_numpy(out["k"].to_numpy())
            assert torch.equal(torch.from_numpy(out["p"].to_numpy()), k * 3 + 1), strategy
    finally:
        dist.destroy_process_group()
