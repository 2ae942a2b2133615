"""The multi-GPU group-by and join with real kernels across a process
boundary: two rank processes share the one GPU of the test box and talk over
gloo, with every device buffer of the exchange staged through host memory
(distributed._a2a / _all_gather / _all_reduce switch on the gloo backend).

Each rank runs the real GpuPartial begin / export / merge (the
partial-state protocol, configs[4]'s path; also with a 1e300 / 1e-300
column wide on one rank only, carried as digit records over the agreed
range), the row shuffle (String keys
longer than 7 bytes), the first / last value exchange, and the join's
shuffle strategy.  The union of the ranks' outputs must equal the
single-GPU result on the concatenated shards bit for bit.  This is the
nearest evidence to the 8-GPU RCCL run the driver makes: the protocol,
the wire formats and the device-side partial -> transport -> merge path are
the same; only the transport differs.
"""

import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _shard(rank, n=120_000):
    rng = np.random.default_rng(500 + rank)
    k = (rng.integers(0, 400, n) * 7919 - 1000).astype(np.int64)
    a = rng.standard_normal(n) * 100 * (1 + rank)  # different windows per rank
    a[rng.random(n) < 0.01] = np.nan
    d = rng.uniform(-5, 5, n)
    long_keys = np.array([f"instrument-{i:04d}" for i in range(300)], dtype=object)[rng.integers(0, 300, n)]
    # x: within one fixed-point window on rank 0, 1e300 / 1e-300 values on
    # rank 1 (wider than any window): the wide-sum digit states
    x = rng.standard_normal(n) * 50
    if rank == 1:
        x[rng.random(n) < 0.3] *= 1e300
        x[rng.random(n) < 0.3] *= 1e-300
    return k, a, d, long_keys, x


def _frame(pl, rank):
    k, a, d, s, x = _shard(rank)
    return pl.DataFrame({"k": pl.Series.from_numpy("k", k), "a": pl.Series.from_numpy("a", a),
                         "d": pl.Series.from_numpy("d", d), "s": pl.Series("s", s.tolist(), pl.String),
                         "x": pl.Series.from_numpy("x", x)})


def _rows(df, cols):
    return {c: df[c].to_list() for c in cols}


def _worker(rank, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        import torch
        import torch.distributed as dist

        import polaroid_amd as pl
        from polaroid_amd import distributed as D

        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=WORLD)
        try:
            df = _frame(pl, rank)
            pred = pl.col("d") > 0.0
            out = {}
            info = {}
            r = D.group_by_agg(df, "k", [pl.col("a").sum().alias("sa"), pl.col("d").mean().alias("md"),
                                         pl.len().alias("n")], pred, info=info)
            out["states"] = (_rows(r, ["k", "sa", "md", "n"]), info.get("protocol", "partial_states"))
            info = {}
            r = D.group_by_agg(df, "k", [pl.col("x").sum().alias("sx"), pl.col("x").mean().alias("mx"),
                                         pl.col("a").sum().alias("sa")], pred, info=info)
            out["wide"] = (_rows(r, ["k", "sx", "mx", "sa"]),
                           (info.get("protocol", "partial_states"), info.get("wide_accs"), info.get("record_words"),
                            info.get("exchange_bytes"), r.height))
            info = {}
            r = D.group_by_agg(df, "s", [pl.col("a").sum().alias("sa"), pl.col("d").first().alias("fd"),
                                         pl.col("d").last().alias("ld")], pred, info=info)
            out["shuffle"] = (_rows(r, ["s", "sa", "fd", "ld"]), info.get("protocol"))
            info = {}
            r = D.group_by_agg(df, "k", [pl.col("d").first().alias("fd"), pl.col("d").last().alias("ld")],
                               None, info=info)
            out["first_last"] = (_rows(r, ["k", "fd", "ld"]), None)
            right = pl.DataFrame({"k": pl.Series.from_numpy("k", (np.arange(150) * 2 * 7919 - 1000).astype(np.int64)),
                                  "w": pl.Series.from_numpy("w", np.arange(150, dtype=np.float64) + rank * 1000)})
            info = {}
            j = D.join(pl.DataFrame([df["k"], df["a"]]), right, on="k", strategy="shuffle", info=info)
            out["join"] = (_rows(j, ["k", "a", "w"]), info.get("strategy"))
            q.put((rank, out, None))
        finally:
            dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        import traceback

        q.put((rank, None, traceback.format_exc()))


def _canon(rows, key):
    names = list(rows)
    return sorted(zip(*[rows[c] for c in names]), key=lambda t: (t[0] is None, str(t[0])))


def _same(a, b):
    """Row lists equal, floats bitwise (NaN as NaN)."""
    assert len(a) == len(b)
    for x, y in zip(a, b):
        for u, v in zip(x, y):
            if isinstance(u, float) and isinstance(v, float):
                assert (np.isnan(u) and np.isnan(v)) or np.float64(u).view(np.uint64) == np.float64(v).view(np.uint64), (x, y)
            else:
                assert u == v, (x, y)


def test_two_rank_processes_real_kernels_over_gloo(gpu):
    import polaroid_amd as pl

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(WORLD):
        rank, out, err = q.get(timeout=240)
        assert err is None, err
        res[rank] = out
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # the single-GPU results on the concatenated shards (rank order = row order)
    parts = [_shard(r) for r in range(WORLD)]
    k, a, d, s, x = (np.concatenate([p[i] for p in parts]) for i in range(5))
    full = pl.DataFrame({"k": pl.Series.from_numpy("k", k), "a": pl.Series.from_numpy("a", a),
                         "d": pl.Series.from_numpy("d", d), "s": pl.Series("s", s.tolist(), pl.String),
                         "x": pl.Series.from_numpy("x", x)})
    pred = pl.col("d") > 0.0
    checks = {
        "states": full.lazy().filter(pred).group_by("k").agg(
            pl.col("a").sum().alias("sa"), pl.col("d").mean().alias("md"), pl.len().alias("n")).collect(),
        "wide": full.lazy().filter(pred).group_by("k").agg(
            pl.col("x").sum().alias("sx"), pl.col("x").mean().alias("mx"), pl.col("a").sum().alias("sa")).collect(),
        "shuffle": full.lazy().filter(pred).group_by("s").agg(
            pl.col("a").sum().alias("sa"), pl.col("d").first().alias("fd"), pl.col("d").last().alias("ld")).collect(),
        "first_last": full.lazy().group_by("k").agg(pl.col("d").first().alias("fd"),
                                                    pl.col("d").last().alias("ld")).collect(),
    }
    cols = {"states": ["k", "sa", "md", "n"], "wide": ["k", "sx", "mx", "sa"], "shuffle": ["s", "sa", "fd", "ld"],
            "first_last": ["k", "fd", "ld"]}
    for name, ref in checks.items():
        union = {c: [] for c in cols[name]}
        seen = set()
        for r in range(WORLD):
            rows, _ = res[r][name]
            keyc = cols[name][0]
            assert not (set(rows[keyc]) & seen), name  # each group on one rank
            seen |= set(rows[keyc])
            for c in cols[name]:
                union[c] += rows[c]
        _same(_canon(union, cols[name][0]), _canon(_rows(ref, cols[name]), cols[name][0]))
    assert res[0]["shuffle"][1] == "row_shuffle"
    # the wide column kept the partial-state protocol on both ranks, as digit
    # records of the agreed range; exchange bytes = records x record size
    for r in range(WORLD):
        proto, nwide, rwords, xbytes, groups = res[r]["wide"][1]
        assert proto == "partial_states" and nwide == 1, res[r]["wide"][1]
        assert rwords == res[0]["wide"][1][2] and rwords > 20
        assert 0 < xbytes <= 2 * 400 * rwords * 8
    # join: every probe row of either shard against the union of the right
    # sides (the rows each rank holds), as a multiset
    def order(t):  # a total order with NaN payloads
        return (t[0], bool(np.isnan(t[1])), 0.0 if np.isnan(t[1]) else t[1], t[2])

    got = sorted((t for r in range(WORLD) for t in zip(*[res[r]["join"][0][c] for c in ("k", "a", "w")])), key=order)
    k, a = (np.concatenate([_shard(r)[i] for r in range(WORLD)]) for i in (0, 1))
    rk = np.concatenate([np.arange(150) * 2 * 7919 - 1000 for _ in range(WORLD)])
    rw = np.concatenate([np.arange(150, dtype=np.float64) + r * 1000 for r in range(WORLD)])
    want = []
    idx = {}
    for j, key in enumerate(rk.tolist()):
        idx.setdefault(key, []).append(rw[j])
    for key, val in zip(k.tolist(), a.tolist()):
        for w in idx.get(key, []):
            want.append((key, val, w))
    want.sort(key=order)
    assert len(got) == len(want)
    _same(got, want)
    assert res[0]["join"][1] == "shuffle"
