"""The multi-GPU group-by protocol (polaroid_amd/distributed.py) on CPU:
world_size 2, and 8 (configs[4]'s rank count), over gloo, with a host model
of the partial stage in place of the GPU kernels (those are covered by
tests/test_gpu_distributed.py).

Checks: the partial stage runs without a collective, each rank's windows
travel with its record counts (one all-to-all of counts + header, one of
records), every destination receives every source's windows in source
order, each group lands on exactly one rank, the union of the partitions
equals the single-process aggregation, and a partial stage that fails on one
rank makes every rank raise instead of hanging in a collective.
"""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from polaroid_amd import distributed as D

RW = 3  # record: [kind, key, sum]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _shard(rank, n=5000, groups=97):
    rng = np.random.default_rng(100 + rank)
    keys = rng.integers(0, groups, n).astype(np.int64) * 7919 - 300
    vals = rng.integers(-10**9, 10**9, n).astype(np.int64)
    return keys, vals


def _bottoms(rank):
    return [10 * rank + 1, -3, 0, 0, 0, rank]


class HostPartial:
    """Models GpuPartial: begin / export / merge over numpy."""

    record_words = RW

    def __init__(self, rank, world, keys, vals, fail_rank):
        self.rank, self.world = rank, world
        self.keys, self.vals = keys, vals
        self.fail_rank = fail_rank
        self.groups = None

    def begin(self):
        if self.rank == self.fail_rank:
            raise D.N.ComputeError("refused on this rank")
        ks, inv = np.unique(self.keys, return_inverse=True)
        self.groups = (ks, np.array([self.vals[inv == i].sum() for i in range(len(ks))], dtype=np.int64))
        return _bottoms(self.rank)

    def export(self):
        ks, sums = self.groups
        dest = ks % self.world
        order = np.argsort(dest, kind="stable")
        rec = np.stack([np.zeros_like(ks), ks, sums], axis=1)[order].reshape(-1)
        counts = [int((dest == r).sum()) for r in range(self.world)]
        return torch.from_numpy(rec.copy()), counts

    def merge(self, recv, src_counts, src_bottoms):
        n = sum(src_counts)
        r = recv.numpy().reshape(n, RW)
        out = {}
        for _, k, s in r:
            out[int(k)] = out.get(int(k), 0) + int(s)
        return (out, list(src_counts), [list(b) for b in src_bottoms]), None


def _worker(rank, world, port, fail_rank, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        keys, vals = _shard(rank)
        part = HostPartial(rank, world, keys, vals, fail_rank)
        try:
            (out, src_counts, src_bottoms), _ = D.run_partitioned(part, world, None, torch.device("cpu"))
            err = None
        except D.N.PolaroidError as e:
            out, src_counts, src_bottoms, err = None, None, None, type(e).__name__ + ": " + str(e)
        # exchange_records on its own: ragged counts including empty
        # segments (rank r sends r + 3 records to rank r + 1 and none to the
        # others; at world 2: [0, 3] and [4, 0])
        rw = 2
        counts = [0] * world
        counts[(rank + 1) % world] = rank + 3
        send = torch.arange(sum(counts) * rw, dtype=torch.int64) + 1000 * rank
        recv, nrec, rows = D.exchange_records(send, counts, rw, header=[7, rank])
        q.put((rank, out, src_counts, src_bottoms, err, recv.tolist(), nrec, rows))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,fail_rank", [(2, -1), (2, 0), (2, 1), (8, -1), (8, 5)])
def test_partitioned_group_by_protocol_gloo(world, fail_rank):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fail_rank, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, out, src_counts, src_bottoms, err, recv, nrec, rows = q.get(timeout=180)
        res[rank] = (out, src_counts, src_bottoms, err, recv, nrec, rows)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # ragged exchange: rank r receives the r + 2 records of rank r - 1 (mod
    # world); every destination gets [count] + each source's header, in
    # source order
    for r in range(world):
        src = (r - 1) % world
        nsrc = src + 3
        assert res[r][5] == nsrc
        assert res[r][4] == [1000 * src + i for i in range(nsrc * 2)]
        assert res[r][6] == [[nsrc if q == src else 0, 7, q] for q in range(world)]
    if fail_rank >= 0:
        # the failing rank re-raises its own error, the others name it
        assert "refused on this rank" in res[fail_rank][3]
        for other in range(world):
            if other != fail_rank:
                assert res[other][3].startswith("ComputeError") and f"[{fail_rank}]" in res[other][3]
        return
    # every destination received each source's own windows, in rank order
    for r in range(world):
        assert res[r][3] is None
        assert res[r][2] == [_bottoms(q) for q in range(world)]
        assert len(res[r][0]) <= sum(res[r][1]) <= world * len(res[r][0])
    # partitions are disjoint and their union is the full aggregation
    seen = set()
    merged = {}
    for r in range(world):
        ks = set(res[r][0])
        assert not (ks & seen)
        seen |= ks
        merged.update(res[r][0])
        assert all(k % world == r for k in res[r][0])
    full = {}
    for r in range(world):
        keys, vals = _shard(r)
        for k, v in zip(keys.tolist(), vals.tolist()):
            full[k] = full.get(k, 0) + v
    assert merged == full


# ------------------------------------------- wide f64 sums: one agreed digit range
def _wide_report(rank):
    """(wide, exmin, exmax) a rank reports for its 6 accs: acc 0 is wide on
    odd ranks only (its range differs per rank), acc 1 a plain f64 sum, the
    rest not f64 sums (0x7FF / 0)."""
    w = [rank % 2, 0, 0, 0, 0, 0]
    lo = [100 + 7 * rank, 1000 - rank, 0x7FF, 0x7FF, 0x7FF, 0x7FF]
    hi = [1900 - 5 * rank, 1060 + rank, 0, 0, 0, 0]
    return w, lo, hi


class HostWidePartial(HostPartial):
    """HostPartial with the wide-sum agreement: records grow by the digit
    words once set_wide runs (here two words: the agreed range's ends)."""

    def __init__(self, *a):
        super().__init__(*a)
        self.agreed = None

    def wide_info(self):
        return _wide_report(self.rank)

    def set_wide(self, wide, exmin, exmax):
        self.agreed = (list(wide), list(exmin), list(exmax))
        self.record_words = RW + 2

    def export(self):
        ks, sums = self.groups
        dest = ks % self.world
        order = np.argsort(dest, kind="stable")
        lo, hi = self.agreed[1][0], self.agreed[2][0]
        rec = np.stack([np.zeros_like(ks), ks, sums, np.full_like(ks, lo), np.full_like(ks, hi)], axis=1)
        return torch.from_numpy(rec[order].reshape(-1).copy()), [int((dest == r).sum()) for r in range(self.world)]

    def merge(self, recv, src_counts, src_bottoms):
        n = sum(src_counts)
        r = recv.numpy().reshape(n, RW + 2)
        out = {}
        for _, k, v, lo, hi in r:
            assert (lo, hi) == (self.agreed[1][0], self.agreed[2][0])
            out[int(k)] = out.get(int(k), 0) + int(v)
        return (out, self.agreed, self.record_words), None


def _wide_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        keys, vals = _shard(rank)
        part = HostWidePartial(rank, world, keys, vals, -1)
        timings = {}
        (out, agreed, rw), _ = D.run_partitioned(part, world, None, torch.device("cpu"), timings)
        q.put((rank, out, agreed, rw, timings["wide_accs"], timings["record_words"]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_wide_sum_agreement_gloo(world):
    """A column wide on some ranks only: one all-reduce gives every rank the
    same wide flags and the union of the ranks' exponent ranges, every rank
    switches to the digit records (record words grow alike), and the
    partitions still add up to the full aggregation."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_wide_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, out, agreed, rw, nwide, rwords = q.get(timeout=180)
        res[rank] = (out, agreed, rw, nwide, rwords)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    reps = [_wide_report(r) for r in range(world)]
    want = ([max(r[0][a] for r in reps) for a in range(6)], [min(r[1][a] for r in reps) for a in range(6)],
            [max(r[2][a] for r in reps) for a in range(6)])
    merged, full = {}, {}
    for r in range(world):
        out, agreed, rw, nwide, rwords = res[r]
        assert agreed == want and rw == RW + 2 and nwide == 1 and rwords == RW + 2
        merged.update(out)
    for r in range(world):
        keys, vals = _shard(r)
        for k, v in zip(keys.tolist(), vals.tolist()):
            full[k] = full.get(k, 0) + v
    assert merged == full


# ------------------------------------------------- first() / last() across ranks
def _fl_shard(rank, n=400):
    """Rows of rank `rank` (rank order = row order): key, nullable key, and a
    nullable value that records its global position."""
    rng = np.random.default_rng(700 + rank)
    keys = rng.integers(0, 37, n).astype(np.int64) - 5
    kvalid = rng.random(n) > 0.05
    vals = np.arange(n, dtype=np.int64) + rank * 1_000_000
    vvalid = rng.random(n) > 0.2
    return keys, kvalid, vals, vvalid


def _first_last(keys, kvalid, vals, vvalid):
    """{(key valid, key): ((first value or None), (last value or None))}."""
    out = {}
    for k, kv, v, vv in zip(keys.tolist(), kvalid.tolist(), vals.tolist(), vvalid.tolist()):
        g = (bool(kv), k if kv else 0)
        x = v if vv else None
        out[g] = (out[g][0], x) if g in out else (x, x)
    return out


class HostFirstLastOps:
    """Models GpuFirstLastOps over numpy: route by key % world (the null key
    to rank 0), wire columns as CPU tensors, combine = first / last row per
    key in arrival order."""

    def route(self, local, world):
        ks = sorted(local)
        dest = [0 if not kv else k % world for kv, k in ks]
        perm = [ks[i] for i in np.argsort(dest, kind="stable")]
        return perm, [dest.count(r) for r in range(world)]

    def to_wire(self, local, perm):
        kv = torch.tensor([int(kv) for kv, _ in perm], dtype=torch.uint8)
        k = torch.tensor([k for _, k in perm], dtype=torch.int64)
        cols = [D.WireColumn("k", D.N.I64, k, kv)]
        for j, nm in enumerate(("first", "last")):
            v = [local[g][j] for g in perm]
            cols.append(D.WireColumn(nm, D.N.I64, torch.tensor([0 if x is None else x for x in v], dtype=torch.int64),
                                     torch.tensor([int(x is not None) for x in v], dtype=torch.uint8)))
        return cols

    def from_wire(self, cols, n):
        return [c.values.tolist() for c in cols], [c.valid.tolist() for c in cols], n

    def combine(self, rows):
        (k, f, l), (kv, fv, lv), n = rows
        out = {}
        for i in range(n):
            g = (bool(kv[i]), k[i] if kv[i] else 0)
            fx, lx = (f[i] if fv[i] else None), (l[i] if lv[i] else None)
            out[g] = (out[g][0], lx) if g in out else (fx, lx)
        return out


def _fl_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        local = _first_last(*_fl_shard(rank))
        q.put((rank, D.run_first_last(HostFirstLastOps(), local, world)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_first_last_protocol_gloo(world):
    """run_first_last: the owners' first / last over the per-rank results,
    received in source-rank order, equal first / last over the concatenated
    shards (nulls included); each group on exactly one rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fl_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    merged = {}
    for r in range(world):
        assert not (set(res[r]) & set(merged))
        assert all((not kv and r == 0) or (kv and k % world == r) for kv, k in res[r])
        merged.update(res[r])
    shards = [_fl_shard(r) for r in range(world)]
    full = _first_last(*[np.concatenate([s[i] for s in shards]) for i in range(4)])
    assert merged == full


def _fl_fail_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        def local():
            if rank == world - 1:
                raise RuntimeError("local first/last stage failed")
            return _first_last(*_fl_shard(rank))

        try:
            D.run_first_last(HostFirstLastOps(), local, world)
            q.put((rank, "no error"))
        except Exception as e:  # noqa: BLE001
            q.put((rank, type(e).__name__))
    finally:
        dist.destroy_process_group()


def test_first_last_failure_reaches_every_rank_gloo():
    """A rank whose local first / last stage fails: every rank raises (the
    status all-reduce before the exchange), none waits in a collective."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fl_fail_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[world - 1] == "RuntimeError"
    assert all(res[r] == "ComputeError" for r in range(world - 1))


# ------------------------------------------------ row-shuffle protocol
_STR = D.N.STR


class HostShuffleOps:
    """Models GpuShuffleOps over numpy: frames are {name: (dtype, values,
    valid)}; String columns are object arrays on the wire as byte lengths +
    UTF-8 bytes (the device wire format); the local group-by keeps first /
    last / sum / len per key in arrival order."""

    @staticmethod
    def select(df, predicate, names):
        assert predicate is None
        return {c: df[c] for c in names}

    @staticmethod
    def logical(df, names):
        return [None] * len(names)

    @staticmethod
    def restore(rows, names, logical):
        return rows

    @staticmethod
    def partition(df, keys, world, nulls_equal):
        n = len(next(iter(df.values()))[1])
        dest = np.zeros(n, dtype=np.int64)
        for k in keys:
            dt, v, m = df[k]
            h = np.array([sum(x.encode()) if dt == _STR else int(x) for x in v], dtype=np.int64)
            if m is not None:
                h[~m] = 0
            dest = dest * 1000003 + h
        dest = np.abs(dest) % world
        perm = np.argsort(dest, kind="stable")
        return perm, [int((dest == r).sum()) for r in range(world)]

    @staticmethod
    def to_wire(df, perm=None):
        out = []
        for name, (dt, v, m) in df.items():
            vv = v[perm]
            mm = None if m is None else torch.from_numpy(m[perm].astype(np.uint8))
            if dt == _STR:
                enc = [x.encode() for x in vv]
                lens = torch.tensor([len(b) for b in enc], dtype=torch.int64)
                data = torch.frombuffer(bytearray(b"".join(enc)) or bytearray(1), dtype=torch.uint8)[:int(lens.sum())]
                out.append(D.WireColumn(name, dt, lens, mm, data.clone()))
            else:
                out.append(D.WireColumn(name, dt, torch.from_numpy(np.ascontiguousarray(vv)), mm))
        return out

    @staticmethod
    def from_wire(cols, n):
        res = {}
        for c in cols:
            m = None if c.valid is None else c.valid.numpy().astype(bool)
            if c.dtype == _STR:
                lens = c.values.numpy()
                raw = bytes(c.data.numpy().tobytes())
                offs = np.concatenate([[0], np.cumsum(lens)])
                v = np.array([raw[offs[i]:offs[i + 1]].decode() for i in range(n)], dtype=object)
            else:
                v = c.values.numpy()
            assert v.shape[0] == n
            res[c.name] = (c.dtype, v, m)
        return res

    @staticmethod
    def local_group_by(rows, key, aggs):
        assert isinstance(key, str)
        _, kv, km = rows[key]
        out = {}
        for i in range(len(kv)):
            k = None if (km is not None and not km[i]) else kv[i]
            _, sv, _ = rows["s"]
            _, xv, _ = rows["x"]
            g = out.setdefault(k, [0, 0, None, None])
            g[0] += int(xv[i])
            g[1] += 1
            if g[2] is None:
                g[2] = sv[i]
            g[3] = sv[i]
        return out

    @staticmethod
    def rows(df):
        return len(df)


def _sh_shard(rank, n=300):
    rng = np.random.default_rng(rank + 11)
    pool = np.array([f"long-symbol-{i}" for i in range(40)] + ["", "é"], dtype=object)
    k = pool[rng.integers(0, pool.size, n)]
    km = rng.random(n) > 0.1
    s = np.array([f"r{rank}-row{i}" for i in range(n)], dtype=object)
    x = rng.integers(-100, 100, n).astype(np.int64)
    return {"k": (_STR, k, km), "s": (_STR, s, None), "x": (D.N.I64, x, None)}


def _sh_worker(rank, world, port, q, fail):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from polaroid_amd.expr import col

        class Ops(HostShuffleOps):
            @staticmethod
            def select(df, predicate, names):
                if fail and rank == 1:
                    raise RuntimeError("local stage failed")
                return HostShuffleOps.select(df, predicate, names)

        aggs = [col("x").sum(), col("s").first(), col("s").last()]
        try:
            out = D.run_shuffled(Ops, _sh_shard(rank), "k", aggs, None, None, torch.device("cpu"))
            q.put((rank, out))
        except Exception as e:  # noqa: BLE001
            q.put((rank, type(e).__name__))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_row_shuffle_protocol_gloo(world):
    """run_shuffled: String keys and payloads cross the wire as lengths +
    bytes, every key lands on exactly one rank, the sources arrive in rank
    order (first / last over the concatenated shards), and the union equals
    the single-process aggregation."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sh_worker, args=(r, world, port, q, False)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    merged = {}
    for r in range(world):
        assert not (set(res[r]) & set(merged))
        merged.update(res[r])
    full = {}
    for r in range(world):
        sh = _sh_shard(r)
        _, kv, km = sh["k"]
        for i in range(len(kv)):
            k = kv[i] if km[i] else None
            g = full.setdefault(k, [0, 0, None, None])
            g[0] += int(sh["x"][1][i])
            g[1] += 1
            if g[2] is None:
                g[2] = sh["s"][1][i]
            g[3] = sh["s"][1][i]
    assert merged == full
    assert None in res[0]  # the null key routes to rank 0


def _agreed_worker(rank, world, port, q):
    """An aggregation input evaluated per shard (the stage _group_by_agg_states
    runs before its first collective): a strict cast that overflows only in
    rank 1's shard.  Afterwards every rank enters the next collective, which
    must not hang."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        shard = np.arange(10, dtype=np.int64) + (300 if rank == 1 else 0)

        def strict_cast_u8():
            if shard.max() > 255:
                raise D.N.InvalidOperationError("conversion from `i64` to `u8` failed in column 'x'")
            return shard.astype(np.uint8)

        try:
            D.agreed_stage(strict_cast_u8, None, torch.device("cpu"), "evaluating an aggregation input")
            res = "ok"
        except Exception as e:  # noqa: BLE001
            res = type(e).__name__
        # the next collective of the protocol: reached by every rank
        t = torch.tensor([rank], dtype=torch.int64)
        dist.all_reduce(t)
        q.put((rank, res, int(t.item())))
        # and a stage that succeeds everywhere returns its value
        assert D.agreed_stage(lambda: rank * 2, None, torch.device("cpu"), "x") == rank * 2
    finally:
        dist.destroy_process_group()


def test_aggregation_input_failure_on_one_rank_reaches_every_rank_gloo():
    """an expression input that fails on one rank's shard only
    makes every rank raise (the failing rank its own error), instead of the
    others waiting in the next collective."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_agreed_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: (s, t) for r, s, t in (q.get(timeout=180) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[1][0] == "InvalidOperationError"
    assert res[0][0] == "ComputeError" and res[2][0] == "ComputeError"
    assert all(t == 0 + 1 + 2 for _, t in res.values())


def test_row_shuffle_failure_reaches_every_rank_gloo():
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sh_worker, args=(r, world, port, q, True)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[1] == "RuntimeError"
    assert res[0] == "ComputeError" and res[2] == "ComputeError"
