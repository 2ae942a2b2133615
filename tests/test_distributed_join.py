"""The multi-GPU join protocol (polaroid_amd/distributed.py run_join,
exchange_columns, allgather_columns) on CPU: world_size 2 and 3 over gloo,
with a host model of the device operations (partition / pack / unpack /
local join) in place of the C-ABI (the GPU kernels are covered by
tests/test_gpu_distributed_join.py).

Checks, for the shuffle and the broadcast strategy: rows are routed by
destination rank (every key lands on exactly one rank in the shuffle), the
schema and nullability agreement makes ragged and null-free shards line up,
empty shards work, and the union of the ranks' results equals the
single-process inner join as a multiset of rows.
"""

import os
import socket
from collections import Counter

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from polaroid_amd import _native as N
from polaroid_amd import distributed as D


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class HostFrame:
    """name -> (dtype code, values ndarray, valid ndarray | None)."""

    def __init__(self, cols):
        self.cols = cols

    @property
    def height(self):
        return len(next(iter(self.cols.values()))[1]) if self.cols else 0

    def rows(self):
        names = list(self.cols)
        out = []
        for i in range(self.height):
            row = []
            for n in names:
                _, v, m = self.cols[n]
                row.append(None if (m is not None and not m[i]) else v[i].item())
            out.append(tuple(row))
        return out


_NP = {N.I64: np.int64, N.F64: np.float64, N.I32: np.int32, N.BOOL: np.uint8}


class HostOps:
    """Models GpuJoinOps over numpy (the routing function is any
    deterministic function of the key, as plgpu_hash_partition's is)."""

    @staticmethod
    def rows(df):
        return df.height

    @staticmethod
    def partition(df, keys, world, nulls_equal):
        n = df.height
        dest = np.zeros(n, dtype=np.int64)
        drop = np.zeros(n, dtype=bool)
        for k in keys:
            _, v, m = df.cols[k]
            dest = dest * 1000003 + v.astype(np.int64)
            if m is not None:
                drop |= ~m
        dest = np.abs(dest) % world
        if nulls_equal:
            dest[drop] = 0
            drop[:] = False
        rows = np.arange(n)[~drop]
        perm = rows[np.argsort(dest[~drop], kind="stable")]
        return perm, [int((dest[~drop] == r).sum()) for r in range(world)]

    @staticmethod
    def to_wire(df, perm=None):
        out = []
        for name, (dt, v, m) in df.cols.items():
            vv = v if perm is None else v[perm]
            if dt == N.F64:
                vv = vv.view(np.int64)
            mm = None if m is None else (m if perm is None else m[perm]).astype(np.uint8)
            out.append(D.WireColumn(name, dt, torch.from_numpy(np.ascontiguousarray(vv)),
                                    None if mm is None else torch.from_numpy(mm)))
        return out

    @staticmethod
    def from_wire(cols, n):
        res = {}
        for c in cols:
            v = c.values.numpy()
            if c.dtype == N.F64:
                v = v.view(np.float64)
            m = None if c.valid is None else c.valid.numpy().astype(bool)
            assert v.shape[0] == n
            res[c.name] = (c.dtype, v, m)
        return HostFrame(res)

    @staticmethod
    def local_join(left, right, lk, rk, suffix, nulls_equal, how="inner"):
        lk = [lk] if isinstance(lk, str) else list(lk)
        rk = [rk] if isinstance(rk, str) else list(rk)
        return _host_join(left, right, lk, rk, suffix, nulls_equal, how)


def _host_join(left, right, lk, rk, suffix, nulls_equal, how="inner"):
    """Rows of a join as the single-GPU executor lays them out (frame._join):
    semi / anti the left rows; otherwise the left columns (without the keys
    for a right join) and the right columns (without the keys unless full),
    None for a missing partner."""
    lrows, rrows = left.rows(), right.rows()
    ln, rn = list(left.cols), list(right.cols)
    li = [ln.index(k) for k in lk]
    ri = [rn.index(k) for k in rk]
    keep_l = [i for i, n in enumerate(ln) if not (how == "right" and n in lk)]
    keep_r = [i for i, n in enumerate(rn) if how == "full" or how == "right" or n not in rk]
    index = {}
    for j, r in enumerate(rrows):
        key = tuple(r[i] for i in ri)
        if None in key and not nulls_equal:
            continue
        index.setdefault(key, []).append(j)
    out = []
    matched = set()
    for lrow in lrows:
        key = tuple(lrow[i] for i in li)
        js = [] if (None in key and not nulls_equal) else index.get(key, [])
        if how == "semi":
            if js:
                out.append(lrow)
            continue
        if how == "anti":
            if not js:
                out.append(lrow)
            continue
        for j in js:
            matched.add(j)
            out.append(tuple(lrow[i] for i in keep_l) + tuple(rrows[j][i] for i in keep_r))
        if not js and how in ("left", "full"):
            out.append(tuple(lrow[i] for i in keep_l) + (None,) * len(keep_r))
    if how in ("right", "full"):
        for j, r in enumerate(rrows):
            if j not in matched:
                out.append((None,) * len(keep_l) + tuple(r[i] for i in keep_r))
    return out


def _shard(rank, world, side, n):
    rng = np.random.default_rng(1000 * world + 10 * rank + (side == "right"))
    if n == 0:
        k = np.zeros(0, dtype=np.int64)
    else:
        k = rng.integers(0, 40, n).astype(np.int64)
    kvalid = rng.random(n) > 0.1
    k2 = (k % 3).astype(np.int32)
    v = rng.standard_normal(n)
    # nulls only on rank 0's payload: the validity mask must still be agreed
    vvalid = (rng.random(n) > 0.2) if rank == 0 else None
    b = (rng.random(n) > 0.5).astype(np.uint8)
    name = "pv" if side == "left" else "bv"
    return HostFrame({"k": (N.I64, k, kvalid), "k2": (N.I32, k2, None), name: (N.F64, v, vvalid),
                      name + "_flag": (N.BOOL, b, None)})


def _worker(rank, world, port, strategy, keys, nulls_equal, sizes, q, how="inner"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        left = _shard(rank, world, "left", sizes[rank][0])
        right = _shard(rank, world, "right", sizes[rank][1])
        info = {}
        out = D.run_join(HostOps, left, right, keys, keys, "_right", nulls_equal, strategy, None,
                         torch.device("cpu"), info, how)
        # keys that landed here (shuffle: each key on one rank only)
        q.put((rank, out, info))
    finally:
        dist.destroy_process_group()


def _run(world, strategy, keys, nulls_equal, sizes, how="inner"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, strategy, keys, nulls_equal, sizes, q, how))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, out, info = q.get(timeout=180)
        res[rank] = (out, info)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def _concat(frames):
    cols = {}
    for name in frames[0].cols:
        dt = frames[0].cols[name][0]
        v = np.concatenate([f.cols[name][1] for f in frames])
        ms = [f.cols[name][2] for f in frames]
        m = None if all(x is None for x in ms) else np.concatenate(
            [x if x is not None else np.ones(f.height, bool) for x, f in zip(ms, frames)])
        cols[name] = (dt, v, m)
    return HostFrame(cols)


@pytest.mark.parametrize("world,strategy,keys,nulls_equal,sizes", [
    (2, "shuffle", ["k"], False, [(300, 200), (250, 180)]),
    (2, "shuffle", ["k", "k2"], True, [(300, 200), (0, 180)]),
    (3, "shuffle", ["k"], True, [(120, 90), (0, 0), (200, 50)]),
    (2, "broadcast", ["k"], False, [(300, 200), (250, 180)]),
    (3, "broadcast", ["k", "k2"], False, [(100, 40), (130, 0), (90, 70)]),
    (2, "auto", ["k"], False, [(50, 500), (60, 400)]),   # auto -> broadcast of the smaller (left) side
])
def test_join_protocol_gloo(world, strategy, keys, nulls_equal, sizes):
    res = _run(world, strategy, keys, nulls_equal, sizes)
    left = _concat([_shard(r, world, "left", sizes[r][0]) for r in range(world)])
    right = _concat([_shard(r, world, "right", sizes[r][1]) for r in range(world)])
    expect = _host_join(left, right, keys, keys, "_right", nulls_equal)
    got = [row for r in range(world) for row in res[r][0]]
    assert Counter(got) == Counter(expect)
    assert len(expect) > 0
    used = res[0][1]["strategy"]
    assert all(res[r][1]["strategy"] == used for r in range(world))
    if strategy == "auto":
        assert used == "broadcast"
    if used == "shuffle":
        # every join key appears on exactly one rank
        seen = {}
        for r in range(world):
            for row in res[r][0]:
                kt = tuple(row[i] for i in range(len(keys)))
                assert seen.setdefault(kt, r) == r


@pytest.mark.parametrize("world,strategy,how,nulls_equal", [
    (2, "shuffle", "left", True), (3, "shuffle", "full", False), (2, "shuffle", "anti", False),
    (2, "broadcast", "right", False), (3, "broadcast", "anti", False), (2, "auto", "semi", False),
])
def test_join_types_protocol_gloo(world, strategy, how, nulls_equal):
    """Every join type over the multi-rank protocol: the union of the ranks'
    results equals the join of the concatenated shards (null-key rows of a
    kept side are routed, not dropped; only the allowed side broadcasts)."""
    sizes = [(200, 150), (180, 120), (90, 60)][:world]
    res = _run(world, strategy, ["k"], nulls_equal, sizes, how)
    left = _concat([_shard(r, world, "left", sizes[r][0]) for r in range(world)])
    right = _concat([_shard(r, world, "right", sizes[r][1]) for r in range(world)])
    expect = _host_join(left, right, ["k"], ["k"], "_right", nulls_equal, how)
    got = [row for r in range(world) for row in res[r][0]]
    assert Counter(got) == Counter(expect) and len(expect) > 0
    used = res[0][1]["strategy"]
    if how == "full":
        assert used == "shuffle"


def test_full_join_cannot_broadcast():
    """In-process world of one: a full join refuses to broadcast."""
    dist.init_process_group("gloo", rank=0, world_size=1, init_method=f"tcp://127.0.0.1:{_free_port()}")
    try:
        f = _shard(0, 1, "left", 10)
        g = _shard(0, 1, "right", 10)
        with pytest.raises(ValueError, match="full join"):
            D.run_join(HostOps, f, g, ["k"], ["k"], "_right", False, "broadcast", None, torch.device("cpu"), None,
                       "full")
        assert D.run_join(HostOps, f, g, ["k"], ["k"], "_right", False, "auto", None, torch.device("cpu"), None,
                          "full") == _host_join(f, g, ["k"], ["k"], "_right", False, "full")
    finally:
        dist.destroy_process_group()


def _a2a_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(rank)
        splits = [int(x) for x in rng.integers(0, 40, world)]
        splits[(rank + 1) % world] = 0  # an empty segment
        inp = torch.arange(sum(splits), dtype=torch.int64) + 1000 * rank
        sc = torch.tensor(splits, dtype=torch.int64)
        rc = torch.empty_like(sc)
        dist.all_to_all_single(rc, sc)
        rsplits = [int(v) for v in rc.tolist()]
        direct = torch.empty(sum(rsplits), dtype=torch.int64)
        dist.all_to_all_single(direct, inp, output_split_sizes=rsplits, input_split_sizes=splits)
        D.A2A_MAX_BYTES = 64  # 8 int64 per peer and round: many rounds
        chunked = torch.full((sum(rsplits),), -1, dtype=torch.int64)
        D.alltoallv(chunked, inp, rsplits, splits)
        q.put((rank, torch.equal(direct, chunked), sum(rsplits)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_alltoallv_rounds_gloo(world):
    """The round-wise point-to-point all-to-all (used above A2A_MAX_BYTES per
    peer) delivers exactly what all_to_all_single does."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_a2a_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, _ in res)
    assert sum(n for _, _, n in res) > 0
