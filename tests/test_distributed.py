"""The multi-GPU group-by protocol (polaroid_amd/distributed.py) on CPU:
world_size 2 over gloo, with a host model of the partial stage in place of
the GPU kernels (those are covered by tests/test_gpu_distributed.py).

Checks: every rank ends on the same fixed-point windows (including a round
where one rank must refit and the others re-run), records are routed by
destination rank with one all-to-all of counts and one of records, each
group lands on exactly one rank, and the union of the partitions equals the
single-process aggregation.
"""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from polaroid_amd import distributed as D

WORLD = 2
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


class HostPartial:
    """Models GpuPartial: begin / export / merge over numpy."""

    record_words = RW

    def __init__(self, rank, world, keys, vals, refit_rank):
        self.rank, self.world = rank, world
        self.keys, self.vals = keys, vals
        self.refit_rank = refit_rank
        self.begins = []
        self.groups = None

    def begin(self, bottoms):
        used = list(bottoms) if bottoms is not None else [10 * self.rank + 1, -3, 0, 0, 0, 0]
        self.begins.append(used)
        ks, inv = np.unique(self.keys, return_inverse=True)
        self.groups = (ks, np.array([self.vals[inv == i].sum() for i in range(len(ks))], dtype=np.int64))
        if self.rank == self.refit_rank and len(self.begins) == 1:
            hint = [u + 50 for u in used]   # "overflow": the window must move up
            return used, True, hint
        return used, False, used

    def export(self):
        ks, sums = self.groups
        dest = ks % self.world
        order = np.argsort(dest, kind="stable")
        rec = np.stack([np.zeros_like(ks), ks, sums], axis=1)[order].reshape(-1)
        counts = [int((dest == r).sum()) for r in range(self.world)]
        return torch.from_numpy(rec.copy()), counts

    def merge(self, recv, n, bottoms):
        r = recv.numpy().reshape(n, RW)
        out = {}
        for _, k, s in r:
            out[int(k)] = out.get(int(k), 0) + int(s)
        return (out, list(bottoms)), None


def _worker(rank, port, refit_rank, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        keys, vals = _shard(rank)
        part = HostPartial(rank, WORLD, keys, vals, refit_rank)
        (out, bottoms), _ = D.run_partitioned(part, WORLD, None, torch.device("cpu"))
        # exchange_records on its own: ragged counts including empty segments
        rw = 2
        counts = [0, 3] if rank == 0 else [5, 0]
        send = torch.arange(sum(counts) * rw, dtype=torch.int64) + 1000 * rank
        recv, nrec = D.exchange_records(send, counts, rw)
        q.put((rank, out, bottoms, part.begins, recv.tolist(), nrec))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("refit_rank", [-1, 0, 1])
def test_partitioned_group_by_protocol_gloo(refit_rank):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, refit_rank, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(WORLD):
        rank, out, bottoms, begins, recv, nrec = q.get(timeout=120)
        res[rank] = (out, bottoms, begins, recv, nrec)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # same windows everywhere, and they are the MAX over the ranks' hints
    b0, b1 = res[0][1], res[1][1]
    assert b0 == b1
    sampled = [[10 * r + 1, -3, 0, 0, 0, 0] for r in range(WORLD)]
    expect = [max(s[i] for s in sampled) for i in range(6)]
    if refit_rank >= 0:
        expect = [max(e, s + 50) for e, s in zip(expect, sampled[refit_rank])]
    assert b0 == expect
    # the partial that was merged ran with the agreed windows
    for r in range(WORLD):
        assert res[r][2][-1] == expect
    # partitions are disjoint and their union is the full aggregation
    k0, k1 = set(res[0][0]), set(res[1][0])
    assert not (k0 & k1)
    full = {}
    for r in range(WORLD):
        keys, vals = _shard(r)
        for k, v in zip(keys.tolist(), vals.tolist()):
            full[k] = full.get(k, 0) + v
    merged = dict(res[0][0])
    merged.update(res[1][0])
    assert merged == full
    for r in range(WORLD):
        assert all(k % WORLD == r for k in res[r][0])
    # ragged exchange: rank 0 receives rank1's 5 records, rank 1 receives rank0's 3
    assert res[0][4] == 5 and res[0][3] == list(range(1000, 1010))
    assert res[1][4] == 3 and res[1][3] == list(range(0, 6))
