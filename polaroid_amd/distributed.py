"""Hash-partitioned multi-GPU group-by: one process per GPU, RCCL all-to-all.

The reference's streaming group-by sink (polars-stream/src/nodes/group_by.rs)
pre-aggregates morsels in thread-local tables, splits the pre-aggregates by a
`HashPartitioner` (group_by.rs:85 `add_pre_agg`, :509) and folds each
partition's share with `combine_subset` (group_by.rs:378) in
`combine_locals` (group_by.rs:216).  Here the "locals" are GPUs:

1. every rank filters + pre-aggregates its own shard in HBM
   (`plgpu_gb_partial_begin`, the same fused kernel as the single-GPU path);
   f64 sums are exact 192-bit fixed-point states, so ranks first agree on
   the fixed-point windows (element-wise MAX all-reduce, a re-run only on a
   rank whose windows moved);
2. the partial groups are written as records grouped by destination rank
   (`plgpu_gb_partial_export`), record counts go through one all-to-all and
   the records through a second one (`torch.distributed.all_to_all_single`,
   RCCL over xGMI on MI355X);
3. each rank folds what it received into its partition and finalizes it
   (`plgpu_gb_merge`), returning a DataFrame of the groups it owns.

The only data-path collective is the record exchange, whose volume is
groups x record size (independent of the row count), so the per-rank work
stays the local HBM pass: weak scaling.
"""

from __future__ import annotations

import ctypes as C
from typing import Any, Sequence

from . import _native as N
from .expr import Expr

MAX_WINDOW_ROUNDS = 4


def _device_for(group) -> Any:
    import torch
    import torch.distributed as dist

    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def _allreduce_max(vals: Sequence[int], group, device) -> list[int]:
    import torch
    import torch.distributed as dist

    t = torch.tensor(list(vals), dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return [int(v) for v in t.tolist()]


def exchange_records(send, counts: Sequence[int], record_words: int, group=None):
    """All-to-all of records grouped by destination rank.  `send` is a flat
    int64 tensor of sum(counts) * record_words words; returns (recv, n)."""
    import torch
    import torch.distributed as dist

    device = send.device
    sc = torch.tensor(list(counts), dtype=torch.int64, device=device)
    rc = torch.empty_like(sc)
    dist.all_to_all_single(rc, sc, group=group)
    rcounts = [int(v) for v in rc.tolist()]
    recv = torch.empty(sum(rcounts) * record_words, dtype=torch.int64, device=device)
    dist.all_to_all_single(recv, send, output_split_sizes=[c * record_words for c in rcounts],
                           input_split_sizes=[c * record_words for c in counts], group=group)
    return recv, sum(rcounts)


def agree_windows(part, world: int, group, device) -> list[int]:
    """Run the partial stage until every rank used the same windows.

    `part.begin(bottoms)` returns (used, refit, hint); bottoms None = the
    shard's sampled windows.  Returns the agreed windows."""
    used, refit, hint = part.begin(None)
    for _ in range(MAX_WINDOW_ROUNDS):
        agreed = _allreduce_max(list(hint), group, device)
        need = int(list(used) != agreed)
        if _allreduce_max([need], group, device)[0] == 0:
            return agreed
        if need:
            used, refit, hint = part.begin(agreed)
    raise N.ComputeError("multi-GPU group-by: fixed-point windows did not converge")


class GpuPartial:
    """One rank's partial aggregation through the C-ABI."""

    def __init__(self, g, world: int):
        self.g = g
        self.world = world
        self.handle = C.c_void_p()
        self.nrec = 0
        self.bottoms = (C.c_int32 * N.GB_MAX_ACC)()
        self.info = N.GroupByInfo()
        w = C.c_int32(0)
        N.check(N.lib().plgpu_gb_record_words(g.cols, g.ncols, g.aggs, g.naggs, C.byref(w)))
        self.record_words = int(w.value)

    def free(self) -> None:
        if self.handle.value:
            N.lib().plgpu_gb_partial_free(self.handle)
            self.handle = C.c_void_p()

    def __del__(self):
        if N is not None and N._lib is not None:  # not during interpreter shutdown
            self.free()

    def begin(self, bottoms):
        self.free()
        g = self.g
        arg = None
        if bottoms is not None:
            arg = (C.c_int32 * N.GB_MAX_ACC)(*bottoms)
        nrec = C.c_int64(0)
        refit = C.c_int32(0)
        hint = (C.c_int32 * N.GB_MAX_ACC)()
        N.check(N.lib().plgpu_gb_partial_begin(C.byref(g.keycol), g.cols, g.ncols, g.prog, g.n_instr, g.aggs,
                                               g.naggs, arg, self.world, C.byref(self.handle), C.byref(nrec),
                                               self.bottoms, C.byref(refit), hint, C.byref(self.info), None))
        self.nrec = int(nrec.value)
        return list(self.bottoms), bool(refit.value), list(hint)

    def export(self):
        """-> (flat int64 CUDA tensor of records grouped by rank, counts)."""
        import torch

        send = torch.empty(self.nrec * self.record_words, dtype=torch.int64,
                           device=torch.device("cuda", torch.cuda.current_device()))
        counts = (C.c_int64 * self.world)()
        N.check(N.lib().plgpu_gb_partial_export(self.handle, send.data_ptr() if self.nrec else None, counts,
                                                None))
        self.free()
        return send, [int(c) for c in counts]

    def merge(self, recv, n: int, bottoms):
        from .frame import _gb_frame

        g = self.g
        b = (C.c_int32 * N.GB_MAX_ACC)(*bottoms)
        out_key = N.Column()
        out_aggs = (N.Column * max(1, g.naggs))()
        mi = N.GroupByInfo()
        N.check(N.lib().plgpu_gb_merge(recv.data_ptr() if n else None, n, g.cols, g.ncols, g.aggs, g.naggs, b,
                                       g.keycol.dtype, C.byref(out_key), out_aggs, C.byref(mi), None))
        return _gb_frame(g, out_key, out_aggs), mi


def run_partitioned(part, world: int, group, device):
    """The protocol of group_by_agg over any partial implementation (the
    GPU one above, or a host model in tests/test_distributed.py)."""
    bottoms = agree_windows(part, world, group, device)
    send, counts = part.export()
    recv, n = exchange_records(send, counts, part.record_words, group)
    return part.merge(recv, n, bottoms)


def group_by_agg(df, key: str, aggs: Sequence[Expr], predicate: Expr | None = None, *, group=None,
                 info: dict | None = None):
    """`df.lazy().filter(predicate).group_by(key).agg(*aggs)` over the shards
    held by all ranks of `group`.  Returns this rank's partition of the
    result (the groups whose key hashes to this rank; the null-key and
    INT64_MIN groups live on rank 0).  Group order is unspecified, as in the
    reference without maintain_order."""
    import torch
    import torch.distributed as dist

    from .frame import _gb_lower
    from .expr import col

    if not dist.is_initialized():
        raise N.InvalidOperationError("torch.distributed is not initialised")
    world = dist.get_world_size(group)
    device = _device_for(group)
    if device.type != "cuda":
        raise N.InvalidOperationError("the GPU group-by needs the nccl (RCCL) backend")
    aggs = [a if isinstance(a, Expr) else col(a) for a in aggs]
    g = _gb_lower(df, key, list(aggs), predicate)
    if g.keycol.dtype not in (N.I64, N.I32) or len(g.keys) != 1:
        raise N.InvalidOperationError("the multi-GPU group-by takes one Int64 / Int32 key column")
    part = GpuPartial(g, world)
    out, mi = run_partitioned(part, world, group, device)
    torch.cuda.synchronize()
    if info is not None:
        d = part.info.as_dict()
        d["merge_groups"] = mi.groups
        d["groups"] = mi.groups
        info.update(d)
    return out
