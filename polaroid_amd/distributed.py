"""Hash-partitioned multi-GPU group-by: one process per GPU, RCCL all-to-all.

The reference's streaming group-by sink (polars-stream/src/nodes/group_by.rs)
pre-aggregates morsels in thread-local tables, splits the pre-aggregates by a
`HashPartitioner` (group_by.rs:85 `add_pre_agg`, :509) and folds each
partition's share with `combine_subset` (group_by.rs:378) in
`combine_locals` (group_by.rs:216).  Here the "locals" are GPUs:

1. every rank filters + pre-aggregates its own shard in HBM
   (`plgpu_gb_partial_begin`, the same fused kernel as the single-GPU path)
   with its own f64 fixed-point windows (exact 192-bit states; a window
   that does not fit the shard is refitted locally); one small all-reduce
   agrees the stage's status and, for an f64 sum whose values span more
   binades than one window on some rank, one digit range per column over
   which every rank keeps that column's exact per-group digit state;
2. the partial groups are written as records grouped by destination rank
   (`plgpu_gb_partial_export`); one all-to-all carries each destination's
   record count together with the sender's windows and status, a second
   one the records (`torch.distributed.all_to_all_single`, RCCL over xGMI
   on MI355X);
3. each rank shifts every source's sum states onto the lowest window
   (exact), folds them into its partition and finalizes it
   (`plgpu_gb_merge_sources`), returning a DataFrame of the groups it owns.

The only data-path collective is the record exchange, whose volume is
groups x record size (independent of the row count; a wide column adds its
digit words to every record), so the per-rank work stays the local HBM
pass: weak scaling.
"""

from __future__ import annotations

import os

import ctypes as C
import time
from typing import Any, Sequence

from . import _native as N
from .expr import Expr

class _RowShuffle(Exception):
    """This input takes the row-shuffle protocol (group_by_agg): raised at
    the same protocol point on every rank (a schema property, or a status
    agreed by a collective), never by one rank alone."""


def _device_for(group) -> Any:
    import torch
    import torch.distributed as dist

    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    # gloo on a process that owns a GPU (ranks sharing one device in a test):
    # device buffers, collectives staged through host memory (_staged)
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def _staged(group, *tensors) -> bool:
    """A gloo group over device tensors (ranks sharing one GPU in a test,
    or a host-only transport): the collective goes through host copies."""
    import torch.distributed as dist

    return dist.get_backend(group) == "gloo" and any(t is not None and t.is_cuda for t in tensors)


def _a2a(out, inp, out_splits=None, in_splits=None, group=None) -> None:
    """all_to_all_single on the group's transport (host-staged for gloo)."""
    import torch.distributed as dist

    kw = {} if out_splits is None else {"output_split_sizes": list(out_splits), "input_split_sizes": list(in_splits)}
    if _staged(group, out, inp):
        o = out.new_empty(out.shape, device="cpu")
        dist.all_to_all_single(o, inp.cpu(), group=group, **kw)
        out.copy_(o)
        return
    dist.all_to_all_single(out, inp, group=group, **kw)


def _all_gather(parts, t, group=None) -> None:
    """all_gather on the group's transport (host-staged for gloo)."""
    import torch.distributed as dist

    if _staged(group, t):
        hp = [p.new_empty(p.shape, device="cpu") for p in parts]
        dist.all_gather(hp, t.cpu(), group=group)
        for p, h in zip(parts, hp):
            p.copy_(h)
        return
    dist.all_gather(parts, t, group=group)


def _all_reduce(t, op, group=None) -> None:
    """all_reduce on the group's transport (host-staged for gloo)."""
    import torch.distributed as dist

    if _staged(group, t):
        h = t.cpu()
        dist.all_reduce(h, op=op, group=group)
        t.copy_(h)
        return
    dist.all_reduce(t, op=op, group=group)


def _allreduce_max(vals: Sequence[int], group, device) -> list[int]:
    import torch
    import torch.distributed as dist

    t = torch.tensor(list(vals), dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return [int(v) for v in t.tolist()]


def agreed_stage(fn, group, device, what: str):
    """Run a rank-local stage whose success can depend on this rank's shard
    (a strict cast that overflows on one shard only, an allocation a larger
    shard cannot get) and agree its outcome with one status all-reduce
    before any other collective: the failing rank re-raises its error, every
    other rank raises ComputeError, so no rank waits in a collective the
    failed one never reaches."""
    err = res = None
    try:
        res = fn()
    except Exception as e:  # noqa: BLE001 -- agreed below, then re-raised
        err = e
    failed = _allreduce_max([1 if err is not None else 0], group, device)[0]
    if err is not None:
        raise err
    if failed:
        raise N.ComputeError(f"multi-GPU group-by: {what} failed on another rank")
    return res


def _settle(device) -> None:
    """Host-wait for the received buffers.  RCCL writes them on its own
    (non-blocking) stream and a synchronous collective only orders torch's
    current stream after it; the library's kernels run on the HIP null
    stream, so without this wait they could read a buffer still being
    received."""
    import torch

    if device.type == "cuda":
        torch.cuda.current_stream(device).synchronize()


# Largest per-peer message of one all-to-all.  On this image's RCCL
# (2.26.6) all_to_all_single loses the second half of any message above
# 1 GiB: tools/repro_a2a_large.py (torch + RCCL only, world 1) gets 1 GiB
# right and 1.99 / 2 / 3 / 4 / 6 GiB wrong from element n/2 on
# (profiles/r02_a2a_repro.log), with the receive fence (_settle) in place
# (tools/check_shuffle_scale.py without rounds: profiles/
# r02_shuffle_no_rounds.log).  Bigger exchanges therefore go in rounds of
# point-to-point transfers of at most this many bytes per peer
# (PLGPU_A2A_MAX_BYTES overrides it for such checks).
A2A_MAX_BYTES = int(os.environ.get("PLGPU_A2A_MAX_BYTES", 1 << 30))


def alltoallv(out, inp, out_splits: Sequence[int], in_splits: Sequence[int], group=None) -> None:
    """all_to_all_single(out, inp, out_splits, in_splits), in rounds of at
    most A2A_MAX_BYTES per peer (views of the flat tensors, no copies)."""
    import torch.distributed as dist

    esz = inp.element_size()
    if max(list(out_splits) + list(in_splits) + [0]) * esz <= A2A_MAX_BYTES or _staged(group, out, inp):
        _a2a(out, inp, out_splits, in_splits, group)
        return
    world = dist.get_world_size(group)
    me = dist.get_rank(group)
    chunk = max(1, A2A_MAX_BYTES // esz)
    soff = [sum(in_splits[:p]) for p in range(world)]
    roff = [sum(out_splits[:p]) for p in range(world)]
    rounds = (max(list(out_splits) + list(in_splits)) + chunk - 1) // chunk
    for r in range(rounds):
        ops = []
        for p in range(world):
            s0, s1 = min(in_splits[p], r * chunk), min(in_splits[p], (r + 1) * chunk)
            r0, r1 = min(out_splits[p], r * chunk), min(out_splits[p], (r + 1) * chunk)
            if p == me:
                if s1 > s0:
                    out[roff[p] + r0: roff[p] + r1].copy_(inp[soff[p] + s0: soff[p] + s1])
                continue
            peer = p if group is None else dist.get_global_rank(group, p)
            if s1 > s0:
                ops.append(dist.P2POp(dist.isend, inp[soff[p] + s0: soff[p] + s1], peer, group))
            if r1 > r0:
                ops.append(dist.P2POp(dist.irecv, out[roff[p] + r0: roff[p] + r1], peer, group))
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()


def exchange_records(send, counts: Sequence[int], record_words: int, group=None, header: Sequence[int] = ()):
    """All-to-all of records grouped by destination rank.  `send` is a flat
    int64 tensor of sum(counts) * record_words words.  `header` (ints) goes
    to every destination with its count.  Returns (recv, n, rows): rows[q] =
    [records from rank q] + rank q's header, in source-rank order (the
    order of the records in `recv`)."""
    import torch
    import torch.distributed as dist

    device = send.device
    world = len(counts)
    h = len(header)
    sc = torch.tensor([[int(c)] + [int(x) for x in header] for c in counts], dtype=torch.int64, device=device)
    rc = torch.empty_like(sc)
    _a2a(rc, sc, group=group)
    rows = [[int(v) for v in r] for r in rc.view(world, 1 + h).tolist()]
    rcounts = [r[0] for r in rows]
    recv = torch.empty(sum(rcounts) * record_words, dtype=torch.int64, device=device)
    alltoallv(recv, send, [c * record_words for c in rcounts], [c * record_words for c in counts], group)
    _settle(device)
    return recv, sum(rcounts), rows


class GpuPartial:
    """One rank's partial aggregation through the C-ABI."""

    def __init__(self, g, world: int):
        self.g = g
        self.world = world
        self.handle = C.c_void_p()
        self.nrec = 0
        self.bottoms = (C.c_int32 * N.GB_MAX_ACC)()
        self.info = N.GroupByInfo()
        self.wide = None  # agreed (wide, exmin, exmax) when some column's states are digits
        w = C.c_int32(0)
        N.check(N.lib().plgpu_gb_record_words(g.cols, g.ncols, g.aggs, g.naggs, C.byref(w)))
        self.record_words = int(w.value)

    def free(self) -> None:
        if self.handle.value:
            N.lib().plgpu_gb_partial_free(self.handle)
            self.handle = C.c_void_p()

    def __del__(self):
        # at interpreter shutdown module globals may already be gone, and a
        # failed __init__ leaves no handle: nothing to free then
        try:
            if getattr(self, "handle", None) is not None and N._lib is not None:
                self.free()
        except (AttributeError, TypeError):
            pass

    def begin(self) -> list[int]:
        """Pre-aggregate the shard with its own windows; returns them."""
        self.free()
        g = self.g
        nrec = C.c_int64(0)
        refit = C.c_int32(0)
        hint = (C.c_int32 * N.GB_MAX_ACC)()
        N.check(N.lib().plgpu_gb_partial_begin(C.byref(g.keycol), g.cols, g.ncols, g.prog, g.n_instr, g.aggs,
                                               g.naggs, None, self.world, C.byref(self.handle), C.byref(nrec),
                                               self.bottoms, C.byref(refit), hint, C.byref(self.info), None))
        self.nrec = int(nrec.value)
        return list(self.bottoms)

    def wide_info(self):
        """-> (wide[a], exmin[a], exmax[a]): which f64 sums of this shard
        need digit states, and the biased exponents each f64 sum's values
        take (plgpu_gb_partial_wide)."""
        A = N.GB_MAX_ACC
        w, lo, hi = (C.c_int32 * A)(), (C.c_int32 * A)(), (C.c_int32 * A)()
        N.check(N.lib().plgpu_gb_partial_wide(self.handle, w, lo, hi))
        return list(w), list(lo), list(hi)

    def set_wide(self, wide, exmin, exmax) -> None:
        """Digit states over the ranks' agreed ranges for the columns in
        `wide`; the record grows by their digit words."""
        A = N.GB_MAX_ACC
        self.wide = ((C.c_int32 * A)(*wide), (C.c_int32 * A)(*exmin), (C.c_int32 * A)(*exmax))
        N.check(N.lib().plgpu_gb_partial_set_wide(self.handle, *self.wide))
        w = C.c_int32(0)
        N.check(N.lib().plgpu_gb_partial_record_words(self.handle, C.byref(w)))
        self.record_words = int(w.value)

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

    def merge(self, recv, src_counts: Sequence[int], src_bottoms: Sequence[Sequence[int]]):
        """Fold the records of every source rank (windows per source)."""
        from .frame import _gb_frame

        g = self.g
        ns = len(src_counts)
        cnt = (C.c_int64 * ns)(*src_counts)
        bot = (C.c_int32 * (ns * N.GB_MAX_ACC))(*[int(b) for row in src_bottoms for b in row])
        out_key = N.Column()
        out_aggs = (N.Column * max(1, g.naggs))()
        mi = N.GroupByInfo()
        rec = recv.data_ptr() if sum(src_counts) else None
        if self.wide is not None:
            N.check(N.lib().plgpu_gb_merge_sources_wide(rec, ns, cnt, bot, *self.wide, g.cols, g.ncols, g.aggs,
                                                        g.naggs, g.keycol.dtype, C.byref(out_key), out_aggs,
                                                        C.byref(mi), None))
        else:
            N.check(N.lib().plgpu_gb_merge_sources(rec, ns, cnt, bot, g.cols, g.ncols, g.aggs, g.naggs,
                                                   g.keycol.dtype, C.byref(out_key), out_aggs, C.byref(mi), None))
        return _gb_frame(g, out_key, out_aggs), mi


def _sync(device) -> None:
    if device.type == "cuda":
        import torch

        torch.cuda.synchronize(device)


def agree_wide(vals, world: int, rank: int, failed: bool, group, device):
    """One max all-reduce after the partial stage: per rank a failure flag,
    and per acc (wide, -exmin, exmax) from `vals` = part.wide_info() (None
    on a failed rank or a partial without f64 sums).  Returns (failed ranks,
    wide, exmin, exmax) over all ranks: a column is wide when it is on any
    rank, and its digit range is the union of every rank's exponent range."""
    A = N.GB_MAX_ACC
    flat = [0] * world + [0] * A + [-0x7FF] * A + [0] * A
    if failed:
        flat[rank] = 1
    elif vals is not None:
        w, lo, hi = vals
        flat[world:world + A] = [int(x) for x in w]
        flat[world + A:world + 2 * A] = [-int(x) for x in lo]
        flat[world + 2 * A:] = [int(x) for x in hi]
    red = flat if world == 1 else _allreduce_max(flat, group, device)  # one rank: nothing to agree
    return ([q for q in range(world) if red[q]], red[world:world + A],
            [-x for x in red[world + A:world + 2 * A]], red[world + 2 * A:])


def run_partitioned(part, world: int, group, device, timings: dict | None = None):
    """The protocol of group_by_agg over any partial implementation (the
    GPU one above, or a host model in tests/test_distributed.py).

    The partial stage runs with no collective.  Its outcome is agreed by one
    small all-reduce (agree_wide): a rank whose stage failed makes every
    rank raise instead of waiting in a collective, and an f64 sum wider than
    one fixed-point window on any rank turns that column's states into exact
    digit words over the union of the ranks' exponent ranges on every rank
    (part.set_wide), so the records still carry it (the single-GPU wide
    sum, bit-identical).  A failure in the export still reaches every rank
    through the count exchange (status 1, no records).  With `timings`, the
    wall time of each phase (device-synchronised) is stored as partial_ms
    (local pre-aggregation and the agreement), exchange_ms (export + the two
    all-to-alls), merge_ms, and wide_accs / record_words."""
    import torch.distributed as dist

    t0 = time.perf_counter()
    err = None
    bottoms = [0] * N.GB_MAX_ACC
    vals = None
    try:
        bottoms = part.begin()
        vals = part.wide_info() if hasattr(part, "wide_info") else None
    except Exception as e:  # noqa: BLE001 -- agreed below, then re-raised
        err = e
        bottoms = [0] * N.GB_MAX_ACC
    failed, wide, exmin, exmax = agree_wide(vals, world, dist.get_rank(group), err is not None, group, device)
    if err is not None:
        raise err
    if failed:
        raise N.ComputeError(f"multi-GPU group-by: the partial stage failed on rank(s) {failed}")
    send = counts = None
    try:
        if any(wide):
            part.set_wide(wide, exmin, exmax)
        if timings is not None:
            _sync(device)
        t1 = time.perf_counter()
        send, counts = part.export()
    except Exception as e:  # noqa: BLE001 -- any failure before the exchange:
        # the count exchange still runs, with the status and no records, so
        # every rank learns of it instead of waiting
        err = e
    if err is not None or send is None:
        import torch

        t1 = time.perf_counter()
        send, counts = torch.empty(0, dtype=torch.int64, device=device), [0] * world
    status = 0 if err is None else 1
    recv, n, rows = exchange_records(send, counts, part.record_words, group, header=[status] + list(bottoms))
    failed = [q for q, r in enumerate(rows) if r[1] == 1]
    if err is not None:
        raise err
    if failed:
        raise N.ComputeError(f"multi-GPU group-by: the export failed on rank(s) {failed}")
    t2 = time.perf_counter()
    res = part.merge(recv, [r[0] for r in rows], [r[2:] for r in rows])
    if timings is not None:
        _sync(device)
        t3 = time.perf_counter()
        timings.update(partial_ms=(t1 - t0) * 1e3, exchange_ms=(t2 - t1) * 1e3, merge_ms=(t3 - t2) * 1e3,
                       wide_accs=sum(1 for w in wide if w), record_words=part.record_words,
                       exchange_bytes=int(sum(counts)) * part.record_words * 8)
    return res


def run_first_last(ops, local, world: int, group=None):
    """first() / last() across ranks (reduce/first_last.rs: the value of the
    group's first / last selected row, nulls included).  The shards are the
    row order: rank r holds the rows after rank r-1's.  Each rank's
    single-GPU group-by gives `local` (key + its first / last values); its
    rows go to the rank owning their key's partial states (`ops.route`, the
    same partition function as the records), arrive in source-rank order
    (all-to-all), and the owner takes first() / last() over them
    (`ops.combine`): the lowest rank holding a group has its first row, the
    highest its last.  Returns this rank's (key + first / last) frame.

    `local` may be a callable producing that frame: a failure there or in
    the routing (on any rank) is agreed by one status all-reduce before the
    exchange, so every rank raises instead of waiting in a collective."""
    err = None
    wire = counts = None
    try:
        if callable(local):
            local = local()
        perm, counts = ops.route(local, world)
        wire = ops.to_wire(local, perm)
    except Exception as e:  # noqa: BLE001
        err = e
    failed = _allreduce_max([1 if err is not None else 0], group, _device_for(group))[0]
    if err is not None:
        raise err
    if failed:
        raise N.ComputeError("multi-GPU first() / last(): the local stage failed on another rank")
    recv, n = exchange_columns(wire, counts, group)
    return ops.combine(ops.from_wire(recv, n))


class GpuFirstLastOps:
    """The device half of run_first_last, through the C-ABI."""

    def __init__(self, key: str, exprs: Sequence[Expr]):
        self.key = key
        self.exprs = list(exprs)

    def route(self, local, world: int):
        from .frame import Series

        perm = N.Column()
        counts = (C.c_int64 * world)()
        N.check(N.lib().plgpu_gb_route(C.byref(local[self.key]._col), world, C.byref(perm), counts, None))
        return Series._from_native("__perm", perm), [int(c) for c in counts]

    @staticmethod
    def to_wire(local, perm):
        return GpuJoinOps.to_wire(local, perm)

    @staticmethod
    def from_wire(cols, n: int):
        return GpuJoinOps.from_wire(cols, n)

    def combine(self, rows):
        from .frame import _agg_base, _group_by
        from .expr import col

        out = []
        for e in self.exprs:
            nm = e.output_name()
            c = col(nm)
            out.append((c.first() if _agg_base(e).op == "first" else c.last()).alias(nm))
        return _group_by(rows, self.key, out, False, None, None)


def _first_last_split(aggs: Sequence[Expr]) -> list[int]:
    from .frame import _agg_base

    return [i for i, e in enumerate(aggs) if _agg_base(e).kind == "agg" and _agg_base(e).op in ("first", "last")]


_PACKABLE = (N.I64, N.I32, N.U32, N.I16, N.U16, N.I8, N.U8, N.BOOL)


def _pack_keys(df, keys: list, group, device):
    """Several integer / Boolean key columns -> one exact Int64 code column
    that every rank computes with the same plan (plgpu_key_ranges on each
    shard, reduced over the ranks, then plgpu_key_pack), so the single-key
    partitioned protocol groups tuples exactly (row_encode.rs:11 semantics:
    a null is its own value).  Returns (plan, frame with the code column,
    its name)."""
    import torch
    import torch.distributed as dist

    from .frame import DataFrame, Series, _col_array

    for k in keys:
        if k not in df.columns:
            raise N.ComputeError(f'unable to find column "{k}"')
        if df[k]._col.dtype not in _PACKABLE:
            raise _RowShuffle("a Float / String column in a key tuple")
    nk = len(keys)
    kcols = _col_array([df[k] for k in keys])
    r = (C.c_int64 * (3 * nk))()
    N.check(N.lib().plgpu_key_ranges(kcols, nk, r, None))
    t = torch.tensor(list(r), dtype=torch.int64, device=device).view(nk, 3)
    lo, hi = t[:, 0].contiguous(), t[:, 1:].contiguous()
    _all_reduce(lo, dist.ReduceOp.MIN, group)
    _all_reduce(hi, dist.ReduceOp.MAX, group)
    agreed = torch.cat([lo.view(nk, 1), hi], dim=1).view(-1).tolist()
    ranges = (C.c_int64 * (3 * nk))(*agreed)
    codes = N.Column()
    ok = C.c_int32(0)
    N.check(N.lib().plgpu_key_pack(kcols, nk, ranges, C.byref(codes), C.byref(ok), None))
    if not ok.value:  # the same agreed ranges on every rank: every rank switches
        raise _RowShuffle("key ranges need more than 63 bits")
    name = "__key"
    while name in df.columns:
        name += "_"
    plan = (keys, [df[k]._col.dtype for k in keys], [df[k]._logical_dtype() for k in keys], ranges)
    return plan, DataFrame(list(df._cols.values()) + [Series._from_native(name, codes)]), name


def _unpack_keys(out, code_name: str, plan, agg_names: list):
    """The code column of a result back into its key columns (first), then
    the aggregations."""
    from .frame import DataFrame, Series

    keys, dtypes, logical, ranges = plan
    nk = len(keys)
    res = (N.Column * nk)()
    N.check(N.lib().plgpu_key_unpack(C.byref(out[code_name]._col), (C.c_int32 * nk)(*dtypes), nk, ranges, res,
                                     None))
    return DataFrame([Series._from_native(k, res[i], logical[i]) for i, k in enumerate(keys)] +
                     [out[nm] for nm in agg_names])


def _group_by_var(df, key, aggs: Sequence[Expr], predicate, group, info: dict | None):
    """var() / std(ddof) across ranks (polars-expr/src/reduce/var_std.rs),
    composed like the single-GPU frame._group_by_var from exact passes:
      1. the multi-GPU group-by with each var / std column's mean and count
         next to the other aggregations (this rank's partition of groups);
      2. the owners' (key, mean) rows all-gathered, so every rank holds every
         group's mean (groups x 8 B per column, independent of rows);
      3. every local row's squared deviation from its group's mean
         (plgpu_group_sq_dev for one integer key, else a left join), exactly
         summed per group by a second multi-GPU group-by (same partitions);
      4. the second result aligned to the first on the key, then
         plgpu_var_finalize (null when count <= ddof; sqrt for std)."""
    from .expr import col
    from .frame import DataFrame, Series, String, _agg_base, _eval, _join, _lower_strings

    keys = [key] if isinstance(key, str) else list(key)
    key = keys[0] if len(keys) == 1 else tuple(keys)
    str_keys = []
    for k in keys:
        if k not in df.columns:
            raise N.ComputeError(f'unable to find column "{k}"')
        if df[k].dtype is String and len(keys) == 1:
            str_keys.append(k)
        elif df[k]._col.dtype not in _TORCH_WIRE:
            raise _RowShuffle("var / std with String keys in a tuple")
    if str_keys:
        # a short String key runs as its exact Int64 codes (the means cross
        # the all-gather as integers) and is decoded at the end
        if predicate is not None:
            predicate, df = _lower_strings(predicate, df)
        codes = N.Column()
        short = C.c_int32(0)
        N.check(N.lib().plgpu_str_encode_short(C.byref(df[key]._col), C.byref(codes), C.byref(short), None))
        if _allreduce_max([0 if short.value else 1], group, _device_for(group))[0]:
            raise _RowShuffle("String keys longer than 7 bytes")
        df = DataFrame([Series._from_native(key, codes) if nm == key else df[nm] for nm in df.columns])
        out = _group_by_var(df, key, aggs, predicate, group, info)
        strs = N.Column()
        N.check(N.lib().plgpu_str_decode_short(C.byref(out[key]._col), C.byref(strs), None))
        return DataFrame([Series._from_native(key, strs) if nm == key else out[nm] for nm in out.columns])
    var_cols: list[str] = []
    plain: list[Expr] = []
    for e in aggs:
        b = _agg_base(e)
        if b.kind == "agg" and b.op in ("std", "var"):
            if b.args[0].kind != "col":
                raise _RowShuffle("var / std of a computed expression")
            if b.args[0].value not in var_cols:
                var_cols.append(b.args[0].value)
        else:
            plain.append(e)
    helpers = []
    for c in var_cols:
        helpers += [col(c).mean().alias(f"__vm_{c}"), col(c).count().alias(f"__vn_{c}")]
    first = group_by_agg(df, key, plain + helpers, predicate, group=group, info=info)
    means = DataFrame([first[k] for k in keys] + [first[f"__vm_{c}"] for c in var_cols])
    wire, total = allgather_columns(GpuJoinOps.to_wire(means), means.height, group)
    allm = GpuJoinOps.from_wire(wire, total)
    for k in keys:  # logical key dtypes (Datetime, ...) survive the wire as their physical
        allm[k]._with_logical(df[k]._logical_dtype())
    if len(keys) == 1 and df[keys[0]]._col.dtype in (N.I64, N.I32, N.U32, N.BOOL):
        sq = []
        for c in var_cols:
            o = N.Column()
            N.check(N.lib().plgpu_group_sq_dev(C.byref(df[keys[0]]._col), C.byref(df[c]._col),
                                               C.byref(allm[keys[0]]._col), C.byref(allm[f"__vm_{c}"]._col),
                                               C.byref(o), None))
            sq.append(Series._from_native(f"__vd_{c}", o))
        rows = DataFrame(list(df._cols.values()) + sq)
    else:
        rows = _join(df, allm, key, key, "_right", "m:m", True, "left", "left")
        sq = [_eval(((col(c).cast("f64") - col(f"__vm_{c}")) * (col(c).cast("f64") - col(f"__vm_{c}")))
                    .alias(f"__vd_{c}"), rows) for c in var_cols]
        rows = DataFrame(list(rows._cols.values()) + sq)
    second = group_by_agg(rows, key, [col(f"__vd_{c}").sum().alias(f"__vd_{c}") for c in var_cols], predicate,
                          group=group)
    # the same groups on this rank, in another order: align on the key
    second = _join(DataFrame([first[k] for k in keys]), second, key, key, "_right", "m:m", True, "left", "inner")
    res: dict[str, Series] = {}
    for e in aggs:
        b = _agg_base(e)
        if not (b.kind == "agg" and b.op in ("std", "var")):
            res[e.output_name()] = first[e.output_name()]
            continue
        c = b.args[0].value
        o = N.Column()
        N.check(N.lib().plgpu_var_finalize(C.byref(second[f"__vd_{c}"]._col), C.byref(first[f"__vn_{c}"]._col),
                                           int(b.value), int(b.op == "std"), C.byref(o), None))
        res[e.output_name()] = Series._from_native(e.output_name(), o)
    return DataFrame([first[k] for k in keys] + [res[e.output_name()] for e in aggs])


def group_by_agg(df, key: str, aggs: Sequence[Expr], predicate: Expr | None = None, *, group=None,
                 info: dict | None = None):
    """`df.lazy().filter(predicate).group_by(key).agg(*aggs)` over the shards
    held by all ranks of `group`.  Returns this rank's partition of the
    result (the groups whose key hashes to this rank; the null-key and
    INT64_MIN groups live on rank 0).  Group order is unspecified, as in the
    reference without maintain_order.

    Two protocols, chosen identically on every rank:
      partial states (the default): each rank pre-aggregates its shard
        with no collective, one small all-reduce agrees the stage's status
        and any wide f64 sum's digit range (agree_wide), and only group
        records cross the links (two all-to-alls, volume ~ groups);
      row shuffle: keys or values no fixed-size record carries -- String
        keys longer than 7 bytes, key tuples with Float / String columns or
        more than 63 bits, var / std with such keys or of an expression -- send the selected
        rows to the rank owning their key (volume ~ selected rows) and
        aggregate them there with the single-GPU group-by."""
    import torch.distributed as dist

    if not dist.is_initialized():
        raise N.InvalidOperationError("torch.distributed is not initialised")
    device = _device_for(group)
    if device.type != "cuda":
        raise N.InvalidOperationError("the GPU group-by needs a process that owns a GPU (nccl / RCCL backend)")
    try:
        return _group_by_agg_states(df, key, aggs, predicate, group, info)
    except _RowShuffle as why:
        return run_shuffled(GpuShuffleOps, df, key, aggs, predicate, group, device, info, str(why))


class GpuShuffleOps:
    """The device half of the row-shuffle group-by, through the C-ABI."""

    @staticmethod
    def select(df, predicate, names: Sequence[str]):
        from .frame import DataFrame

        src = df.filter(predicate) if predicate is not None else df
        return DataFrame([src[c] for c in names])

    partition = staticmethod(lambda df, keys, world, nulls_equal: GpuJoinOps.partition(df, keys, world, nulls_equal))
    to_wire = staticmethod(lambda df, perm=None: GpuJoinOps.to_wire(df, perm))
    from_wire = staticmethod(lambda cols, n: GpuJoinOps.from_wire(cols, n))

    @staticmethod
    def logical(df, names: Sequence[str]):
        return [df[c]._logical_dtype() for c in names]

    @staticmethod
    def restore(rows, names: Sequence[str], logical):
        for c, lg in zip(names, logical):
            rows[c]._with_logical(lg)
        return rows

    @staticmethod
    def local_group_by(rows, key, aggs):
        from .frame import _group_by

        return _group_by(rows, key, list(aggs), False, None, None)

    @staticmethod
    def rows(df) -> int:
        return df.height


def run_shuffled(ops, df, key, aggs: Sequence[Expr], predicate, group, device, info: dict | None = None,
                 why: str = ""):
    """Row-shuffle group-by over any `ops` (the GPU one above, or a host
    model in tests/test_distributed.py): the predicate and a projection onto
    the key and input columns run locally, the selected rows go to the rank
    owning their key (plgpu_hash_partition: the same key -- TotalEq for
    floats, the bytes for Strings -- routes alike on every rank; null keys to
    rank 0) in one all-to-all per buffer, and each rank aggregates what it
    received with the single-GPU group-by.  The partitions are stable and
    the exchange concatenates sources in rank order, so every group's rows
    arrive in the global row order (first() / last() hold).  A failure
    before the exchange is agreed by one status all-reduce."""
    import torch.distributed as dist

    from .expr import col

    world = dist.get_world_size(group)
    keys = [key] if isinstance(key, str) else list(key)
    aggs = [a if isinstance(a, Expr) else col(a) for a in aggs]
    err = wire = counts = None
    names: list[str] = []
    try:
        names = list(dict.fromkeys(keys + [c for e in aggs for c in e.meta_root_names()]))
        sub = ops.select(df, predicate, names)
        logical = ops.logical(sub, names)
        perm, counts = ops.partition(sub, keys, world, True)
        wire = ops.to_wire(sub, perm)
    except Exception as e:  # noqa: BLE001
        err = e
    failed = _allreduce_max([1 if err is not None else 0], group, device)[0]
    if err is not None:
        raise err
    if failed:
        raise N.ComputeError("multi-GPU group-by (row shuffle): the local stage failed on another rank")
    cols, n = exchange_columns(wire, counts, group)
    rows = ops.restore(ops.from_wire(cols, n), names, logical)
    out = ops.local_group_by(rows, keys[0] if len(keys) == 1 else tuple(keys), aggs)
    if info is not None:
        info.update({"protocol": "row_shuffle", "reason": why, "rows_sent": int(sum(counts)), "rows_received": n,
                     "groups": ops.rows(out)})
    return out


def _group_by_agg_states(df, key, aggs: Sequence[Expr], predicate, group, info: dict | None):
    """The partial-states protocol of group_by_agg; raises _RowShuffle (on
    every rank alike) for an input it cannot carry."""
    import torch
    import torch.distributed as dist

    from .frame import _agg_base, _gb_lower, _group_by, _join, _lower_strings
    from .expr import col

    world = dist.get_world_size(group)
    device = _device_for(group)
    from .frame import DataFrame, Series, String

    aggs = [a if isinstance(a, Expr) else col(a) for a in aggs]
    # aggregations over expressions: each expression evaluated once into a
    # column of this rank's shard, whose partial states then cross the
    # protocol as a column's do (elementwise, so sharding does not change it)
    from .frame import _eval

    todo = []
    for i, e in enumerate(aggs):
        b = _agg_base(e)
        if b.kind == "agg" and b.args[0].kind != "col":
            nm = f"__in{i}"
            while nm in df.columns:
                nm += "_"
            todo.append(b.args[0].alias(nm))
            aggs[i] = Expr("agg", (col(nm),), op=b.op, value=b.value).alias(e.output_name())
    if todo:
        # whether an expression evaluates depends on the shard's data (a
        # strict cast, memory): agreed before the first collective
        extra = agreed_stage(lambda: [_eval(x, df) for x in todo], group, device,
                             "evaluating an aggregation input")
        df = DataFrame(list(df._cols.values()) + extra)
    if any(_agg_base(e).kind == "agg" and _agg_base(e).op in ("std", "var") for e in aggs):
        return _group_by_var(df, key, aggs, predicate, group, info)
    if predicate is not None:
        # String comparisons / pattern tests become Boolean columns first,
        # against the String columns as they are (before the key turns into
        # its Int64 codes), as the single-GPU group-by does
        predicate, df = _lower_strings(predicate, df)
    string_key = isinstance(key, str) and key in df.columns and df[key].dtype is String
    if string_key:
        # String symbols of <= 7 bytes cross the integer-keyed protocol as
        # exact Int64 codes (the same code on every rank); decoded at the end
        codes = N.Column()
        short = C.c_int32(0)
        err = None
        try:
            N.check(N.lib().plgpu_str_encode_short(C.byref(df[key]._col), C.byref(codes), C.byref(short), None))
        except N.PolaroidError as e:
            err = e
        failed, longer = _allreduce_max([1 if err is not None else 0, 0 if short.value else 1], group, device)
        if err is not None:
            raise err
        if failed:
            raise N.ComputeError("multi-GPU group-by: encoding the String key failed on another rank")
        if longer:
            raise _RowShuffle("String keys longer than 7 bytes")
        df = DataFrame([Series._from_native(key, codes) if nm == key else df[nm] for nm in df.columns])
    packed = None
    float_key = None
    if isinstance(key, str) and key in df.columns and df[key]._col.dtype in (N.F64, N.F32):
        # a float key crosses as the Int64 of its canonical bits (TotalEq
        # classes: -0.0 with 0.0, every NaN together); decoded at the end
        # The output key is each group's first selected value (the reference
        # takes the group's first row: -0.0 or 0.0, the NaN's own bits), so
        # the original column rides along as a first() aggregation.
        float_key = "__kf_first"
        while float_key in df.columns:
            float_key += "_"
        codes = N.Column()
        N.check(N.lib().plgpu_float_key_encode(C.byref(df[key]._col), C.byref(codes), None))
        df = DataFrame([Series._from_native(key, codes) if nm == key else df[nm] for nm in df.columns] +
                       [df[key].alias(float_key)])
        aggs = aggs + [col(float_key).first().alias(float_key)]
    if not isinstance(key, str) and len(key) == 1:
        key = key[0]
    if not isinstance(key, str) or (key in df.columns and df[key]._col.dtype in _PACKABLE
                                    and df[key]._col.dtype not in (N.I64, N.I32)):
        # several integer / Boolean keys, or one narrow / unsigned / Boolean
        # key: one exact Int64 code with a plan agreed over the ranks
        packed, df, key = _pack_keys(df, [key] if isinstance(key, str) else list(key), group, device)
    if not isinstance(key, str) or key not in df.columns or df[key]._col.dtype not in (N.I64, N.I32):
        raise _RowShuffle("a key the record protocol does not carry")
    # first() / last() travel as values (run_first_last); every other
    # aggregation as exact partial states
    fl = _first_last_split(aggs)
    rest = [e for i, e in enumerate(aggs) if i not in fl]
    for i in fl:
        c = _agg_base(aggs[i]).args[0]
        if c.kind != "col" or c.value not in df.columns or df[c.value]._col.dtype not in _TORCH_WIRE:
            raise _RowShuffle("first() / last() of a String column")
    timings: dict = {}
    out = part = mi = None
    if rest or not fl:
        g = _gb_lower(df, key, rest, predicate)
        part = GpuPartial(g, world)
        out, mi = run_partitioned(part, world, group, device, timings if info is not None else None)
    if fl:
        t0 = time.perf_counter()
        ops = GpuFirstLastOps(key, [aggs[i] for i in fl])
        logical = {}

        def local_stage():
            loc = _group_by(df, key, ops.exprs, False, predicate, None)
            logical.update({e.output_name(): loc[e.output_name()]._logical_dtype() for e in ops.exprs})
            return loc

        owned = run_first_last(ops, local_stage, world, group)
        for nm, lg in logical.items():
            owned[nm]._with_logical(lg)
        if out is None:
            joined = owned
        else:
            # both hold exactly this rank's groups (the same rows selected, the
            # same partition function); the null key matches itself
            joined = _join(out, owned, key, key, "_right", "m:m", True, "left", "inner")
        out = DataFrame([joined[key]] + [joined[e.output_name()] for e in aggs])
        if info is not None:
            torch.cuda.synchronize()
            timings["first_last_ms"] = (time.perf_counter() - t0) * 1e3
    if packed is not None:
        out = _unpack_keys(out, key, packed, [e.output_name() for e in aggs])
    if float_key is not None:
        out = DataFrame([out[float_key].alias(key) if nm == key else out[nm] for nm in out.columns
                         if nm != float_key])
    if string_key:
        strs = N.Column()
        N.check(N.lib().plgpu_str_decode_short(C.byref(out[key]._col), C.byref(strs), None))
        out = DataFrame([Series._from_native(key, strs) if nm == key else out[nm] for nm in out.columns])
    torch.cuda.synchronize()
    if info is not None:
        d = part.info.as_dict() if part is not None else {}
        d["merge_groups"] = d["groups"] = mi.groups if mi is not None else out.height
        d.update(timings)
        info.update(d)
    return out


# ====================================================================== join
# Multi-GPU inner equi-join.  The reference's streaming equi-join
# (polars-stream/src/nodes/joins/equi_join.rs) splits both sides with one
# HashPartitioner (:445 partition_and_sink for the build side, :740
# partition_and_probe for the probe side) so that partition p of the build
# side only meets partition p of the probe side.  Across GPUs:
#
#   shuffle   - every rank hash-partitions both of its shards by key into
#               `world` partitions (plgpu_hash_partition), packs the rows
#               partition-major into flat buffers (plgpu_gather_rows) and
#               exchanges them with one all-to-all per buffer (RCCL over
#               xGMI); each rank then joins the partition it owns with the
#               single-GPU join.  Volume = both sides' rows, once.
#   broadcast - when the smaller side is small (a dimension table such as
#               BASELINE configs[3]'s 1e7-row build), it is all-gathered to
#               every rank and each rank joins its local shard of the larger
#               side against it: the large side never moves, so the per-rank
#               work is the local probe (weak scaling).
#
# Either way each rank returns its share of the inner join; the union over
# ranks equals the single-process join as a multiset of rows (the order is
# unspecified, as with the reference's maintain_order="none").

JOIN_BROADCAST_ROWS = 1 << 26  # the smaller side is broadcast up to 64M rows (all ranks)

_TORCH_WIRE = {N.I64: "int64", N.F64: "int64", N.I32: "int32", N.U32: "int32", N.BOOL: "uint8", N.U64: "int64",
               N.F32: "int32", N.I16: "int16", N.U16: "int16", N.I8: "int8", N.U8: "uint8"}


class WireColumn:
    """One column on the wire: values (8 / 4 bytes per row, Booleans one
    byte) and an optional validity byte mask, as flat torch tensors.  A
    String column sends each row's byte length as its values and the bytes
    themselves, rows in order, in `data` (uint8)."""

    __slots__ = ("name", "dtype", "values", "valid", "data")

    def __init__(self, name: str, dtype: int, values, valid, data=None):
        self.name, self.dtype, self.values, self.valid, self.data = name, dtype, values, valid, data


def _segment_sums(lens, counts: Sequence[int]) -> list[int]:
    """Sums of `lens` over consecutive segments of counts[i] rows (the
    bytes of each destination's rows of a String column)."""
    import torch

    if not counts:
        return []
    ends = torch.tensor([sum(counts[:i + 1]) for i in range(len(counts))], dtype=torch.int64, device=lens.device)
    cs = torch.cat([torch.zeros(1, dtype=torch.int64, device=lens.device), torch.cumsum(lens, 0)])
    at = cs[ends].tolist()
    return [int(a - b) for a, b in zip(at, [0] + at[:-1])]


def _wire_spec(cols: Sequence[WireColumn], group) -> list[tuple[str, int, bool]]:
    """(name, dtype, nullable) agreed by all ranks: the schemas must match and
    a column is sent with a validity mask if any rank holds nulls in it."""
    import torch.distributed as dist

    mine = [(c.name, int(c.dtype), c.valid is not None) for c in cols]
    world = dist.get_world_size(group)
    allspecs: list = [None] * world
    dist.all_gather_object(allspecs, mine, group=group)
    base = [(n, d) for n, d, _ in allspecs[0]]
    for s in allspecs[1:]:
        if [(n, d) for n, d, _ in s] != base:
            raise N.ComputeError("multi-GPU join: the ranks' shards have different schemas")
    return [(n, d, any(s[i][2] for s in allspecs)) for i, (n, d) in enumerate(base)]


def _fill_valid(c: WireColumn, nullable: bool):
    import torch

    if nullable and c.valid is None:
        c.valid = torch.ones(c.values.shape[0], dtype=torch.uint8, device=c.values.device)
    elif not nullable:
        c.valid = None


def exchange_columns(cols: Sequence[WireColumn], counts: Sequence[int], group=None):
    """All-to-all of rows grouped by destination rank (`counts[r]` rows for
    rank r, in rank order).  Returns (received columns, rows received)."""
    import torch
    import torch.distributed as dist

    spec = _wire_spec(cols, group)
    device = cols[0].values.device if cols else torch.device("cpu")
    sc = torch.tensor(list(counts), dtype=torch.int64, device=device)
    rc = torch.empty_like(sc)
    _a2a(rc, sc, group=group)
    rcounts = [int(v) for v in rc.tolist()]
    n = sum(rcounts)
    out = []
    for c, (name, dt, nullable) in zip(cols, spec):
        _fill_valid(c, nullable)
        bufs = []
        for t in (c.values, c.valid):
            if t is None:
                bufs.append(None)
                continue
            r = torch.empty(n, dtype=t.dtype, device=t.device)
            alltoallv(r, t, rcounts, list(counts), group)
            bufs.append(r)
        data = None
        if dt == N.STR:
            # the bytes of each destination's rows: their byte counts first
            sb = _segment_sums(c.values, counts)
            sbt = torch.tensor(sb, dtype=torch.int64, device=device)
            rbt = torch.empty_like(sbt)
            _a2a(rbt, sbt, group=group)
            rb = [int(v) for v in rbt.tolist()]
            data = torch.empty(sum(rb), dtype=torch.uint8, device=device)
            alltoallv(data, c.data, rb, sb, group)
        out.append(WireColumn(name, dt, bufs[0], bufs[1], data))
    _settle(device)
    return out, n


def allgather_columns(cols: Sequence[WireColumn], rows: int, group=None):
    """Every rank receives every rank's rows (rank order).  Returns
    (columns, total rows)."""
    import torch
    import torch.distributed as dist

    spec = _wire_spec(cols, group)
    world = dist.get_world_size(group)
    device = cols[0].values.device if cols else torch.device("cpu")
    cnt = torch.tensor([rows], dtype=torch.int64, device=device)
    allc = [torch.empty_like(cnt) for _ in range(world)]
    _all_gather(allc, cnt, group)
    counts = [int(t.item()) for t in allc]
    cap = max(counts) if counts else 0
    total = sum(counts)
    out = []
    for c, (name, dt, nullable) in zip(cols, spec):
        _fill_valid(c, nullable)
        bufs = []
        for t in (c.values, c.valid):
            if t is None:
                bufs.append(None)
                continue
            padded = torch.zeros(cap, dtype=t.dtype, device=t.device)
            padded[:rows] = t[:rows]
            parts = [torch.empty(cap, dtype=t.dtype, device=t.device) for _ in range(world)]
            _all_gather(parts, padded, group)
            bufs.append(torch.cat([p[:k] for p, k in zip(parts, counts)]) if total else
                        torch.empty(0, dtype=t.dtype, device=t.device))
        data = None
        if dt == N.STR:
            nb = torch.tensor([int(c.data.numel())], dtype=torch.int64, device=device)
            alln = [torch.empty_like(nb) for _ in range(world)]
            _all_gather(alln, nb, group)
            bcounts = [int(t.item()) for t in alln]
            bcap = max(bcounts) if bcounts else 0
            padded = torch.zeros(bcap, dtype=torch.uint8, device=device)
            padded[:bcounts[dist.get_rank(group)]] = c.data
            parts = [torch.empty(bcap, dtype=torch.uint8, device=device) for _ in range(world)]
            _all_gather(parts, padded, group)
            data = torch.cat([p[:k] for p, k in zip(parts, bcounts)]) if bcap else \
                torch.empty(0, dtype=torch.uint8, device=device)
        out.append(WireColumn(name, dt, bufs[0], bufs[1], data))
    _settle(device)
    return out, total


class GpuJoinOps:
    """The device half of the multi-GPU join, all through the C-ABI."""

    @staticmethod
    def rows(df) -> int:
        return df.height

    @staticmethod
    def partition(df, keys: Sequence[str], world: int, nulls_equal: bool):
        from .frame import _col_array

        perm = N.Column()
        counts = (C.c_int64 * world)()
        ks = [df[k] for k in keys]
        N.check(N.lib().plgpu_hash_partition(_col_array(ks), len(ks), world, int(nulls_equal), C.byref(perm),
                                             counts, None))
        from .frame import Series

        return Series._from_native("__perm", perm), [int(c) for c in counts]

    @staticmethod
    def to_wire(df, perm=None) -> list[WireColumn]:
        import torch

        from .frame import _col_array

        n = df.height if perm is None else perm.len()
        dev = torch.device("cuda", torch.cuda.current_device())
        names = df.columns
        fixed = [nm for nm in names if df[nm]._col.dtype != N.STR]
        wire = {}
        for nm in fixed:
            s = df[nm]
            dt = s._col.dtype
            vals = torch.empty(n, dtype=getattr(torch, _TORCH_WIRE[dt]), device=dev)
            valid = torch.empty(n, dtype=torch.uint8, device=dev) if s._col.validity else None
            wire[nm] = WireColumn(nm, dt, vals, valid)
        if fixed and n:
            out = [wire[nm] for nm in fixed]
            dv = (C.c_void_p * len(fixed))(*[c.values.data_ptr() for c in out])
            vv = (C.c_void_p * len(fixed))(*[c.valid.data_ptr() if c.valid is not None else None for c in out])
            N.check(N.lib().plgpu_gather_rows(_col_array([df[nm] for nm in fixed]), len(fixed),
                                              C.byref(perm._col) if perm is not None else None, dv, vv, None))
        for nm in names:
            if nm not in wire:
                wire[nm] = GpuJoinOps._string_to_wire(df[nm], perm, n, dev)
        return [wire[nm] for nm in names]

    @staticmethod
    def _string_to_wire(s, perm, n: int, dev) -> WireColumn:
        """A String column (rows in `perm` order) -> per-row byte lengths,
        a validity byte mask and the bytes (plgpu_gather packs the rows)."""
        import torch

        from .frame import Series, UInt32, _col_array

        if perm is None:
            idx_t = torch.arange(n, dtype=torch.int32, device=dev)
            perm = Series.from_device("__perm", UInt32, idx_t.data_ptr(), n, keepalive=idx_t)
        g = N.Column()
        N.check(N.lib().plgpu_gather(_col_array([s]), 1, C.byref(perm._col), C.byref(g), None))
        gs = Series._from_native(s.name, g)
        offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
        N.check(N.lib().plgpu_memcpy_d2d(C.c_void_p(offs.data_ptr()), C.c_void_p(int(g.values) + 8 * int(g.offset)),
                                         8 * (n + 1), None))
        N.check(N.lib().plgpu_synchronize(None))
        b0, b1 = (int(v) for v in offs[[0, n]].tolist())
        data = torch.empty(b1 - b0, dtype=torch.uint8, device=dev)
        if b1 > b0:
            N.check(N.lib().plgpu_memcpy_d2d(C.c_void_p(data.data_ptr()), C.c_void_p(int(g.data) + b0), b1 - b0, None))
        valid = None
        if g.validity:
            nbytes = (int(g.offset) + n + 7) // 8
            bits = torch.empty(nbytes, dtype=torch.uint8, device=dev)
            N.check(N.lib().plgpu_memcpy_d2d(C.c_void_p(bits.data_ptr()), C.c_void_p(int(g.validity)), nbytes, None))
            shifts = torch.arange(8, dtype=torch.uint8, device=dev)
            valid = ((bits.view(-1, 1) >> shifts) & 1).view(-1)[int(g.offset): int(g.offset) + n].contiguous()
        N.check(N.lib().plgpu_synchronize(None))
        del gs
        return WireColumn(s.name, N.STR, (offs[1:] - offs[:-1]).contiguous(), valid, data)

    @staticmethod
    def from_wire(cols: Sequence[WireColumn], n: int):
        from .frame import DataFrame, Series, _BY_CODE

        import torch

        series = []
        for c in cols:
            dt = _BY_CODE[c.dtype]
            if c.dtype == N.STR:
                offs = torch.zeros(n + 1, dtype=torch.int64, device=c.values.device)
                if n:
                    torch.cumsum(c.values, 0, out=offs[1:])
                data = c.data if c.data.numel() else torch.zeros(1, dtype=torch.uint8, device=c.values.device)
                keep = [offs, data, c.valid]
                mptr, nulls = None, 0
                if c.valid is not None:
                    vb = N.DeviceBuffer(((n + 63) // 64) * 8)
                    z = C.c_int64(0)
                    N.check(N.lib().plgpu_pack_bits(C.c_void_p(c.valid.data_ptr()), n, C.c_void_p(vb.ptr),
                                                    C.byref(z), None))
                    mptr, nulls = vb.ptr, int(z.value)
                    keep.append(vb)
                series.append(Series.from_device(c.name, dt, offs.data_ptr(), n, mptr, keepalive=keep,
                                                 null_count=nulls, data_ptr=data.data_ptr()))
                continue
            keep: list = [c.values, c.valid]
            vptr = c.values.data_ptr()
            if c.dtype == N.BOOL:
                bits = N.DeviceBuffer(((n + 63) // 64) * 8)
                N.check(N.lib().plgpu_pack_bits(C.c_void_p(vptr), n, C.c_void_p(bits.ptr), None, None))
                vptr = bits.ptr
                keep.append(bits)
            mptr, nulls = None, 0
            if c.valid is not None:
                vb = N.DeviceBuffer(((n + 63) // 64) * 8)
                z = C.c_int64(0)
                N.check(N.lib().plgpu_pack_bits(C.c_void_p(c.valid.data_ptr()), n, C.c_void_p(vb.ptr), C.byref(z),
                                                None))
                mptr, nulls = vb.ptr, int(z.value)
                keep.append(vb)
            series.append(Series.from_device(c.name, dt, vptr, n, mptr, keepalive=keep, null_count=nulls))
        return DataFrame(series)

    @staticmethod
    def local_join(left, right, left_on, right_on, suffix: str, nulls_equal: bool, how: str = "inner"):
        from .frame import _join

        return _join(left, right, left_on, right_on, suffix, "m:m", nulls_equal, "none", how)


# Which side a join type may broadcast: the side whose unmatched rows the
# result does not keep (a broadcast side is seen by every rank, so rows it
# keeps would come out once per rank).  A full join keeps both: shuffle only.
_BROADCASTABLE = {"inner": ("left", "right"), "left": ("right",), "semi": ("right",), "anti": ("right",),
                  "right": ("left",), "full": ()}


def run_join(ops, left, right, left_keys: Sequence[str], right_keys: Sequence[str], suffix: str,
             nulls_equal: bool, strategy: str, group, device, info: dict | None = None, how: str = "inner"):
    """The multi-GPU join protocol over any `ops` implementation (the GPU one
    above, or a host model in tests/test_distributed_join.py)."""
    import torch
    import torch.distributed as dist

    if how not in _BROADCASTABLE:
        raise ValueError(f"invalid join type {how!r}")
    world = dist.get_world_size(group)
    sizes = torch.tensor([ops.rows(left), ops.rows(right)], dtype=torch.int64, device=device)
    _all_reduce(sizes, dist.ReduceOp.SUM, group)
    nl, nr = (int(v) for v in sizes.tolist())
    allowed = _BROADCASTABLE[how]
    # the side to broadcast: the smaller allowed one
    bside = min(allowed, key=lambda sd: nl if sd == "left" else nr) if allowed else None
    if strategy == "auto":
        small = bside is not None and (nl if bside == "left" else nr) <= JOIN_BROADCAST_ROWS
        strategy = "broadcast" if small else "shuffle"
    if strategy not in ("broadcast", "shuffle"):
        raise ValueError(f"invalid join strategy {strategy!r}")
    if strategy == "broadcast" and bside is None:
        raise ValueError("a full join cannot broadcast either side; use strategy='shuffle'")
    lk = left_keys[0] if len(left_keys) == 1 else tuple(left_keys)
    rk = right_keys[0] if len(right_keys) == 1 else tuple(right_keys)
    if strategy == "broadcast":
        if bside == "right":
            cols, n = allgather_columns(ops.to_wire(right), ops.rows(right), group)
            right = ops.from_wire(cols, n)
        else:
            cols, n = allgather_columns(ops.to_wire(left), ops.rows(left), group)
            left = ops.from_wire(cols, n)
        moved = n
    else:
        moved = 0
        sides = []
        # a side whose unmatched rows are kept must keep its null-key rows
        # too: they are routed (to rank 0) instead of dropped
        keep_nulls = {"left": how in ("left", "anti", "full"), "right": how in ("right", "full")}
        for sd, df, keys in (("left", left, left_keys), ("right", right, right_keys)):
            perm, counts = ops.partition(df, keys, world, nulls_equal or keep_nulls[sd])
            cols, n = exchange_columns(ops.to_wire(df, perm), counts, group)
            sides.append(ops.from_wire(cols, n))
            moved += n
        left, right = sides
    out = ops.local_join(left, right, lk, rk, suffix, nulls_equal, how)
    if info is not None:
        info.update({"strategy": strategy, "left_rows": nl, "right_rows": nr, "rows_received": moved})
    return out


def join(left, right, on: str | Sequence[str] | None = None, how: str = "inner", *, left_on=None, right_on=None,
         suffix: str = "_right", nulls_equal: bool = False, strategy: str = "auto", group=None,
         info: dict | None = None):
    """`left.join(right, on=..., how=...)` over the shards held by all ranks
    of `group` (one GPU per rank, RCCL); how = inner / left / right / full /
    semi / anti.  Returns this rank's share of the result; the union over
    ranks is the join of the concatenated shards.  strategy: "auto"
    (broadcast the smaller side the join type allows -- the right side of a
    left / semi / anti join, the left of a right join, none for a full join
    -- up to JOIN_BROADCAST_ROWS rows, else shuffle), "broadcast" or
    "shuffle"."""
    import torch
    import torch.distributed as dist

    if not dist.is_initialized():
        raise N.InvalidOperationError("torch.distributed is not initialised")
    device = _device_for(group)
    if device.type != "cuda":
        raise N.InvalidOperationError("the GPU join needs a process that owns a GPU (nccl / RCCL backend)")
    if on is not None:
        left_on = right_on = on
    if left_on is None or right_on is None:
        raise ValueError("must specify `on` OR `left_on` and `right_on`")
    lks = [left_on] if isinstance(left_on, str) else list(left_on)
    rks = [right_on] if isinstance(right_on, str) else list(right_on)
    if len(lks) != len(rks):
        raise N.InvalidOperationError("the number of join key columns must be equal on both sides")
    out = run_join(GpuJoinOps, left, right, lks, rks, suffix, nulls_equal, strategy, group, device, info, how)
    torch.cuda.synchronize()
    return out
