"""Headline benchmark: Mrows/s of filter -> group_by -> agg(sum) over a
1e9-row OHLCV-shaped frame (symbol: i64, open/high/low/close: f64), inputs
resident in HBM, on N GPUs (one process per GPU).

    python bench.py [--gpus N --steps K --warmup W --rows R --groups G]

One step = one full query `filter(close > 250).group_by(symbol).agg(
open.sum(), high.sum(), low.sum(), close.sum())` through the C-ABI.  With
N > 1 each rank holds its own R-row shard (weak scaling), aggregates it
locally into exact partial states, and the partial states are hash-
partitioned by key and exchanged with one RCCL all-to-all, then merged
(DESIGN.md §Multi-GPU).  Rank 0 prints one JSON line.

`python bench.py --gpus N` with N > 1 outside a torch.distributed launch
starts `torch.distributed.run --nproc-per-node N` on this same command as a
child process (before anything touches the GPU) and exits with its code.
At N = 8 the default shard is 1.25e9 rows per GPU: BASELINE configs[4]'s
1e10-row group-by on one 8-GPU node.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mrows/sec filter+groupby-agg on 1e9-row f64/i64; achieved HBM GB/s vs peak"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
THRESHOLD = 250.0
BYTES_PER_ROW = 8 + 4 * 8      # key + open/high/low/close read once (close is also the predicate)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=float, default=None,
                    help="rows per GPU (default 1e9; 1.25e9 at 8 GPUs = configs[4]'s 1e10 rows)")
    ap.add_argument("--groups", type=int, default=100, help="distinct symbols (h2oai id4: K=100)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="cpu_baseline time budget")
    ap.add_argument("--cpu-rows", type=float, default=1e7, help="cpu_baseline sample rows (configs[0]: 1e7)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--plugin-rows", type=float, default=1e8,
                    help="rows of the plugin leg (host Arrow frame through execute_with_polaroid; configs[1] = 1e8)")
    ap.add_argument("--no-plugin", action="store_true")
    ap.add_argument("--no-vwap", action="store_true")
    ap.add_argument("--no-std", action="store_true")
    ap.add_argument("--dry-run", action="store_true",
                    help="print this rank's launch parameters and exit before touching the GPU (tests)")
    return ap.parse_args()


def make_data(torch, n: int, groups: int, seed: int):
    """OHLCV-shaped synthetic columns generated on the device, chunked."""
    dev = torch.device("cuda")
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    base = torch.rand(groups, device=dev, generator=g, dtype=torch.float64) * 480.0 + 10.0
    sym = torch.empty(n, dtype=torch.int64, device=dev)
    cols = {k: torch.empty(n, dtype=torch.float64, device=dev) for k in ("open", "high", "low", "close")}
    chunk = 1 << 26
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        m = e - s
        k = torch.randint(0, groups, (m,), device=dev, generator=g, dtype=torch.int64)
        sym[s:e] = k * 7919 + 1_000_000  # sparse symbol ids
        p = base[k]
        o = p * torch.exp(0.02 * torch.randn(m, device=dev, generator=g, dtype=torch.float64))
        c = p * torch.exp(0.02 * torch.randn(m, device=dev, generator=g, dtype=torch.float64))
        spread = torch.rand(m, device=dev, generator=g, dtype=torch.float64) * 0.01
        cols["open"][s:e] = o
        cols["close"][s:e] = c
        cols["high"][s:e] = torch.maximum(o, c) * (1.0 + spread)
        cols["low"][s:e] = torch.minimum(o, c) * (1.0 - spread)
    torch.cuda.synchronize()
    return sym, cols


def host_cores() -> tuple[int, str]:
    """Every host core this process may run on: the CPU affinity set,
    capped by the cgroup's CPU quota when one is set (a container's share)."""
    aff = len(os.sched_getaffinity(0))
    note = f"sched_getaffinity: {aff}"
    n = aff
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            q = max(1, int(int(quota) // int(period)))
            note += f", cgroup cpu.max quota: {q}"
            n = min(n, q)
    except (OSError, ValueError):
        pass
    return n, note


def cpu_baseline(rows: int, groups: int, seconds: float) -> dict:
    """The oracle's OpenMP restatement of the reference's streaming hash
    aggregation, timed on the host cores (rank 0, N=1 only)."""
    from oracle import oracle as O

    threads, cores_note = host_cores()
    rng = np.random.default_rng(1)
    base = rng.uniform(10, 490, groups)
    k = rng.integers(0, groups, rows)
    key = (k * 7919 + 1_000_000).astype(np.int64)
    p = base[k]
    o = p * np.exp(0.02 * rng.standard_normal(rows))
    c = p * np.exp(0.02 * rng.standard_normal(rows))
    sp = rng.random(rows) * 0.01
    h = np.maximum(o, c) * (1 + sp)
    lo = np.minimum(o, c) * (1 - sp)
    O.baseline_filter_groupby_sum(key[:1000], c[:1000], THRESHOLD, [o[:1000], h[:1000], lo[:1000], c[:1000]],
                                  threads)
    times = []
    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end or not times:
        t0 = time.perf_counter()
        O.baseline_filter_groupby_sum(key, c, THRESHOLD, [o, h, lo, c], threads)
        times.append(time.perf_counter() - t0)
    t = float(np.median(times))
    return {"value": rows / t / 1e6, "unit": "Mrows/s", "cores": threads, "kind": "port",
            "sample": f"{rows:.0e} rows (configs[0] size) x {len(times)} runs of the same query (median), OpenMP "
                      f"{threads} threads ({cores_note}), oracle/polars_oracle.c:or_baseline_filter_groupby_sum"}


def plugin_leg(rows: int, groups: int) -> dict:
    """The headline query through the polars plugin (execute_with_polaroid,
    driven by a model of polars' NodeTraverser, tools/ir_model.py) on a host
    Arrow frame: cold = the first query (scan: Arrow chunks -> HBM over the
    host link, then the query), warm = the same query again (the scanned
    columns resident in the plugin's ColumnCache).  rank 0, N = 1 only."""
    import pyarrow as pa

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import ir_model

    from polaroid_amd import polars_engine as PE

    rng = np.random.default_rng(7)
    base = rng.uniform(10, 490, groups)
    k = rng.integers(0, groups, rows)
    p = base[k]
    o = p * np.exp(0.02 * rng.standard_normal(rows))
    c = p * np.exp(0.02 * rng.standard_normal(rows))
    sp = rng.random(rows) * 0.01
    table = pa.table({"symbol": pa.array((k * 7919 + 1_000_000).astype(np.int64)), "open": pa.array(o),
                      "high": pa.array(np.maximum(o, c) * (1 + sp)), "low": pa.array(np.minimum(o, c) * (1 - sp)),
                      "close": pa.array(c)})
    del k, p, o, c, sp
    cols = ["open", "high", "low", "close"]
    PE.column_cache().clear()
    times = []
    for _ in range(3):
        nt = ir_model.filter_group_by_sum(table, "symbol", "close", THRESHOLD, cols, chunk_rows=1 << 23)
        PE.execute_with_polaroid(nt, None, config={"device_cache_bytes": 64 << 30}, to_frame=lambda t: t)
        t0 = time.perf_counter()
        out = nt.udf(None, None, None, False)
        times.append((time.perf_counter() - t0) * 1e3)
        assert 0 < out.num_rows <= groups
    PE.column_cache().clear()
    cold, warm = times[0], min(times[1:])
    return {"rows": rows, "bytes": int(table.nbytes), "cold_ms": round(cold, 2), "warm_ms": round(warm, 3),
            "cold_Mrows_s": round(rows / cold / 1e3, 1), "warm_Mrows_s": round(rows / warm / 1e3, 1),
            "note": "execute_with_polaroid on a host Arrow frame of 8M-row RecordBatches; cold = scan over the "
                    "host link + query, warm = scanned columns resident (ColumnCache); result to Arrow"}


def timed_leg(torch, q, n: int, steps: int, warmup: int, bytes_per_row: int) -> dict:
    """Wall time per collect() of a resident-frame query and the mean HIP-event
    time of its aggregation kernel, with the kernel's HBM fraction at the
    query's algorithmic bytes per row."""
    for _ in range(warmup):
        q.collect()
    torch.cuda.synchronize()
    kms = []
    t0 = time.perf_counter()
    for _ in range(steps):
        info = {}
        out = q.collect(info=info)
        kms.append(info.get("main_kernel_ms", float("nan")))
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    k = float(np.mean(kms))
    achieved = bytes_per_row * n / (k * 1e-3) / 1e9
    assert 0 < out.height <= n
    return {"rows": n, "ms_per_step": round(dt * 1e3, 3), "Mrows_s": round(n / dt / 1e6, 1),
            "kernel_ms": round(k, 4), "bytes_per_row": bytes_per_row, "achieved_GBs": round(achieved, 1),
            "frac": round(achieved / HBM_PEAK_GBS, 4), "path": info.get("path")}


def vwap_leg(torch, pl, df, sym, close, steps: int, warmup: int) -> dict:
    """VWAP over the same resident frame: filter(close > 250).group_by(symbol)
    .agg((close * volume).sum(), volume.sum()); the product is computed in the
    fused kernel's registers (DESIGN.md "Aggregations over expressions"), so the
    algorithmic bytes are key + close + volume = 24 B/row.  rank 0, N = 1."""
    n = sym.numel()
    g = torch.Generator(device=sym.device)
    g.manual_seed(99)
    vol = torch.empty(n, dtype=torch.float64, device=sym.device)
    chunk = 1 << 26
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        vol[s:e] = torch.floor(torch.rand(e - s, device=sym.device, generator=g, dtype=torch.float64) * 1000.0) + 1.0
    vdf = pl.DataFrame([pl.Series.from_torch("symbol", sym), pl.Series.from_torch("close", close),
                        pl.Series.from_torch("volume", vol)])
    q = vdf.lazy().filter(pl.col("close") > THRESHOLD).group_by("symbol").agg(
        (pl.col("close") * pl.col("volume")).sum().alias("pv"), pl.col("volume").sum().alias("v"))
    r = timed_leg(torch, q, n, steps, warmup, 24)
    del vdf, vol
    return {"query": "filter(close > 250).group_by(symbol).agg((close * volume).sum(), volume.sum())",
            "kernel": "gb_fast_kernel<NACC=2,PRED=1,SUMONLY,DERIV> (close * volume in registers)", **r}


def std_leg(torch, pl, df, steps: int, warmup: int) -> dict:
    """close.std() per symbol over the same resident frame (one fused pass:
    exact sums of x, x * x and its error, DESIGN.md "var / std in one pass");
    algorithmic bytes key + close = 16 B/row.  rank 0, N = 1."""
    q = df.lazy().filter(pl.col("close") > THRESHOLD).group_by("symbol").agg(pl.col("close").std().alias("sd"))
    r = timed_leg(torch, q, df.height, steps, warmup, 16)
    return {"query": "filter(close > 250).group_by(symbol).agg(close.std())",
            "kernel": "gb_fast_kernel<NACC=3,PRED=1,SUMONLY,VAR> (variance triple)", **r}


def load_traffic(n_rows: int):
    """HBM bytes per launch from the committed rocprofv3 PMC summary, if any
    (profiles/traffic.json written by tools/pmc_traffic.py)."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(path):
        return None
    try:
        t = json.load(open(path))
        if int(t.get("rows", -1)) == n_rows:
            return float(t["hbm_bytes_per_launch"])
    except Exception:
        return None
    return None


def launch_ranks(n: int) -> int:
    """Run this command under torch.distributed.run with n ranks (one per
    GPU) as a child process; called before any GPU call in this process."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def main():
    args = parse()
    if args.gpus > 1 and "RANK" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if "RANK" in os.environ and world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.rows is None:
        args.rows = 1.25e9 if world == 8 else 1e9
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        print(json.dumps({"rank": rank, "local_rank": local, "world": world, "rows_per_gpu": args.rows,
                          "master_addr": os.environ.get("MASTER_ADDR")}), flush=True)
        return
    # launched by torch.distributed.run (even with one rank): the
    # hash-partitioned path over RCCL; plain `python bench.py`: one GPU
    distributed = "RANK" in os.environ and "MASTER_ADDR" in os.environ
    json_out = sys.stdout
    if distributed:
        # RCCL prints its version banner on the process's stdout when the
        # first communicator forms: send fd 1 to stderr for the run and keep
        # the original stdout for the one JSON line
        sys.stdout.flush()
        json_out = os.fdopen(os.dup(1), "w")
        os.dup2(2, 1)
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import polaroid_amd as pl
    from polaroid_amd import distributed as pdist

    pl._native.check(pl._native.lib().plgpu_set_device(torch.cuda.current_device()))
    n = int(args.rows)
    sym, cols = make_data(torch, n, args.groups, seed=1234 + rank)
    df = pl.DataFrame([pl.Series.from_torch("symbol", sym)] +
                      [pl.Series.from_torch(k, v) for k, v in cols.items()])
    aggs = [pl.col(k).sum() for k in ("open", "high", "low", "close")]
    query = df.lazy().filter(pl.col("close") > THRESHOLD).group_by("symbol").agg(*aggs)

    def step(info):
        if not distributed:
            return query.collect(info=info)
        return pdist.group_by_agg(df, "symbol", aggs, pl.col("close") > THRESHOLD, info=info)

    for _ in range(args.warmup):
        step({})
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    kernel_ms, phases = [], []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        info = {}
        out = step(info)
        kernel_ms.append(info.get("main_kernel_ms", float("nan")))
        phases.append([info.get(k, float("nan")) for k in ("partial_ms", "exchange_ms", "merge_ms")])
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    dt = time.perf_counter() - t0
    if distributed:
        t = torch.tensor([dt], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    per_rank = None
    if distributed:
        # per-rank fused-kernel and phase times (ms per step), gathered to rank 0
        mine = torch.tensor([float(np.mean(kernel_ms))] + list(np.mean(np.array(phases), axis=0)),
                            device="cuda", dtype=torch.float64)
        allr = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        per_rank = [[round(float(x), 4) for x in t.tolist()] for t in allr]
    ms_per_step = dt / args.steps * 1e3
    total_rows = n * world
    value = total_rows * args.steps / dt / 1e6
    kms = float(np.mean(kernel_ms))
    achieved = BYTES_PER_ROW * n / (kms * 1e-3) / 1e9
    traffic = load_traffic(n)
    result = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "Mrows/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic OHLCV-shaped columns generated on device (torch RNG), inputs resident in HBM",
        "config": {
            "workload": "filter(close > 250).group_by(symbol).agg(open/high/low/close.sum()) "
                        f"{n:.3g} rows per GPU, {args.groups} groups"
                        + (f" = {total_rows:.3g} rows over {world} GPUs (configs[4])" if world == 8 else
                           " (metric size; configs[1] = 1e8 rows)"),
            "rows_per_gpu": n, "groups": args.groups, "global_batch": total_rows,
            "columns": "symbol:i64 open,high,low,close:f64",
            "selectivity": None if out is None else round(float(info.get("rows_selected", 0)) / n, 4),
            "parallelism": f"hash-partitioned x{world} (RCCL all-to-all of partial states)" if distributed
            else "single GPU",
        },
        "ranks": None if per_rank is None else {
            "rccl_world_size": dist.get_world_size(),
            "backend": dist.get_backend(),
            "fields": ["kernel_ms", "partial_ms", "exchange_ms", "merge_ms"],
            "per_rank": per_rank,
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "kernel": f"gb_fast_kernel<NACC=4,PRED=1,SUMONLY,ROWS=2,LIMBS={info.get('sum_limbs', 3)}> "
                      f"(fused filter + LDS hash aggregation, exact f64 sums), grid {info.get('grid')}",
            "kernel_ms": round(kms, 4),
            "bytes_per_row": BYTES_PER_ROW,
        },
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(int(args.cpu_rows), args.groups, args.cpu_seconds)
    if rank == 0 and world == 1 and not args.no_vwap:
        result["vwap"] = vwap_leg(torch, pl, df, sym, cols["close"], args.steps, args.warmup)
    if rank == 0 and world == 1 and not args.no_std:
        result["std"] = std_leg(torch, pl, df, args.steps, args.warmup)
    if rank == 0 and world == 1 and not args.no_plugin:
        del df, query, out, sym, cols
        torch.cuda.empty_cache()
        result["plugin"] = plugin_leg(int(args.plugin_rows), args.groups)
        result["plugin_cold_ms"] = result["plugin"]["cold_ms"]
        result["plugin_warm_ms"] = result["plugin"]["warm_ms"]
    if rank == 0:
        print(json.dumps(result), file=json_out, flush=True)
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
