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


def progress(msg: str) -> None:
    """One line per finished phase on stderr (the JSON line stays alone on
    stdout), so a long run shows it is alive."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


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
    ap.add_argument("--no-sort", action="store_true", help="skip the configs[2] sort + rolling leg")
    ap.add_argument("--no-join", action="store_true", help="skip the configs[3] join leg")
    ap.add_argument("--no-keys", action="store_true", help="skip the Categorical / String / (symbol, day) legs")
    ap.add_argument("--no-nulls", action="store_true", help="skip the validity-bitmap leg (1 %% nulls)")
    ap.add_argument("--no-filter", action="store_true", help="skip the filter-only leg (row a1)")
    ap.add_argument("--no-many-groups", action="store_true", help="skip the many-groups leg")
    ap.add_argument("--many-groups", type=str, default=",".join(str(g) for g in MANY_GROUPS),
                    help="comma-separated group counts of the many-groups leg")
    ap.add_argument("--leg-steps", type=int, default=5, help="timed steps of the sort and join legs (<= --steps)")
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
    for _ in range(6):
        nt = ir_model.filter_group_by_sum(table, "symbol", "close", THRESHOLD, cols, chunk_rows=1 << 23)
        PE.execute_with_polaroid(nt, None, config={"device_cache_bytes": 64 << 30}, to_frame=lambda t: t)
        t0 = time.perf_counter()
        out = nt.udf(None, None, None, False)
        times.append((time.perf_counter() - t0) * 1e3)
        assert 0 < out.num_rows <= groups
    PE.column_cache().clear()
    cold, warm = times[0], min(times[1:])
    return {"rows": rows, "bytes": int(table.nbytes), "cold_ms": round(cold, 2), "warm_ms": round(warm, 3),
            "warm_median_ms": round(float(np.median(times[1:])), 3),
            "cold_Mrows_s": round(rows / cold / 1e3, 1), "warm_Mrows_s": round(rows / warm / 1e3, 1),
            "note": "execute_with_polaroid on a host Arrow frame of 8M-row RecordBatches; cold = scan over the "
                    "host link + query (first query), warm = scanned columns resident (ColumnCache), min / "
                    "median of the next 5 queries; result to Arrow"}


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
            "kernel": "gb_fast_kernel<NACC=2,PRED=1,SUMONLY,VAR=2> (product pair: close * volume in registers)", **r}


def std_leg(torch, pl, df, steps: int, warmup: int) -> dict:
    """close.std() per symbol over the same resident frame (one fused pass:
    exact sums of x, x * x and its error, DESIGN.md "var / std in one pass");
    algorithmic bytes key + close = 16 B/row.  rank 0, N = 1."""
    q = df.lazy().filter(pl.col("close") > THRESHOLD).group_by("symbol").agg(pl.col("close").std().alias("sd"))
    r = timed_leg(torch, q, df.height, steps, warmup, 16)
    return {"query": "filter(close > 250).group_by(symbol).agg(close.std())",
            "kernel": "gb_fast_kernel<NACC=3,PRED=1,SUMONLY,VAR> (variance triple)", **r}


def key_frame(torch, pl, sym, cols: dict, case: str):
    """The headline frame with another symbol encoding (the same rows):
    "categorical" (UInt32 codes over a 100-string dictionary, as polars
    exports a Categorical), "string" (5-byte tickers as Arrow large_string)
    or "sym_day" (the Int64 symbol and an Int32 day rising with the row
    number: time-ordered daily bars).  Returns (frame, group-by keys, buffers
    to keep alive)."""
    import pyarrow as pa

    from polaroid_amd import _native as N

    n = sym.numel()
    vals = [pl.Series.from_torch(nm, t) for nm, t in cols.items()]
    k = (sym - 1_000_000) // 7919  # 0..99
    if case == "categorical":
        codes = k.to(torch.int32)
        cs = pl.Series.from_device("symbol", pl.UInt32, codes.data_ptr(), n, keepalive=codes)
        dictionary = pl.Series.from_arrow("symbol", pa.array([f"SYM{i:02d}" for i in range(100)], pa.large_string()))
        return pl.DataFrame([pl.Series._categorical("symbol", dictionary, cs)] + vals), ("symbol",), [codes]
    if case == "string":
        pool = torch.tensor([list(f"SYM{i:02d}".encode()) for i in range(100)], dtype=torch.uint8, device=sym.device)
        data = torch.empty(n * 5, dtype=torch.uint8, device=sym.device)
        ch = 1 << 27
        for s in range(0, n, ch):
            e = min(n, s + ch)
            data[s * 5:e * 5] = pool[k[s:e]].reshape(-1)
        offsets = torch.arange(0, (n + 1) * 5, 5, dtype=torch.int64, device=sym.device)
        st = pl.Series.from_device("symbol", pl.Int64, offsets.data_ptr(), n, keepalive=(offsets, data))
        st._col.dtype = N.STR
        st._col.data = data.data_ptr()
        return pl.DataFrame([st] + vals), ("symbol",), [offsets, data]
    day = (torch.arange(n, device=sym.device, dtype=torch.int64) // (n // 250 + 1)).to(torch.int32)
    return (pl.DataFrame([pl.Series.from_torch("symbol", sym), pl.Series.from_torch("day", day)] + vals),
            ("symbol", "day"), [day])


def keys_leg(torch, pl, sym, cols: dict, steps: int, warmup: int, headline_ms: float) -> dict:
    """The headline query over the other key encodings of the same rows
    (key_frame): Categorical symbol (grouped by its UInt32 codes, the
    reference's into_groups.rs:132-139), String symbol, and (symbol, day)
    (both keys packed into the group code inside the fused kernel).  Each
    case: ms per collect(), the fused kernel's HIP-event time, and the ratio
    to the Int64 headline's step.  rank 0, N = 1."""
    from polaroid_amd import _native as N

    out = {}
    sums = [pl.col(c).sum() for c in ("open", "high", "low", "close")]
    for case, bpr in (("categorical", 36), ("sym_day", 44), ("string", 45)):
        df, keys, keep = key_frame(torch, pl, sym, cols, case)
        q = df.lazy().filter(pl.col("close") > THRESHOLD).group_by(*keys).agg(*sums)

        def step():
            info = {}
            q.collect(info=info)
            return info

        ms, kernels, info = _time_steps(torch, step, steps, warmup)
        kms = kernels.get("gb_fast_kernel", {}).get("ms_mean")
        out[case] = {"ms_per_step": round(ms, 3), "vs_int64_headline": round(ms / headline_ms, 3),
                     "kernel_ms": kms, "bytes_per_row": bpr,
                     "frac": round(bpr * sym.numel() / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if kms else None,
                     "key_pack": info.get("key_pack"), "categorical_codes": info.get("categorical_codes", 0),
                     "kernels": kernels}
        del df, q, keep
        torch.cuda.empty_cache()
    out["note"] = ("bytes_per_row: the fused kernel's algorithmic bytes (categorical: 4 B codes + 32 B; sym_day: "
                   "8 + 4 + 32; string: 8 B offsets + 5 B of bytes + 32)")
    return out


def filter_leg(torch, pl, df, steps: int, warmup: int, cpu_rows: int, cpu_seconds: float, no_cpu: bool) -> dict:
    """Row a1: `filter(close > 250).collect()` over the headline frame's 5
    columns (no aggregation): the mask + tile-count pass, the tile scan and
    the one multi-column scatter (polars-compute/src/filter/mod.rs:18 filter,
    each column by the one mask; option filt_fused: the one-pass look-back
    kernel instead, measured slower).  Algorithmic bytes: the 5 columns read
    once (40 B/row) and the selected rows written once (40 B each).  rank 0,
    N = 1."""
    n = df.height

    def step():
        return df.filter(pl.col("close") > THRESHOLD).height

    ms, kernels, sel = _time_steps(torch, step, steps, warmup)
    algo = n * 40 + sel * 40
    if "filter_fused8_kernel" in kernels:
        # the one-pass look-back kernel: the algorithmic bytes are the leg's
        scatter = _leg_roofline(kernels, "filter_fused8_kernel", algo,
                                "5 x 8 B read per row (the predicate column once), 5 x 8 B written per selected row")
        mask = None
    else:
        scatter = _leg_roofline(kernels, "filter_scatter8_kernel", n * 40 + n / 8 + sel * 40,
                                "5 x 8 B read per row + the mask bit, 5 x 8 B written per selected row")
        mask = _leg_roofline(kernels, "filter_mask_kernel", n * 8 + n / 8,
                             "8 B predicate read per row + 1 mask bit written")
    r = {"query": "filter(close > 250).collect() over symbol, open, high, low, close", "rows": n,
         "rows_selected": sel, "ms_per_step": round(ms, 3), "Mrows_s": round(n / ms / 1e3, 1),
         "algorithmic_GB": round(algo / 1e9, 2), "step_frac": round(algo / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
         "roofline": scatter, "mask": mask, "kernels": kernels,
         "note": "step_frac: 5 columns read once + selected rows written once over the step time; roofline: the "
                 "dominant kernel (the multi-column scatter) at its own algorithmic bytes"}
    if not no_cpu:
        from oracle import oracle as O

        threads, cores_note = host_cores()
        rng = np.random.default_rng(3)
        c = rng.uniform(10, 490, cpu_rows)
        hc = [rng.integers(0, 1 << 40, cpu_rows).astype(np.int64)] + [c * rng.uniform(0.99, 1.01, cpu_rows)
                                                                       for _ in range(3)] + [c]
        O.baseline_filter(c[:1000], THRESHOLD, [x[:1000] for x in hc], threads)
        times = []
        t_end = time.perf_counter() + cpu_seconds
        while time.perf_counter() < t_end or not times:
            t0 = time.perf_counter()
            O.baseline_filter(c, THRESHOLD, hc, threads)
            times.append(time.perf_counter() - t0)
        t = float(np.median(times))
        r["cpu_baseline"] = {"value": round(cpu_rows / t / 1e6, 1), "unit": "Mrows/s", "cores": threads,
                             "kind": "port",
                             "sample": f"{cpu_rows:.0e} rows x 5 columns x {len(times)} runs (median), OpenMP "
                                       f"{threads} threads ({cores_note}), oracle/polars_oracle.c:or_baseline_filter"}
    return r


MANY_GROUPS = (20_000, 600_000, 1_000_000, 10_000_000)


def many_groups_leg(torch, pl, cols: dict, steps: int, warmup: int, groups_list, cpu_rows: int,
                    cpu_seconds: float, no_cpu: bool) -> dict:
    """The headline query with G random symbols (G = 2e4 ... 1e7) over the
    same 1e9 price rows: the partitioned path (DESIGN.md "Group-by for many
    groups") -- count pass, one or two radix scatter passes, then the
    partitions' LDS aggregation.  Per G: ms per step, the path taken, and
    each kernel's HBM fraction at its own algorithmic bytes (count: key +
    predicate read, 8 B key per selected row at level 2; scatter: 40 B read
    per row + 40 B written per selected row at level 1, 40 + 40 B per
    selected row at level 2; aggregation: 40 B per selected row).  rank 0,
    N = 1."""
    n = cols["close"].numel()
    dev = cols["close"].device
    sums = [pl.col(c).sum() for c in ("open", "high", "low", "close")]
    out = {}
    for G in groups_list:
        g = torch.Generator(device=dev)
        g.manual_seed(G)
        key = torch.empty(n, dtype=torch.int64, device=dev)
        chunk = 1 << 26
        for s0 in range(0, n, chunk):
            e = min(n, s0 + chunk)
            key[s0:e] = torch.randint(0, G, (e - s0,), device=dev, generator=g, dtype=torch.int64) * 7919 + 1_000_000
        df = pl.DataFrame([pl.Series.from_torch("symbol", key)] + [pl.Series.from_torch(k, v) for k, v in cols.items()])
        q = df.lazy().filter(pl.col("close") > THRESHOLD).group_by("symbol").agg(*sums)

        def step():
            info = {}
            res = q.collect(info=info)
            info["out_groups"] = res.height
            return info

        ms, kernels, info = _time_steps(torch, step, steps, warmup)
        sel = int(info.get("rows_selected", 0))
        levels = int(info.get("part_layout", 0)) >> 8
        r = {"groups": int(info.get("out_groups", 0)), "ms_per_step": round(ms, 3), "Mrows_s": round(n / ms / 1e3, 1),
             "path": info.get("path"), "partition_bits": int(info.get("part_layout", 0)) & 0xFF,
             "scatter_passes": levels, "rows_selected": sel,
             "lds_miss_rows": int(info.get("global_path_rows", 0)), "reruns": int(info.get("reruns", 0)),
             "step_frac_read_once": round(40 * n / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
        if info.get("path") == 3:
            r["count"] = _leg_roofline(kernels, "gbp_count_kernel", n * 16 + (sel * 8 if levels == 2 else 0),
                                       "key + predicate read per row (+ 8 B key per selected row at level 2)", True)
            r["scatter"] = _leg_roofline(kernels, "gbp_scatter_kernel",
                                         n * 40 + sel * 40 + (sel * 80 if levels == 2 else 0),
                                         "40 B read per row + 40 B written per selected row (+ 40 + 40 B per "
                                         "selected row at level 2)", True)
            r["aggregate"] = _leg_roofline(kernels, "gb_part_agg_kernel", sel * 40, "40 B read per selected row",
                                           True)
        r["kernels"] = kernels
        out[str(G)] = r
        progress(f"many_groups {G}: {r['ms_per_step']} ms per step")
        del df, q, key
        torch.cuda.empty_cache()
    if not no_cpu:
        from oracle import oracle as O

        threads, cores_note = host_cores()
        G = 1_000_000
        rng = np.random.default_rng(5)
        key = (rng.integers(0, G, cpu_rows) * 7919 + 1_000_000).astype(np.int64)
        c = rng.uniform(10, 490, cpu_rows)
        hs = [c * rng.uniform(0.99, 1.01, cpu_rows) for _ in range(3)] + [c]
        times = []
        t_end = time.perf_counter() + cpu_seconds
        while time.perf_counter() < t_end or not times:
            t0 = time.perf_counter()
            O.baseline_filter_groupby_sum(key, c, THRESHOLD, hs, threads)
            times.append(time.perf_counter() - t0)
        t = float(np.median(times))
        out["cpu_baseline"] = {"value": round(cpu_rows / t / 1e6, 1), "unit": "Mrows/s", "cores": threads,
                               "kind": "port",
                               "sample": f"{cpu_rows:.0e} rows, {G:.0e} random groups x {len(times)} runs (median), "
                                         f"OpenMP {threads} threads ({cores_note}), "
                                         "oracle/polars_oracle.c:or_baseline_filter_groupby_sum"}
    return out


NULLS_GROUPS = (100, 1_000_000)
NULL_FRAC = 0.01


def null_bitmap(torch, n: int, frac: float, seed: int, dev):
    """An Arrow validity bitmap (LSB-first bit per row, 1 = valid) with about
    `frac` nulls at random rows, generated on the device in chunks."""
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    nbytes = (n + 7) // 8
    out = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    w = torch.tensor([1, 2, 4, 8, 16, 32, 64, 128], dtype=torch.uint8, device=dev)
    chunk = 1 << 24
    for s0 in range(0, nbytes, chunk):
        e = min(nbytes, s0 + chunk)
        bits = (torch.rand((e - s0) * 8, device=dev, generator=g) >= frac).to(torch.uint8).view(e - s0, 8)
        out[s0:e] = (bits * w).sum(dim=1).to(torch.uint8)
    return out


def nulls_leg(torch, pl, sym, cols: dict, steps: int, warmup: int, headline_ms: float) -> dict:
    """The headline query with Arrow validity bitmaps: ~1 % nulls in each of
    open, high, low, close ("values"), and the same plus ~1 % null symbols
    ("key_and_values"), at 100 groups (the headline's keys: the fused
    kernel's NULLS variant) and 1e6 random groups (the partitioned path, the
    null bits travelling with the partitioned rows), each against the
    null-free step of the same keys (100: the headline's step; 1e6: measured
    here).  Reference: polars-expr/src/reduce/sum.rs:108 reduce_one over
    Option<T>, :117 the has_nulls branch; polars-stream/src/nodes/
    group_by.rs:85 add_pre_agg.  rank 0, N = 1."""
    n = sym.numel()
    dev = sym.device
    sums = [pl.col(c).sum() for c in ("open", "high", "low", "close")]
    bitmaps = {c: null_bitmap(torch, n, NULL_FRAC, 500 + i, dev) for i, c in enumerate(cols)}
    kbits = null_bitmap(torch, n, NULL_FRAC, 600, dev)
    out = {"null_fraction": NULL_FRAC}
    for G in NULLS_GROUPS:
        if G == 100:
            key = sym
        else:
            g = torch.Generator(device=dev)
            g.manual_seed(G)
            key = torch.empty(n, dtype=torch.int64, device=dev)
            for s0 in range(0, n, 1 << 26):
                e = min(n, s0 + (1 << 26))
                key[s0:e] = torch.randint(0, G, (e - s0,), device=dev, generator=g, dtype=torch.int64) * 7919 + 1_000_000
        cases = {}
        variants = (("null_free", False, False), ("values", True, False), ("key_and_values", True, True))
        for name, vnull, knull in variants:
            if name == "null_free" and G == 100:
                continue
            df = pl.DataFrame([pl.Series.from_torch("symbol", key, kbits if knull else None)] +
                              [pl.Series.from_torch(c, t, bitmaps[c] if vnull else None) for c, t in cols.items()])
            q = df.lazy().filter(pl.col("close") > THRESHOLD).group_by("symbol").agg(*sums)

            def step():
                info = {}
                res = q.collect(info=info)
                info["out_groups"] = res.height
                return info

            ms, kernels, info = _time_steps(torch, step, steps, warmup)
            bpr = 40 + (0.5 if vnull else 0) + (0.125 if knull else 0)
            r = {"ms_per_step": round(ms, 3), "groups": int(info.get("out_groups", 0)), "path": info.get("path"),
                 "rows_selected": int(info.get("rows_selected", 0)), "bytes_per_row": bpr, "kernels": kernels}
            kms = kernels.get("gb_fast_kernel", {}).get("ms_mean")
            if info.get("path") in (1, 2) and kms:
                r["kernel_ms"] = kms
                r["frac"] = round(bpr * n / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
            cases[name] = r
            progress(f"nulls leg {G} {name}: {r['ms_per_step']} ms per step (path {r['path']})")
            del df, q
        base = headline_ms if G == 100 else cases["null_free"]["ms_per_step"]
        for name in ("values", "key_and_values"):
            cases[name]["vs_null_free"] = round(cases[name]["ms_per_step"] / base, 3)
        cases["null_free_ms"] = round(base, 3)
        out[str(G)] = cases
        if G != 100:
            del key
        torch.cuda.empty_cache()
    del bitmaps, kbits
    out["note"] = ("vs_null_free: step over the null-free step of the same keys (100 groups: the headline step of "
                   "this run); bytes_per_row: 40 + 1 validity bit per nullable column; frac: the fused kernel at "
                   "those bytes")
    return out


def _kernel_table(kt: dict, steps: int) -> dict:
    """plgpu_ktime_read sums -> {kernel: {ms_mean (per launch), ms_per_step, launches}}."""
    return {k: {"ms_mean": round(ms / max(c, 1), 4), "ms_per_step": round(ms / steps, 4), "launches": c}
            for k, (ms, c) in sorted(kt.items(), key=lambda kv: -kv[1][0])}


def _time_steps(torch, step, steps: int, warmup: int):
    """Warm up, then time `steps` calls of step() between device
    synchronisations with the library's kernel timer on (HIP events around
    each named launch, on the stream it runs on).  Returns (ms per step,
    per-kernel table, last result)."""
    from polaroid_amd import _native as N

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    prev = N.set_option("ktime", 1)
    N.ktime_read(reset=True)
    try:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            res = step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        kt = N.ktime_read(reset=True)
    finally:
        N.set_option("ktime", prev)
    return dt * 1e3, _kernel_table(kt, steps), res


def _leg_roofline(kernels: dict, name: str, algo_bytes: float, what: str, per_step: bool = False) -> dict:
    """The kernel's HBM fraction at `algo_bytes` per launch (per_step: per
    step, over all its launches in the step, e.g. both scatter passes)."""
    k = kernels.get(name, {}).get("ms_per_step" if per_step else "ms_mean")
    if not k:
        return {"kernel": name, "kernel_ms": None}
    gbs = algo_bytes / (k * 1e-3) / 1e9
    return {"kernel": name, "kernel_ms": k, "algorithmic_GB": round(algo_bytes / 1e9, 3), "bytes": what,
            "achieved_GBs": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4)}


SORT_ROWS = 1_000_000_000      # configs[2]: 1e9 rows, 8 columns mixed i64 / f64
SORT_WINDOW = 20
JOIN_PROBE, JOIN_BUILD = 1_000_000_000, 10_000_000   # configs[3]
# random 128-byte line requests per second from a 256 MiB table on one
# MI355X (tools/randread_bench.hip, profiles/r02_randread.txt: 54.5 G/s at
# grid 8192): the floor of a probe pass that needs one table line per row
RANDREQ_PER_S = 54.5e9


def sort_leg(torch, pl, steps: int, warmup: int, rows: int = SORT_ROWS, window: int = SORT_WINDOW) -> dict:
    """configs[2]: `df.sort("ts")` of a 1e9-row frame of 8 columns (ts, sym,
    qty, flags: i64; price, bid, ask, vol: f64; ts a shuffled timestamp
    below 2^40), then `rolling_mean(20)` of the sorted price.  One step = the
    radix arg_sort + the gather of all 8 columns + the rolling window.
    Reference: polars-core/src/chunked_array/ops/sort/arg_sort.rs:82 and
    polars-compute/src/rolling/no_nulls/mean.rs.  rank 0, N = 1."""
    dev = torch.device("cuda")
    g = torch.Generator(device=dev)
    g.manual_seed(11)
    chunk = 1 << 27
    cols = {}
    for k in ("ts", "sym", "qty", "flags"):
        t = torch.empty(rows, dtype=torch.int64, device=dev)
        hi = (1 << 40) if k == "ts" else (1 << 20)
        for s in range(0, rows, chunk):
            e = min(rows, s + chunk)
            t[s:e] = torch.randint(0, hi, (e - s,), device=dev, generator=g)
        cols[k] = t
    for k in ("price", "bid", "ask", "vol"):
        t = torch.empty(rows, dtype=torch.float64, device=dev)
        for s in range(0, rows, chunk):
            e = min(rows, s + chunk)
            t[s:e] = 100 + torch.rand(e - s, device=dev, generator=g, dtype=torch.float64) * 50
        cols[k] = t
    df = pl.DataFrame([pl.Series.from_torch(k, v) for k, v in cols.items()])

    def step():
        srt = df.sort("ts")
        roll = srt["price"].rolling_mean(window)
        return srt.height + roll.len()

    ms, kernels, res = _time_steps(torch, step, steps, warmup)
    assert res == 2 * rows
    # rolling_std(20) of the price column on its own (volatility: the exact
    # windowed second moment, rl_wave_var_kernel)
    price = df["price"]
    ms_std, kern_std, _ = _time_steps(torch, lambda: price.rolling_std(window).len(), steps, warmup)
    del df, cols, price
    torch.cuda.empty_cache()
    # the sort's floor: read the 8 input columns once and write the 8 sorted
    # columns once (128 B/row); rolling_mean reads and writes 8 B/row
    algo = rows * (8 * 8 * 2 + 16)
    gather = _leg_roofline(kernels, "aos_gather_kernel", rows * (64 + 4 + 64),
                           "64 B packed row read + 4 B row id read + 64 B column stores per row")
    pack = _leg_roofline(kernels, "aos_pack_kernel", rows * 128, "64 B read + 64 B packed row written per row")
    roll = _leg_roofline(kernels, "rl_wave_kernel", rows * 16, "8 B read + 8 B written per row")
    roll_std = _leg_roofline(kern_std, "rl_wave_var_kernel", rows * 16, "8 B read + 8 B written per row")
    roll_std["ms_per_step"] = round(ms_std, 3)
    roll_std["query"] = f"price.rolling_std({window})"
    return {"query": f"df.sort('ts') (8 columns: 4 x i64, 4 x f64) + sorted price.rolling_mean({window})",
            "rows": rows, "ms_per_step": round(ms, 3), "Mrows_s": round(rows / ms / 1e3, 1),
            "algorithmic_GB": round(algo / 1e9, 1),
            "step_frac": round(algo / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "roofline": gather, "pack": pack, "rolling": roll, "rolling_std": roll_std, "kernels": kernels,
            "note": "step_frac: the read-once / write-once floor (128 B/row sort + 16 B/row rolling) over the step "
                    "time; roofline: the dominant kernel (aos_gather_kernel) at its own algorithmic bytes"}


def join_leg(torch, pl, steps: int, warmup: int, n: int = JOIN_PROBE, m: int = JOIN_BUILD) -> dict:
    """configs[3]: `probe.join(build, on="k")` inner, 1e9 probe rows x 1e7
    unique build keys (i64), half the probe rows match; every output column
    materialised (k, probe payload, build payload).  Reference: polars-ops/
    src/frame/join/hash_join/single_keys_inner.rs:40 + general.rs:17
    _finish_join.  rank 0, N = 1."""
    dev = torch.device("cuda")
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    pk = torch.empty(n, dtype=torch.int64, device=dev)
    pv = torch.empty(n, dtype=torch.float64, device=dev)
    chunk = 1 << 27
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        pk[s:e] = torch.randint(0, 2 * m, (e - s,), device=dev, generator=g)
        pv[s:e] = torch.rand(e - s, device=dev, generator=g, dtype=torch.float64)
    bk = torch.randperm(2 * m, device=dev, generator=g)[:m].to(torch.int64)
    bv = torch.rand(m, device=dev, generator=g, dtype=torch.float64)
    probe = pl.DataFrame([pl.Series.from_torch("k", pk), pl.Series.from_torch("pv", pv)])
    build = pl.DataFrame([pl.Series.from_torch("k", bk), pl.Series.from_torch("bv", bv)])
    out_rows = []

    def step():
        out = probe.join(build, on="k")
        out_rows.append(out.height)
        return out.height

    ms, kernels, res = _time_steps(torch, step, steps, warmup)
    assert 0.45 * n < res < 0.55 * n
    del probe, build, pk, pv, bk, bv
    torch.cuda.empty_cache()
    algo = n * 16 + m * 16 + res * 24
    out = {"query": "probe.join(build, on='k') inner, output k, pv, bv", "probe_rows": n, "build_rows": m,
           "output_rows": res, "ms_per_step": round(ms, 3), "Mrows_s": round(n / ms / 1e3, 1),
           "algorithmic_GB": round(algo / 1e9, 2),
           "step_frac": round(algo / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "kernels": kernels}
    if "rj_match_kernel" in kernels:
        # the partitioned join (join.hip jn_radix_take): count + scatter of
        # the probe rows into 2^8 partitions, the L2-resident match pass,
        # then the row-format join's emit
        match = _leg_roofline(kernels, "rj_match_kernel", n * 8 + n / 8 + res * 8,
                              "partitioned key read (8 B per probe row), hit bits + the hits' payload words "
                              "written; sub-table reads served by the XCD's L2")
        match.update(_pmc_traffic("rj_match_kernel"))
        emit = _leg_roofline(kernels, "jn_take_emit_kernel", n * (16 + 1 / 8) + res * (8 + 24),
                             "partitioned k, pv + hit bits read per row, the hit's payload read, 3 x 8 B written "
                             "per output row")
        emit.update(_pmc_traffic("jn_take_emit_kernel"))
        count = _leg_roofline(kernels, "gbp_count_kernel", n * 8, "8 B probe key read per row")
        scatter = _leg_roofline(kernels, "gbp_scatter_kernel", n * 32, "k, pv read and written once (32 B per row)")
        floor = n * 8 + n * 32 + (n * 8 + res * 8) + (n * 16 + res * 32) + m * 16
        out.update({"path": "partitioned (radix) join", "roofline": match, "emit": emit, "count": count,
                    "scatter": scatter, "design_floor_GB": round(floor / 1e9, 2),
                    "design_floor_ms_at_peak": round(floor / (HBM_PEAK_GBS * 1e9) * 1e3, 3),
                    "note": "step_frac: probe (k, pv) + build (k, bv) read once, 3 output columns written once, "
                            "over the step time; design floor: count (8 B) + scatter (32 B) + match (8 B + 8 B "
                            "per hit) + emit (16 B + 32 B per hit) + build; roofline: the match pass"})
        return out
    match = _leg_roofline(kernels, "jn_probe_match_kernel", n * (8 + 8) + n // 8,
                          "8 B probe key read + 8 B payload word written per row + 1 hit bit")
    if match.get("kernel_ms"):
        floor_ms = n / RANDREQ_PER_S * 1e3
        match["random_request_floor_ms"] = round(floor_ms, 3)
        match["frac_of_request_floor"] = round(floor_ms / match["kernel_ms"], 4)
        match["request_floor_note"] = ("one random 128 B table line per probe row at 54.5 G requests/s "
                                       "(profiles/r02_randread.txt, 256 MiB table)")
    emit = _leg_roofline(kernels, "jn_take_emit_kernel", n * (8 + 8 + 1 / 8) + res * 24,
                         "payload words + probe payload read, 3 x 8 B written per output row")
    out.update({"path": "row-format table", "roofline": match, "emit": emit,
                "note": "step_frac: probe (k, pv) + build (k, bv) read once, 3 output columns written once, over "
                        "the step time; roofline: the match pass (bound by random table line requests, not bytes)"})
    return out


def cpu_sort_baseline(rows: int, seconds: float) -> dict:
    """configs[2]'s query on the host cores: the oracle's restatement of the
    reference's parallel stable arg_sort + per-column take + Kahan
    rolling_mean (oracle/polars_oracle.c:or_baseline_sort_rolling)."""
    from oracle import oracle as O

    threads, cores_note = host_cores()
    rng = np.random.default_rng(11)
    key = rng.integers(0, 1 << 40, rows).astype(np.int64)
    cols = [key] + [rng.integers(0, 1 << 20, rows).astype(np.int64) for _ in range(3)] + \
           [100 + rng.random(rows) * 50 for _ in range(4)]
    times = []
    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end or not times:
        t0 = time.perf_counter()
        O.baseline_sort_rolling(key, cols, 4, SORT_WINDOW, threads)
        times.append(time.perf_counter() - t0)
    t = float(np.median(times))
    return {"value": rows / t / 1e6, "unit": "Mrows/s", "cores": threads, "kind": "port",
            "sample": f"{rows:.0e} rows x 8 columns x {len(times)} runs (median), OpenMP {threads} threads "
                      f"({cores_note}), oracle/polars_oracle.c:or_baseline_sort_rolling"}


def cpu_join_baseline(probe_rows: int, seconds: float) -> dict:
    """configs[3]'s join on the host cores: the full 1e7-key build side and a
    probe sample, through the oracle's restatement of the reference's
    partitioned build + chunked probe + take (or_baseline_join_inner)."""
    from oracle import oracle as O

    threads, cores_note = host_cores()
    rng = np.random.default_rng(7)
    bk = rng.permutation(2 * JOIN_BUILD)[:JOIN_BUILD].astype(np.int64)
    bv = rng.random(JOIN_BUILD)
    pk = rng.integers(0, 2 * JOIN_BUILD, probe_rows).astype(np.int64)
    pv = rng.random(probe_rows)
    times = []
    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end or not times:
        t0 = time.perf_counter()
        O.baseline_join_inner(pk, pv, bk, bv, threads)
        times.append(time.perf_counter() - t0)
    t = float(np.median(times))
    return {"value": probe_rows / t / 1e6, "unit": "Mrows/s (probe rows)", "cores": threads, "kind": "port",
            "sample": f"{probe_rows:.0e} probe rows x {JOIN_BUILD:.0e} build keys (configs[3]'s build side) x "
                      f"{len(times)} runs (median), build included, OpenMP {threads} threads ({cores_note}), "
                      "oracle/polars_oracle.c:or_baseline_join_inner"}


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


def _pmc_traffic(kernel: str) -> dict:
    """A leg kernel's HBM bytes per launch from the committed rocprofv3 PMC
    passes (profiles/traffic.json "legs", written by tools/bench_evidence.py
    from the same command's FETCH_SIZE / WRITE_SIZE passes), if present."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        t = json.load(open(path)).get("legs", {}).get(kernel)
    except Exception:
        return {}
    if not t:
        return {}
    return {"pmc_traffic_GB": round(float(t["hbm_bytes_per_launch"]) / 1e9, 3),
            "pmc_source": t.get("source", "profiles/traffic.json")}


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
    progress(f"headline: {ms_per_step:.3f} ms per step")
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
        progress("cpu_baseline done")
    if rank == 0 and world == 1 and not args.no_vwap:
        result["vwap"] = vwap_leg(torch, pl, df, sym, cols["close"], args.steps, args.warmup)
        progress("vwap leg done")
    if rank == 0 and world == 1 and not args.no_std:
        result["std"] = std_leg(torch, pl, df, args.steps, args.warmup)
        progress("std leg done")
    if rank == 0 and world == 1 and not args.no_nulls:
        result["nulls"] = nulls_leg(torch, pl, sym, cols, args.leg_steps, 2, ms_per_step)
        progress("nulls leg done")
    if rank == 0 and world == 1 and not args.no_keys:
        torch.cuda.empty_cache()
        pl._native.release_cached()
        result["keys"] = keys_leg(torch, pl, sym, cols, args.leg_steps * 2, 2, ms_per_step)
        progress("keys leg done")
    if rank == 0 and world == 1 and not args.no_many_groups:
        del query, out
        query = out = None
        torch.cuda.empty_cache()
        result["many_groups"] = many_groups_leg(torch, pl, cols, max(2, args.leg_steps // 2), 1,
                                                [int(x) for x in args.many_groups.split(",") if x],
                                                int(args.cpu_rows), args.cpu_seconds / 2, args.no_cpu)
        progress("many_groups leg done")
    if rank == 0 and world == 1 and not args.no_filter:
        # over the headline frame, behind the other legs' allocations (the
        # pool is not returned first: the scatter's 10.0-11.5 ms spread
        # follows where its outputs land in HBM, from a returned pool or not,
        # profiles/r06_ab/r06r_filter_k0.json, tools/filter_pool_ab.py)
        result["filter"] = filter_leg(torch, pl, df, args.leg_steps, 2, int(args.cpu_rows), args.cpu_seconds / 2,
                                      args.no_cpu)
        progress(f"filter leg: {result['filter']['ms_per_step']} ms per step")
    if rank == 0 and world == 1 and not (args.no_sort and args.no_join and args.no_plugin):
        # the remaining legs need the HBM the headline frame holds
        del df, query, out, sym, cols
        torch.cuda.empty_cache()
        pl._native.release_cached()
    leg_steps = max(1, min(args.steps, args.leg_steps))
    if rank == 0 and world == 1 and not args.no_sort:
        result["sort"] = sort_leg(torch, pl, leg_steps, 1)
        progress(f"sort leg: {result['sort']['ms_per_step']} ms per step")
        if not args.no_cpu:
            result["sort"]["cpu_baseline"] = cpu_sort_baseline(int(args.cpu_rows), args.cpu_seconds / 2)
        pl._native.release_cached()
    if rank == 0 and world == 1 and not args.no_join:
        result["join"] = join_leg(torch, pl, leg_steps, 1)
        progress(f"join leg: {result['join']['ms_per_step']} ms per step")
        if not args.no_cpu:
            result["join"]["cpu_baseline"] = cpu_join_baseline(int(args.cpu_rows), args.cpu_seconds / 2)
        pl._native.release_cached()
    if rank == 0 and world == 1 and not args.no_plugin:
        result["plugin"] = plugin_leg(int(args.plugin_rows), args.groups)
        progress("plugin leg done")
        result["plugin_cold_ms"] = result["plugin"]["cold_ms"]
        result["plugin_warm_ms"] = result["plugin"]["warm_ms"]
    if rank == 0:
        print(json.dumps(result), file=json_out, flush=True)
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
