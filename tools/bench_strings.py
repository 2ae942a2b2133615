"""The headline query with a String symbol column (the usual OHLCV schema):
filter(close > 250).group_by(symbol).agg(open/high/low/close.sum()) over
--rows rows of 100 distinct 5-byte symbols, one GPU, inputs in HBM.

    python tools/bench_strings.py [--rows 1e9 --steps 5 --warmup 1]

Symbol strings are built on device as Arrow large_string buffers (int64
offsets + bytes).  Prints one JSON line; `groupby_info` is the library's
diagnostics of the last step.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=float, default=1e9)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    args = ap.parse_args()
    import torch

    import polaroid_amd as pl
    from polaroid_amd import _native as N

    n = int(args.rows)
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    pool = torch.tensor([list(f"SYM{i:02d}".encode()) for i in range(100)], dtype=torch.uint8, device="cuda")
    chunk = 1 << 27
    data = torch.empty(n * 5, dtype=torch.uint8, device="cuda")
    cols = {nm: torch.empty(n, dtype=torch.float64, device="cuda") for nm in ("open", "high", "low", "close")}
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        code = torch.randint(0, 100, (e - s,), device="cuda", generator=g)
        data[s * 5:e * 5] = pool[code].reshape(-1)
        base = torch.rand(e - s, device="cuda", generator=g, dtype=torch.float64) * 500
        for nm in cols:
            cols[nm][s:e] = base + torch.rand(e - s, device="cuda", generator=g, dtype=torch.float64)
        del code, base
    offsets = torch.arange(0, (n + 1) * 5, 5, dtype=torch.int64, device="cuda")
    sym = pl.Series.from_device("symbol", pl.Int64, offsets.data_ptr(), n, keepalive=(offsets, data))
    sym._col.dtype = N.STR
    sym._col.data = data.data_ptr()
    df = pl.DataFrame([sym] + [pl.Series.from_torch(nm, t) for nm, t in cols.items()])
    q = (df.lazy().filter(pl.col("close") > 250.0).group_by("symbol")
         .agg(pl.col("open").sum(), pl.col("high").sum(), pl.col("low").sum(), pl.col("close").sum()))
    info = {}
    out = None
    for _ in range(args.warmup):
        out = q.collect(info=info)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = q.collect(info=info)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    print(json.dumps({
        "metric": "Mrows/sec filter+groupby-agg, String symbol key (5-byte symbols), 4 f64 sums",
        "value": round(n / dt / 1e6, 1), "unit": "Mrows/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(dt * 1e3, 3), "higher_is_better": True, "dtype": "f64",
        "data": "synthetic OHLCV columns, symbols as Arrow large_string built on device",
        "config": {"workload": "filter(close > 250).group_by(symbol: String).agg(open/high/low/close.sum())",
                   "rows": n, "groups": out.height},
        "groupby_info": {k: v for k, v in info.items() if k in ("path", "reruns", "main_kernel_ms", "groups")},
    }), flush=True)


if __name__ == "__main__":
    main()
