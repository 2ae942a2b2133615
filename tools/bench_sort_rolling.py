"""Sort + rolling workload of BASELINE.json configs[2]: a 1e9-row, 8-column
frame (4 x i64, 4 x f64) sorted by an i64 timestamp-like key, then
rolling_mean over one f64 column of the sorted frame; one GPU, inputs
resident in HBM.

    python tools/bench_sort_rolling.py [--rows 1e9 --window 20 --steps 3 --warmup 1]

A step = `df.sort("ts")` (radix arg-sort + gather of all 8 columns) followed
by `sorted["price"].rolling_mean(window)`.  The key is a shuffled timestamp
(values < 2^40, so 5 of the 8 radix passes run).  Prints one JSON line with
the per-phase times.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=float, default=1e9)
    ap.add_argument("--window", type=int, default=20)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    args = ap.parse_args()
    import torch

    import polaroid_amd as pl

    n = int(args.rows)
    g = torch.Generator(device="cuda")
    g.manual_seed(11)
    cols = {}
    ts = torch.empty(n, dtype=torch.int64, device="cuda")
    chunk = 1 << 27
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        ts[s:e] = torch.randint(0, 1 << 40, (e - s,), device="cuda", generator=g)
    cols["ts"] = ts
    for k in ("sym", "qty", "flags"):
        cols[k] = torch.randint(0, 1 << 20, (n,), device="cuda", generator=g, dtype=torch.int64)
    for k in ("price", "bid", "ask", "vol"):
        t = torch.empty(n, dtype=torch.float64, device="cuda")
        for s in range(0, n, chunk):
            e = min(n, s + chunk)
            t[s:e] = 100 + torch.rand(e - s, device="cuda", generator=g, dtype=torch.float64) * 50
        cols[k] = t
    df = pl.DataFrame([pl.Series.from_torch(k, v) for k, v in cols.items()])

    def step():
        t0 = time.perf_counter()
        srt = df.sort("ts")
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        roll = srt["price"].rolling_mean(args.window)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        return srt, roll, t1 - t0, t2 - t1

    for _ in range(args.warmup):
        step()
    ts_sort, ts_roll = [], []
    for _ in range(args.steps):
        _, _, a, b = step()
        ts_sort.append(a)
        ts_roll.append(b)
    sort_s, roll_s = min(ts_sort), min(ts_roll)
    total = sort_s + roll_s
    print(json.dumps({
        "metric": "Mrows/sec sort_by(i64) + rolling_mean on a 1e9-row 8-column frame",
        "value": round(n / total / 1e6, 1), "unit": "Mrows/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(total * 1e3, 3), "higher_is_better": True,
        "dtype": "int64/f64", "data": "synthetic, generated on device",
        "config": {"workload": f"df.sort('ts') (8 cols) + price.rolling_mean({args.window})", "rows": n,
                   "sort_ms": round(sort_s * 1e3, 3), "rolling_ms": round(roll_s * 1e3, 3),
                   "rolling_GBps": round(16 * n / roll_s / 1e9, 1)},
    }), flush=True)


if __name__ == "__main__":
    main()
