"""Standalone filter compaction over a resident 1e9-row OHLCV frame (4 f64
columns): `df.filter(col("close") > 250)` through plgpu_filter_expr.

    python tools/bench_filter.py [--rows 1e9 --steps 5 --threshold 250]

Prints one JSON line: ms per filter (host-timed, synchronised), rows kept,
and the algorithmic rate: 32 B read per row (the predicate column is one of
the four) + 32 B written per kept row."""
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
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--threshold", type=float, default=250.0)
    args = ap.parse_args()
    import torch

    import polaroid_amd as pl

    n = int(args.rows)
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    cols = {}
    for k in ("open", "high", "low", "close"):
        cols[k] = 10 + torch.rand(n, device="cuda", generator=g, dtype=torch.float64) * 480
    df = pl.DataFrame([pl.Series.from_torch(k, v) for k, v in cols.items()])
    q = pl.col("close") > args.threshold
    out = df.filter(q)
    torch.cuda.synchronize()
    ts = []
    for _ in range(args.steps):
        t0 = time.perf_counter()
        out = df.filter(q)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    t = min(ts)
    kept = out.height
    alg = 32 * n + 32 * kept
    print(json.dumps({"rows": n, "kept": kept, "ms": round(t * 1e3, 3),
                      "GBps_algorithmic": round(alg / t / 1e9, 1), "bytes_algorithmic": alg}), flush=True)


if __name__ == "__main__":
    main()
