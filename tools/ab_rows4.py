"""A/B of the fused group-by kernel's rows per thread (option rows4) on the
few-column queries of bench.py's vwap / std legs and a plain two-sum query,
1e9 rows, 100 groups, inputs resident in HBM.  Runs alternate between the
2-row tile (rows4 = 0) and the 4-row tile (rows4 = 7) so drift hits both.

    python tools/ab_rows4.py [--rows 1e9 --steps 5 --rounds 3]

One JSON line per (query, variant): ms per collect() and the fused kernel's
mean HIP-event time, with its HBM fraction at the query's algorithmic bytes.
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
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    import numpy as np
    import torch

    import bench
    import polaroid_amd as pl
    from polaroid_amd import _native as N

    n = int(args.rows)
    sym, cols = bench.make_data(torch, n, 100, seed=1234)
    g = torch.Generator(device="cuda")
    g.manual_seed(99)
    vol = torch.empty(n, dtype=torch.float64, device="cuda")
    for s in range(0, n, 1 << 26):
        e = min(n, s + (1 << 26))
        vol[s:e] = torch.floor(torch.rand(e - s, device="cuda", generator=g, dtype=torch.float64) * 1000.0) + 1.0
    df = pl.DataFrame([pl.Series.from_torch("symbol", sym), pl.Series.from_torch("close", cols["close"]),
                       pl.Series.from_torch("open", cols["open"]), pl.Series.from_torch("volume", vol)])
    f = df.lazy().filter(pl.col("close") > bench.THRESHOLD).group_by("symbol")
    queries = {
        "vwap": (f.agg((pl.col("close") * pl.col("volume")).sum().alias("pv"), pl.col("volume").sum().alias("v")), 24),
        "std": (f.agg(pl.col("close").std().alias("sd")), 16),
        "two_sums": (f.agg(pl.col("open").sum(), pl.col("volume").sum()), 32),
    }
    ref = {}
    res = {}
    for rnd in range(args.rounds):
        for variant in (0, 7):
            N.set_option("rows4", variant)
            for name, (q, bpr) in queries.items():
                out = q.collect()
                # bit-identical results across the variants (exact sums)
                key = name
                got = out.sort("symbol").to_arrow()
                if key in ref:
                    assert got.equals(ref[key]), (name, variant)
                else:
                    ref[key] = got
                torch.cuda.synchronize()
                kms = []
                t0 = time.perf_counter()
                for _ in range(args.steps):
                    info = {}
                    q.collect(info=info)
                    kms.append(info.get("main_kernel_ms", float("nan")))
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) / args.steps
                res.setdefault((name, variant), []).append((dt * 1e3, float(np.mean(kms)), info.get("grid")))
    N.set_option("rows4", 0)
    for (name, variant), v in res.items():
        bpr = queries[name][1]
        k = min(x[1] for x in v)
        print(json.dumps({"query": name, "rows4": variant, "ms_per_step": round(min(x[0] for x in v), 3),
                          "kernel_ms_min": round(k, 4), "kernel_ms_all": [round(x[1], 4) for x in v],
                          "frac": round(bpr * n / (k * 1e-3) / 1e9 / bench.HBM_PEAK_GBS, 4),
                          "grid": v[-1][2]}), flush=True)


if __name__ == "__main__":
    main()
