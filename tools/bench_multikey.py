"""Multi-key workloads on one GPU, inputs resident in HBM:

  groupby : filter(v0 > 0.5).group_by("sym", "day").agg(v0.sum(), v1.sum())
            over n rows (sym < 100, day < 250: 25,000 groups)
  join    : probe.join(build, on=["sym", "day"]) inner, maintain_order none
            (n probe rows x n/100 unique build tuples, ~50% hit rate)
  sort    : df.sort("day", "ts") on n rows x 4 columns
  groupby_hc : filter(v0 > 0.5).group_by("id").agg(v0.sum(), v1.sum()), 100,000 ids

    python tools/bench_multikey.py [--rows 1e9 --steps 3 --warmup 1 --only groupby,join,sort]

Prints one JSON line per workload with the best step time.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _timed(fn, steps, warmup):
    import torch

    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    best = float("inf")
    out = None
    for _ in range(steps):
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=float, default=1e9)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--only", default="groupby,groupby_hc,join,sort")
    ap.add_argument("--values", default="unit", help="unit: v0, v1 uniform on [0, 1); prices: uniform on [10, 500)")
    args = ap.parse_args()
    import torch

    import polaroid_amd as pl

    n = int(args.rows)
    only = set(args.only.split(","))
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    dev = "cuda"

    def ints(lo, hi, m):
        return torch.randint(lo, hi, (m,), device=dev, generator=g, dtype=torch.int64)

    def floats(m):
        x = torch.rand(m, device=dev, generator=g, dtype=torch.float64)
        return x * 490 + 10 if args.values == "prices" else x

    thr = 255.0 if args.values == "prices" else 0.5
    if "groupby" in only:
        df = pl.DataFrame([pl.Series.from_torch("sym", ints(0, 100, n)), pl.Series.from_torch("day", ints(0, 250, n)),
                           pl.Series.from_torch("v0", floats(n)), pl.Series.from_torch("v1", floats(n))])
        q = (df.lazy().filter(pl.col("v0") > thr).group_by("sym", "day")
             .agg(pl.col("v0").sum(), pl.col("v1").sum()))
        info = {}
        t, out = _timed(lambda: q.collect(info=info), args.steps, args.warmup)
        print(json.dumps({"workload": "filter + group_by(sym, day).agg(2 x f64 sum)", "rows": n,
                          "ms": round(t * 1e3, 3), "Mrows_per_s": round(n / t / 1e6, 1), "groups": out.height,
                          "reruns": info.get("reruns"), "path": info.get("path")}), flush=True)
        del df, q, out
        torch.cuda.empty_cache()

    if "groupby_hc" in only:
        card = 100_000
        df = pl.DataFrame([pl.Series.from_torch("id", ints(0, card, n)), pl.Series.from_torch("v0", floats(n)),
                           pl.Series.from_torch("v1", floats(n))])
        q = df.lazy().filter(pl.col("v0") > thr).group_by("id").agg(pl.col("v0").sum(), pl.col("v1").sum())
        info = {}
        t, out = _timed(lambda: q.collect(info=info), args.steps, args.warmup)
        print(json.dumps({"workload": f"filter + group_by(id: {card} groups).agg(2 x f64 sum)", "rows": n,
                          "ms": round(t * 1e3, 3), "Mrows_per_s": round(n / t / 1e6, 1), "groups": out.height,
                          "path": info.get("path")}), flush=True)
        del df, q, out
        torch.cuda.empty_cache()

    if "join" in only:
        nb = max(1, n // 100)
        # build: unique (sym, day) tuples; probe tuples hit ~50%
        bs = torch.arange(nb, device=dev, dtype=torch.int64)
        build = pl.DataFrame([pl.Series.from_torch("sym", bs // 1000), pl.Series.from_torch("day", bs % 1000),
                              pl.Series.from_torch("bv", floats(nb))])
        ps = ints(0, 2 * nb, n)
        probe = pl.DataFrame([pl.Series.from_torch("sym", ps // 1000), pl.Series.from_torch("day", ps % 1000),
                              pl.Series.from_torch("pv", floats(n))])
        del ps
        t, out = _timed(lambda: probe.join(build, on=["sym", "day"]), args.steps, args.warmup)
        print(json.dumps({"workload": "inner join on (sym, day), output sym, day, pv, bv", "probe_rows": n,
                          "build_rows": nb, "ms": round(t * 1e3, 3), "Mrows_per_s": round(n / t / 1e6, 1),
                          "output_rows": out.height}), flush=True)
        del probe, build, out
        torch.cuda.empty_cache()

    if "sort" in only:
        df = pl.DataFrame([pl.Series.from_torch("day", ints(0, 250, n)), pl.Series.from_torch("ts", ints(0, 1 << 30, n)),
                           pl.Series.from_torch("px", floats(n)), pl.Series.from_torch("qty", ints(0, 1000, n))])
        t, out = _timed(lambda: df.sort("day", "ts"), args.steps, args.warmup)
        print(json.dumps({"workload": "sort by (day, ts), 4 columns", "rows": n, "ms": round(t * 1e3, 3),
                          "Mrows_per_s": round(n / t / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
