"""Host-side cost of one headline query (filter -> group_by -> 4 sums) on a
tiny resident frame, where the kernels take microseconds: wall time per
collect() and a cProfile of the Python side.

    python tools/host_overhead.py [--rows 1e4 --calls 300]
"""
import argparse
import cProfile
import io
import json
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=float, default=1e4)
    ap.add_argument("--calls", type=int, default=300)
    ap.add_argument("--keys", default="symbol", help="symbol | sym_day (Int64 symbol + Int32 day, packed in the kernel)")
    args = ap.parse_args()
    import torch

    import polaroid_amd as pl

    n = int(args.rows)
    g = torch.Generator(device="cuda")
    g.manual_seed(1)
    sym = torch.randint(0, 100, (n,), device="cuda", generator=g)
    cols = {k: torch.rand(n, device="cuda", generator=g, dtype=torch.float64) * 500
            for k in ("open", "high", "low", "close")}
    series = [pl.Series.from_torch("symbol", sym)] + [pl.Series.from_torch(k, v) for k, v in cols.items()]
    by = ["symbol"]
    if args.keys == "sym_day":
        series.append(pl.Series.from_torch("day", (torch.arange(n, device="cuda") * 250 // n).to(torch.int32)))
        by = ["symbol", "day"]
    df = pl.DataFrame(series)
    q = df.lazy().filter(pl.col("close") > 250.0).group_by(*by).agg(
        *[pl.col(k).sum() for k in ("open", "high", "low", "close")])
    for _ in range(20):
        q.collect()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.calls):
        q.collect(info={})
    torch.cuda.synchronize()
    per = (time.perf_counter() - t0) / args.calls
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(args.calls):
        q.collect(info={})
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(18)
    print(json.dumps({"rows": n, "keys": args.keys, "ms_per_collect": round(per * 1e3, 4)}), flush=True)
    print(s.getvalue())


if __name__ == "__main__":
    main()
