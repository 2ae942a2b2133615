"""One of bench.py's resident-frame legs alone (for profilers): the
headline, vwap, std, filter or many_groups (--groups G random symbols) query over configs[1]'s 1e9-row frame.

    python tools/bench_legs.py --leg vwap [--rows 1e9 --steps 5 --warmup 2]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--leg", choices=["headline", "vwap", "std", "filter", "many_groups", "sort", "join", "nulls"], required=True)
    ap.add_argument("--rows", type=float, default=1e9)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--groups", type=int, default=100, help="distinct symbols (the headline's 100 by default)")
    args = ap.parse_args()
    import torch

    import bench
    import polaroid_amd as pl

    n = int(args.rows)
    if args.leg in ("sort", "join"):
        r = (bench.sort_leg if args.leg == "sort" else bench.join_leg)(torch, pl, args.steps, args.warmup)
        print(json.dumps({"leg": args.leg, **r}), flush=True)
        return
    sym, cols = bench.make_data(torch, n, args.groups, seed=1234)
    df = pl.DataFrame([pl.Series.from_torch("symbol", sym)] + [pl.Series.from_torch(c, t) for c, t in cols.items()])
    if args.leg == "vwap":
        r = bench.vwap_leg(torch, pl, df, sym, cols["close"], args.steps, args.warmup)
    elif args.leg == "filter":
        r = bench.filter_leg(torch, pl, df, args.steps, args.warmup, 0, 0.0, True)
    elif args.leg == "many_groups":
        del df
        r = bench.many_groups_leg(torch, pl, cols, args.steps, args.warmup, [args.groups], 0, 0.0, True)
    elif args.leg == "nulls":
        q = df.lazy().filter(pl.col("close") > bench.THRESHOLD).group_by("symbol").agg(
            *[pl.col(c).sum() for c in ("open", "high", "low", "close")])
        h = bench.timed_leg(torch, q, n, args.steps, args.warmup, 40)
        del q, df
        r = {"headline": h, **bench.nulls_leg(torch, pl, sym, cols, args.steps, args.warmup, h["ms_per_step"])}
    elif args.leg == "std":
        r = bench.std_leg(torch, pl, df, args.steps, args.warmup)
    else:
        q = df.lazy().filter(pl.col("close") > bench.THRESHOLD).group_by("symbol").agg(
            *[pl.col(c).sum() for c in ("open", "high", "low", "close")])
        r = bench.timed_leg(torch, q, n, args.steps, args.warmup, 40)
    print(json.dumps({"leg": args.leg, "groups": args.groups, **r}), flush=True)


if __name__ == "__main__":
    main()
