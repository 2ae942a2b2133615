"""The headline query over the key encodings of an OHLCV frame, 1e9 rows,
one GPU, inputs resident in HBM:

  int64        symbol: Int64 (the bench.py headline)
  categorical  symbol: Categorical (UInt32 codes + a 100-string dictionary)
  string       symbol: String (5-byte tickers, Arrow large_string)
  sym_day      group_by(symbol: Int64, day: Int32), days in row order

    python tools/bench_keys.py [--rows 1e9 --steps 10 --warmup 2 --only a,b]

One JSON line per case: ms per collect(), the fused kernel's HIP-event time
and the library's per-kernel times (plgpu_ktime_read) of the timed steps.
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
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--only", default="int64,categorical,string,sym_day")
    args = ap.parse_args()
    import torch

    import bench
    import polaroid_amd as pl
    from polaroid_amd import _native as N

    n = int(args.rows)
    sym, cols = bench.make_data(torch, n, 100, seed=1234)
    vals = [pl.Series.from_torch(nm, t) for nm, t in cols.items()]
    sums = [pl.col(c).sum() for c in ("open", "high", "low", "close")]
    pred = pl.col("close") > bench.THRESHOLD

    def frame(case):
        if case == "int64":
            return pl.DataFrame([pl.Series.from_torch("symbol", sym)] + vals), ("symbol",), []
        return bench.key_frame(torch, pl, sym, cols, case)

    for case in args.only.split(","):
        df, keys, keep = frame(case)
        q = df.lazy().filter(pred).group_by(*keys).agg(*sums)
        for _ in range(args.warmup):
            q.collect()
        torch.cuda.synchronize()
        prev = N.set_option("ktime", 1)
        N.ktime_read(reset=True)
        kms = []
        t0 = time.perf_counter()
        for _ in range(args.steps):
            info = {}
            out = q.collect(info=info)
            kms.append(info.get("main_kernel_ms"))
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.steps
        kt = N.ktime_read(reset=True)
        N.set_option("ktime", prev)
        print(json.dumps({
            "case": case, "rows": n, "groups": out.height, "ms_per_step": round(dt * 1e3, 3),
            "Mrows_s": round(n / dt / 1e6, 1), "fused_kernel_ms": round(sum(kms) / len(kms), 4),
            "key_pack": info.get("key_pack"), "categorical_codes": info.get("categorical_codes", 0),
            "path": info.get("path"), "local_range": info.get("local_range"),
            "kernels": {nm: round(ms / args.steps, 4) for nm, (ms, c) in kt.items()},
        }), flush=True)
        del df, q, out, keep
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
