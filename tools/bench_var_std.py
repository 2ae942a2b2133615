"""group_by(symbol).agg(close.std()) over --rows f64 rows (100 groups,
filter close > 250), one GPU, inputs in HBM, next to the plain sum query on
the same frame for the cost ratio of the composed passes (DESIGN.md
"Group variance / standard deviation").

    python tools/bench_var_std.py [--rows 1e9 --steps 3]
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
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--maintain-order", action="store_true")
    args = ap.parse_args()
    import torch

    import polaroid_amd as pl

    n = int(args.rows)
    g = torch.Generator(device="cuda")
    g.manual_seed(9)
    sym = torch.randint(0, 100, (n,), device="cuda", generator=g, dtype=torch.int64)
    close = torch.rand(n, device="cuda", generator=g, dtype=torch.float64) * 500
    df = pl.DataFrame([pl.Series.from_torch("symbol", sym), pl.Series.from_torch("close", close)])
    base = df.lazy().filter(pl.col("close") > 250.0).group_by("symbol", maintain_order=args.maintain_order)
    for name, q in (("sum", base.agg(pl.col("close").sum())), ("std", base.agg(pl.col("close").std())),
                    ("var", base.agg(pl.col("close").var(0)))):
        info = {}
        out = q.collect(info=info)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        kms = []
        for _ in range(args.steps):
            it = {}
            out = q.collect(info=it)
            kms.append(it.get("main_kernel_ms", float("nan")))
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.steps
        print(json.dumps({"query": f"filter(close > 250).group_by(symbol).agg(close.{name}())", "rows": n,
                          "groups": out.height, "ms": round(dt * 1e3, 3), "kernel_ms": round(sum(kms) / len(kms), 3),
                          "path": info.get("var_path"), "kernel_path": info.get("path"),
                          "maintain_order": args.maintain_order, "Mrows_per_s": round(n / dt / 1e6, 1)}), flush=True)
        del out


if __name__ == "__main__":
    main()
