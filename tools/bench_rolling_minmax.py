"""rolling_min / rolling_max over 1e9 f64 rows, one GPU, inputs in HBM.

    python tools/bench_rolling_minmax.py [--rows 1e9 --windows 20,1000]

Prints one JSON line per (kind, window): ms per call and the HBM rate of
the algorithmic bytes (8 B read + 8 B written + validity per row)."""
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
    ap.add_argument("--windows", default="20,1000")
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()
    import torch

    import polaroid_amd as pl

    n = int(args.rows)
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    x = torch.randn(n, dtype=torch.float64, device="cuda", generator=g)
    s = pl.Series.from_torch("x", x)
    for w in (int(v) for v in args.windows.split(",")):
        for kind in ("min", "max"):
            fn = getattr(s, "rolling_" + kind)
            out = fn(w)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                out = fn(w)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / args.steps
            print(json.dumps({"op": f"rolling_{kind}({w})", "rows": n, "ms": round(dt * 1e3, 3),
                              "algorithmic_GBps": round(n * 16.125 / dt / 1e9, 1),
                              "path": "direct" if w <= 64 else "van Herk blocks"}), flush=True)
            del out


if __name__ == "__main__":
    main()
