"""rolling_sum / rolling_mean alone over one resident f64 column (the
rolling half of BASELINE configs[2]); for kernel profiles.

    python tools/bench_rolling.py [--rows 1e9 --window 20 --kind mean --steps 5]

Prints one JSON line: ms per call (host-timed, synchronised) and the
algorithmic rate (8 B in + 8 B out per row)."""
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
    ap.add_argument("--kind", default="mean")
    ap.add_argument("--center", action="store_true")
    ap.add_argument("--data", default="price", help="price (100..150) | mixed (40 binades, mixed signs)")
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    import torch

    import polaroid_amd as pl

    n = int(args.rows)
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    if args.data == "price":
        x = 100 + torch.rand(n, device="cuda", generator=g, dtype=torch.float64) * 50
    else:
        x = torch.randn(n, device="cuda", generator=g, dtype=torch.float64)
        x *= torch.exp2(torch.randint(-20, 20, (n,), device="cuda", generator=g).to(torch.float64))
    from polaroid_amd import _native as N

    s = pl.Series.from_torch("x", x)
    fn = getattr(s, "rolling_" + args.kind)
    fn(args.window, center=args.center)
    torch.cuda.synchronize()
    N.set_option("ktime", 1)
    N.ktime_read(reset=True)
    ts = []
    for _ in range(args.steps):
        t0 = time.perf_counter()
        fn(args.window, center=args.center)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    kt = N.ktime_read(reset=True)
    t = min(ts)
    kern = {k: round(ms / max(c, 1), 4) for k, (ms, c) in kt.items()}
    km = max(kern.values()) if kern else None
    print(json.dumps({"rows": n, "window": args.window, "kind": args.kind, "center": args.center, "data": args.data,
                      "ms": round(t * 1e3, 3), "GBps_algorithmic": round(16 * n / t / 1e9, 1), "kernel_ms": kern,
                      "kernel_frac": round(16 * n / (km * 1e-3) / 1e9 / 8000.0, 4) if km else None,
                      "options": {k: v for k, v in os.environ.items() if k.startswith("PLGPU_")}}), flush=True)


if __name__ == "__main__":
    main()
