"""Input placement probe: the headline query and the filter over the
headline frame as generated (five separate 8 GB column blocks) and over the
same columns copied to staggered starts inside one block (column i at
i * (n + 2^18 + 512) words), in one process, alternating twice.

    python tools/stagger_probe.py [--rows 1e9]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=float, default=1e9)
    args = ap.parse_args()
    import torch

    import bench
    import polaroid_amd as pl

    n = int(args.rows)
    sym, cols = bench.make_data(torch, n, 100, seed=1234)
    names = ["symbol"] + list(cols)
    src = [sym] + list(cols.values())
    df = pl.DataFrame([pl.Series.from_torch(nm, t) for nm, t in zip(names, src)])
    step = n + (1 << 18) + 512
    blk = torch.empty(step * len(src), dtype=torch.int64, device="cuda")
    views = []
    for i, t in enumerate(src):
        v = blk[i * step:i * step + n].view(t.dtype)
        v.copy_(t)
        views.append(v)
    ds = pl.DataFrame([pl.Series.from_torch(nm, v) for nm, v in zip(names, views)])
    for rep in range(2):
        for tag, frame in (("separate", df), ("staggered", ds)):
            q = frame.lazy().filter(pl.col("close") > bench.THRESHOLD).group_by("symbol").agg(
                *[pl.col(c).sum() for c in ("open", "high", "low", "close")])
            h = bench.timed_leg(torch, q, n, 10, 3, 40)
            f = bench.filter_leg(torch, pl, frame, 5, 2, 0, 0.0, True)
            print(json.dumps({"rep": rep, "frame": tag, "headline_ms": h["ms_per_step"],
                              "headline_kernel_ms": h.get("kernel_ms"), "filter_ms": f["ms_per_step"],
                              "scatter_ms": f["kernels"].get("filter_scatter8_kernel", {}).get("ms_mean")}),
                  flush=True)
            del q


if __name__ == "__main__":
    main()
