"""Timing ablations of the fused group-by kernel (results are wrong in
ablation modes; only main_kernel_ms matters).  Interleaved rounds in one
process (cdna_hip_programming.md §5.4 rule 24)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import polaroid_amd as pl  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else int(1e9)
modes = [m for m in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["0", "1", "2", "3"])]
sym, cols = bench.make_data(torch, n, 100, 1234)
df = pl.DataFrame([pl.Series.from_torch("symbol", sym)] + [pl.Series.from_torch(k, v) for k, v in cols.items()])
q = df.lazy().filter(pl.col("close") > bench.THRESHOLD).group_by("symbol").agg(
    *[pl.col(k).sum() for k in ("open", "high", "low", "close")])
res = {m: [] for m in modes}
for rnd in range(6):
    for m in modes:
        os.environ["PLGPU_ABLATE"] = m
        for k in ("PLGPU_NO_FAST", "PLGPU_NO_SUMONLY"):
            os.environ.pop(k, None)
        if m.startswith("nofast"):
            os.environ["PLGPU_NO_FAST"] = "1"
            os.environ["PLGPU_ABLATE"] = "0"
        if m.startswith("nosumonly"):
            os.environ["PLGPU_NO_SUMONLY"] = "1"
            os.environ["PLGPU_ABLATE"] = "0"
        info = {}
        q.collect(info=info)
        if rnd > 0:
            res[m].append(info["main_kernel_ms"])
for m in modes:
    v = res[m]
    print(f"mode {m:8s} median {np.median(v):8.3f} ms  min {min(v):8.3f}  -> {40 * n / (np.median(v) * 1e-3) / 1e9:7.1f} GB/s")
