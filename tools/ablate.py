"""Timing variants of the fused group-by kernel on the headline query.

    python tools/ablate.py ROWS MODE [MODE ...]

A MODE is an integer (PLGPU_ABLATE: kernel ablations whose results are
wrong on purpose, only main_kernel_ms matters), `base`, or `K=V;K=V`
environment settings (e.g. `PLGPU_OCC_GRID=2`, `PLGPU_NO_LIMB2=1`).  Modes
run interleaved in one process, 6 rounds, first round discarded
(cdna_hip_programming.md §5.4 rule 24)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import polaroid_amd as pl  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else int(1e9)
modes = sys.argv[2:] or ["base"]
KNOBS = ("PLGPU_ABLATE", "PLGPU_NO_FAST", "PLGPU_NO_SUMONLY", "PLGPU_OCC_GRID", "PLGPU_NO_LIMB2", "PLGPU_FAST_THREADS")
sym, cols = bench.make_data(torch, n, 100, 1234)
df = pl.DataFrame([pl.Series.from_torch("symbol", sym)] + [pl.Series.from_torch(k, v) for k, v in cols.items()])
q = df.lazy().filter(pl.col("close") > bench.THRESHOLD).group_by("symbol").agg(
    *[pl.col(k).sum() for k in ("open", "high", "low", "close")])
res = {m: [] for m in modes}
for rnd in range(6):
    for m in modes:
        for k in KNOBS:
            os.environ.pop(k, None)
        if m != "base":
            for kv in m.split(";"):
                if kv.isdigit():
                    os.environ["PLGPU_ABLATE"] = kv
                else:
                    k, v = kv.split("=")
                    os.environ[k] = v
        info = {}
        q.collect(info=info)
        if rnd > 0:
            res[m].append(info["main_kernel_ms"])
        if rnd == 1:
            print(m, {k: info[k] for k in ("grid", "path", "sum_limbs", "reruns", "lds_slots")}, flush=True)
for m in modes:
    v = res[m]
    print(f"mode {m:24s} median {np.median(v):8.3f} ms  min {min(v):8.3f}  -> "
          f"{40 * n / (np.median(v) * 1e-3) / 1e9:7.1f} GB/s")
