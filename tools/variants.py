"""Interleaved timing of fast-kernel configuration variants (env-driven)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import polaroid_amd as pl  # noqa: E402

n = int(float(sys.argv[1]))
variants = [dict(kv.split("=") for kv in v.split(":") if kv) for v in sys.argv[2].split(",")]
sym, cols = bench.make_data(torch, n, 100, 1234)
df = pl.DataFrame([pl.Series.from_torch("symbol", sym)] + [pl.Series.from_torch(k, v) for k, v in cols.items()])
q = df.lazy().filter(pl.col("close") > bench.THRESHOLD).group_by("symbol").agg(
    *[pl.col(k).sum() for k in ("open", "high", "low", "close")])
keys = sorted({k for v in variants for k in v})
res = [[] for _ in variants]
ref = None
for rnd in range(6):
    for i, v in enumerate(variants):
        for k in keys:
            os.environ.pop(k, None)
        os.environ.update(v)
        info = {}
        out = q.collect(info=info)
        o = np.argsort(out["symbol"].to_numpy())
        got = out["close"].to_numpy()[o]
        if ref is None:
            ref = got
        assert np.array_equal(got.view(np.uint64), ref.view(np.uint64)), v
        if rnd > 0:
            res[i].append(info["main_kernel_ms"])
for v, r in zip(variants, res):
    print(f"{str(v):60s} median {np.median(r):8.3f} ms -> {40 * n / (np.median(r) * 1e-3) / 1e9:7.1f} GB/s")
