"""The headline query on symbol-sorted rows (all rows of one symbol
together, as a frame sorted by (symbol, time) holds them) against the
default random order, 1e9 rows, single GPU: total and fused-kernel ms."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
import polaroid_amd as pl  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else int(1e9)
mixed = len(sys.argv) > 2 and sys.argv[2] == "mixed"  # min / max / count next to sums
sym, cols = bench.make_data(torch, n, 100, seed=1234)
aggs = [pl.col(k).sum() for k in ("open", "high", "low", "close")]
if mixed:
    aggs = [pl.col("open").sum(), pl.col("high").max(), pl.col("low").min(), pl.col("close").count()]
for order in ("random", "sorted"):
    if order == "sorted":
        perm = torch.sort(sym, stable=True).indices
        sym = sym[perm]
        cols = {k: v[perm] for k, v in cols.items()}
        del perm
    df = pl.DataFrame([pl.Series.from_torch("symbol", sym)] + [pl.Series.from_torch(k, v) for k, v in cols.items()])
    q = df.lazy().filter(pl.col("close") > bench.THRESHOLD).group_by("symbol").agg(*aggs)
    res = []
    for i in range(4):
        info = {}
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = q.collect(info=info)
        torch.cuda.synchronize()
        res.append(((time.perf_counter() - t0) * 1e3, info["main_kernel_ms"]))
    print(order, "mixed" if mixed else "sums", "total / kernel ms:", [(round(a, 2), round(b, 2)) for a, b in res[1:]], "groups", out.height, flush=True)
