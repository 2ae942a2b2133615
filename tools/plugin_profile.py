"""Where the plugin's time goes (bench.py's plugin leg, configs[1]'s 1e8
rows): the cold query (scan over the host link + query) and the warm query
(columns resident in the ColumnCache), each split into phases with device
synchronisations between them, plus a cProfile of the warm query.

    python tools/plugin_profile.py [--rows 1e8 --calls 20]
"""
import argparse
import cProfile
import io
import json
import os
import pstats
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=float, default=1e8)
    ap.add_argument("--calls", type=int, default=20)
    ap.add_argument("--prewarm", action="store_true", help="a small query first, then the pool released (bench.py's state)")
    args = ap.parse_args()
    import pyarrow as pa
    import torch

    import bench
    import ir_model
    from polaroid_amd import _native as N
    from polaroid_amd import polars_engine as PE
    from polaroid_amd.frame import LazyFrame

    rows = int(args.rows)
    rng = np.random.default_rng(7)
    base = rng.uniform(10, 490, 100)
    k = rng.integers(0, 100, rows)
    p = base[k]
    o = p * np.exp(0.02 * rng.standard_normal(rows))
    c = p * np.exp(0.02 * rng.standard_normal(rows))
    sp = rng.random(rows) * 0.01
    table = pa.table({"symbol": pa.array((k * 7919 + 1_000_000).astype(np.int64)), "open": pa.array(o),
                      "high": pa.array(np.maximum(o, c) * (1 + sp)), "low": pa.array(np.minimum(o, c) * (1 - sp)),
                      "close": pa.array(c)})
    del k, p, o, c, sp
    cols = ["open", "high", "low", "close"]
    nt = ir_model.filter_group_by_sum(table, "symbol", "close", bench.THRESHOLD, cols, chunk_rows=1 << 23)
    t0 = time.perf_counter()
    plan = PE.translate(nt)
    t_translate = time.perf_counter() - t0
    cache = PE.column_cache()
    cache.clear()

    def phases(label):
        torch.cuda.synchronize()
        t = {}
        t0 = time.perf_counter()
        bound = PE._bind_scans(plan, cache)
        N.check(N.lib().plgpu_synchronize(None))
        t["scan_ms"] = (time.perf_counter() - t0) * 1e3
        t1 = time.perf_counter()
        info = {}
        out = LazyFrame(bound).collect(info=info)
        N.check(N.lib().plgpu_synchronize(None))
        t["query_ms"] = (time.perf_counter() - t1) * 1e3
        t["fused_kernel_ms"] = info.get("main_kernel_ms")
        t2 = time.perf_counter()
        tab = out.to_arrow()
        t["to_arrow_ms"] = (time.perf_counter() - t2) * 1e3
        t["total_ms"] = (time.perf_counter() - t0) * 1e3
        print(json.dumps({"phase": label, "rows": rows, **{k: round(v, 3) if isinstance(v, float) else v
                                                          for k, v in t.items()}, "groups": tab.num_rows}),
              flush=True)

    if args.prewarm:
        # as inside bench.py: the library's code object loaded and the host
        # link's copy path initialised by earlier work in the process, its
        # memory pool released before the leg
        small = pa.table({c: table.column(c).slice(0, 1 << 20) for c in table.column_names})
        snt = ir_model.filter_group_by_sum(small, "symbol", "close", bench.THRESHOLD, cols, chunk_rows=1 << 20)
        PE.execute_with_polaroid(snt, None, to_frame=lambda t: t)
        snt.udf(None, None, None, False)
        cache.clear()
        N.release_cached()
    phases("cold")
    for i in range(3):
        phases(f"warm{i}")
    PE.execute_with_polaroid(nt, None, to_frame=lambda t: t)
    for _ in range(3):
        nt.udf(None, None, None, False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.calls):
        nt.udf(None, None, None, False)
    torch.cuda.synchronize()
    per = (time.perf_counter() - t0) / args.calls * 1e3
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(args.calls):
        nt.udf(None, None, None, False)
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumtime").print_stats(30)
    print(json.dumps({"udf_warm_ms": round(per, 3), "translate_ms": round(t_translate * 1e3, 3)}), flush=True)
    print(s.getvalue())


if __name__ == "__main__":
    main()
