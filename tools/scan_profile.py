"""Where the plugin's cold scan goes (bench.py's plugin leg table: 1e8 rows,
5 columns, 8M-row RecordBatches, 4 GB): device allocation, the per-chunk
host -> HBM copies, and the synchronisation, each timed on its own, for a
fresh allocation (hipMalloc) and for pooled memory.

    python tools/scan_profile.py [--rows 1e8 --chunk 8388608 --reps 3]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=float, default=1e8)
    ap.add_argument("--chunk", type=int, default=1 << 23)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--warm-copy-mb", type=int, default=0,
                    help="one host -> device copy of this many MB (fresh host and device buffers) first")
    ap.add_argument("--no-torch", action="store_true")
    args = ap.parse_args()
    import pyarrow as pa

    from polaroid_amd import _native as N
    from polaroid_amd.frame import _ingest_chunks

    rows = int(args.rows)
    rng = np.random.default_rng(7)
    k = rng.integers(0, 100, rows)
    cols = {"symbol": (k * 7919 + 1_000_000).astype(np.int64)}
    for c in ("open", "high", "low", "close"):
        cols[c] = rng.uniform(10, 490, rows)
    table = pa.table(cols)
    batches = table.to_batches(max_chunksize=args.chunk)
    names = list(cols)
    nbytes = sum(a.nbytes for a in cols.values())
    lib = N.lib()
    if args.warm_copy_mb:
        w = np.ones(args.warm_copy_mb << 17)
        dp = C.c_void_p()
        N.check(lib.plgpu_alloc(C.byref(dp), w.nbytes, None))
        t0 = time.perf_counter()
        N.check(lib.plgpu_memcpy_h2d(dp, w.ctypes.data, w.nbytes, None))
        N.check(lib.plgpu_synchronize(None))
        print(json.dumps({"warm_copy_mb": args.warm_copy_mb, "ms": round((time.perf_counter() - t0) * 1e3, 3)}),
              flush=True)
        N.check(lib.plgpu_free(dp, None))
    for rep in range(args.reps):
        N.check(lib.plgpu_synchronize(None))
        t = {}
        t0 = time.perf_counter()
        outs = []
        for nm in names:
            col = N.Column()
            N.check(lib.plgpu_column_alloc(N.F64 if nm != "symbol" else N.I64, rows, 0, 0, C.byref(col), None))
            outs.append(col)
        N.check(lib.plgpu_synchronize(None))
        t["alloc_ms"] = (time.perf_counter() - t0) * 1e3
        t1 = time.perf_counter()
        for j, nm in enumerate(names):
            row = 0
            for b in batches:
                a = b.column(j)
                bufs = a.buffers()
                N.check(lib.plgpu_ingest_chunk(C.byref(outs[j]), row, 0, bufs[1].address, None, None, a.offset,
                                               len(a), None))
                row += len(a)
        t["copy_issue_ms"] = (time.perf_counter() - t1) * 1e3
        N.check(lib.plgpu_synchronize(None))
        t["copy_ms"] = (time.perf_counter() - t1) * 1e3
        t["copy_GBs"] = nbytes / (t["copy_ms"] * 1e-3) / 1e9
        for col in outs:
            lib.plgpu_column_release(C.byref(col))
        # the product path: _ingest_chunks per column (one sync per column)
        t2 = time.perf_counter()
        series = [_ingest_chunks(nm, [b.column(j) for b in batches], batches[0].schema.field(j).type)
                  for j, nm in enumerate(names)]
        N.check(lib.plgpu_synchronize(None))
        t["ingest_chunks_ms"] = (time.perf_counter() - t2) * 1e3
        del series
        if rep == 0:
            t["note"] = "rep 0: fresh device memory (hipMalloc); later reps: pooled"
        print(json.dumps({"rep": rep, "rows": rows, "bytes": nbytes, "batches": len(batches),
                          **{k: round(v, 3) if isinstance(v, float) else v for k, v in t.items()}}), flush=True)
        N.release_cached()
    # fresh device memory: first writes by the host-link copy vs a device
    # memset first (torch tensors, never freed during the test, so every
    # allocation is a new hipMalloc)
    if args.no_torch:
        return
    import torch

    keep = []
    src = [torch.from_numpy(cols[c]) for c in names]
    for mode in ("fresh", "memset_first", "fresh", "memset_first"):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dst = [torch.empty(rows, dtype=torch.float64 if c != "symbol" else torch.int64, device="cuda") for c in names]
        if mode == "memset_first":
            for d in dst:
                d.zero_()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for d, s_ in zip(dst, src):
            d.copy_(s_)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        keep.append(dst)
        print(json.dumps({"mode": mode, "alloc_prep_ms": round((t1 - t0) * 1e3, 3), "copy_ms": round((t2 - t1) * 1e3, 3),
                          "copy_GBs": round(nbytes / (t2 - t1) / 1e9, 2)}), flush=True)


if __name__ == "__main__":
    main()
