"""Host -> HBM ingestion rate of Arrow RecordBatches (the plugin's scan).

    python tools/bench_ingest.py [--rows 1e8 --chunk 1048576 --reps 3]

An OHLCV-shaped table (symbol i64, open/high/low/close f64 with 1 % nulls
in `close`) is cut into RecordBatches of --chunk rows, the form in which
PyDataFrame.to_arrow hands a frame over (crates/polars-python/src/
dataframe/export.rs:80).  Times (the pinned-staging and page-registering
copy modes measured in profiles/r02_ingest.jsonl were removed from the
library as no faster, see polaroid_amd/csrc/ingest.hip):
  staged_ms  DataFrame.from_batches: plgpu_column_alloc + plgpu_ingest_chunk
          per chunk and column (bitmaps placed on the device), one
          synchronisation at the end;
  pageable one hipMemcpy per whole column from pageable host memory
          (plgpu_memcpy_h2d) after a host concatenation, the round-1 path
          without its host bitmap repacking.
Prints one JSON line; bytes = value + validity bytes moved to HBM.
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
    ap.add_argument("--chunk", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import pyarrow as pa

    import polaroid_amd as pl
    from polaroid_amd import _native as N

    n = int(args.rows)
    rng = np.random.default_rng(0)
    cols = {"symbol": pa.array(rng.integers(0, 100, n).astype(np.int64))}
    for c in ("open", "high", "low"):
        cols[c] = pa.array(rng.random(n) * 500)
    cols["close"] = pa.array(rng.random(n) * 500, mask=rng.random(n) < 0.01)
    table = pa.table(cols)
    batches = table.to_batches(max_chunksize=args.chunk)
    nbytes = n * 8 * 5 + (n + 7) // 8
    pl.DataFrame.from_batches(batches[:2])  # warm: library, pinned staging, allocator
    staged = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        df = pl.DataFrame.from_batches(batches)
        staged.append(time.perf_counter() - t0)
        del df
    # reference point: whole-column pageable copies of host-concatenated buffers
    flat = {k: table.column(k).combine_chunks() for k in table.column_names}
    pageable = []
    for _ in range(args.reps):
        bufs = []
        t0 = time.perf_counter()
        for k, a in flat.items():
            vb = a.buffers()[1]
            d = N.DeviceBuffer(n * 8)
            N.check(N.lib().plgpu_memcpy_h2d(C.c_void_p(d.ptr), C.c_void_p(vb.address), n * 8, None))
            bufs.append(d)
        pageable.append(time.perf_counter() - t0)
        del bufs
    ts, tp = min(staged), min(pageable)
    print(json.dumps({
        "bench": "arrow ingestion host->HBM", "mode": "pageable", "rows": n, "chunk_rows": args.chunk, "batches": len(batches),
        "bytes": nbytes, "staged_ms": round(ts * 1e3, 2), "staged_GBps": round(nbytes / ts / 1e9, 2),
        "pageable_whole_column_ms": round(tp * 1e3, 2), "pageable_GBps": round(n * 40 / tp / 1e9, 2),
    }), flush=True)


if __name__ == "__main__":
    main()
