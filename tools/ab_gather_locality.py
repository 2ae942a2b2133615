"""How much does source locality buy the packed row gather (plgpu_gather of
8 null-free 8-byte columns)?  Times the gather of a 1e9-row, 8-column frame
by index columns whose destination block j // B reads only source rows of
block j // B (random inside the block), for several block sizes B, against a
uniformly random index.  Prints one JSON line per variant.

    python tools/ab_gather_locality.py [--rows 1e9 --steps 3]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=float, default=1e9)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--blocks", default="0,22,20,18,16")
    args = ap.parse_args()
    import torch

    import polaroid_amd as pl
    from polaroid_amd import _native as N
    from polaroid_amd.frame import _col_array

    n = int(args.rows)
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    cols = [pl.Series.from_torch(f"c{k}", torch.randint(0, 1 << 40, (n,), device="cuda", generator=g))
            for k in range(8)]
    idx_t = torch.empty(n, dtype=torch.int32, device="cuda")
    chunk = 1 << 26
    for lb in [int(x) for x in args.blocks.split(",")]:
        for s in range(0, n, chunk):
            e = min(n, s + chunk)
            if lb < 0:
                idx_t[s:e] = torch.arange(s, e, device="cuda", dtype=torch.int32)
            elif lb == 0:
                idx_t[s:e] = torch.randint(0, n, (e - s,), device="cuda", generator=g, dtype=torch.int64).to(torch.int32)
            else:
                B = 1 << lb
                j = torch.arange(s, e, device="cuda", dtype=torch.int64)
                lo = (j >> lb) << lb
                span = torch.clamp(n - lo, max=B)
                r = torch.randint(0, 1 << 62, (e - s,), device="cuda", generator=g) % span
                idx_t[s:e] = (lo + r).to(torch.int32)
        idx = pl.Series.from_device("idx", pl.UInt32, idx_t.data_ptr(), n, None, keepalive=(idx_t,))
        ts = []
        for _ in range(args.steps + 1):
            out = (N.Column * 8)()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            N.check(N.lib().plgpu_gather(_col_array(cols), 8, C.byref(idx._col), out, None))
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
            for k in range(8):
                N.lib().plgpu_column_release(C.byref(out[k]))
        print(json.dumps({"block_log2": lb, "block_MB": (64 << lb) >> 20 if lb > 0 else None,
                          "gather_ms": round(min(ts[1:]) * 1e3, 3)}), flush=True)


if __name__ == "__main__":
    main()
