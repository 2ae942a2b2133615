"""The filter leg's scatter against the state of the device memory it
allocates its outputs from (round-5 verdict item 6): the headline frame's
filter(close > 250) timed

  A  from a returned pool (plgpu release_cached + torch empty_cache),
  B  right after the nulls / keys / many-groups legs' allocations (their
     blocks left cached in the library's pool),
  C  after B with the pool returned again,
  D<m> the pool returned and a block of m MiB + 4 KiB held (placement probe),
  S  the same columns copied into one block at staggered starts,

each 5 steps after 2 warm-ups, one JSON line per state with the scatter and
mask kernel times (HIP events) and the pool's cached bytes before the state.

    python tools/filter_pool_ab.py [--rows 1e9]
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
    ap.add_argument("--states", default="A,B,C")
    args = ap.parse_args()
    import torch

    import bench
    import polaroid_amd as pl

    n = int(args.rows)
    sym, cols = bench.make_data(torch, n, 100, seed=1234)
    df = pl.DataFrame([pl.Series.from_torch("symbol", sym)] + [pl.Series.from_torch(c, t) for c, t in cols.items()])

    # S: the same columns copied to staggered starts (column i at i * 2 MiB +
    # i * 4 KiB past a 2 MiB boundary of one shared block), so the five
    # streams do not share their start offsets modulo any large power of two
    stag = None

    def staggered():
        names = ["symbol"] + list(cols)
        src = [sym] + list(cols.values())
        step = n + (1 << 18) + 512
        blk = torch.empty(step * len(src), dtype=torch.int64, device="cuda")
        out = []
        for i, (nm, t) in enumerate(zip(names, src)):
            o = i * step + i * 512
            v = blk[o:o + n].view(t.dtype)
            v.copy_(t)
            out.append(pl.Series.from_torch(nm, v))
        return pl.DataFrame(out), blk

    def run(tag, frame=None):
        r = bench.filter_leg(torch, pl, frame if frame is not None else df, 5, 2, 0, 0.0, True)
        k = r["kernels"]
        print(json.dumps({"state": tag, "ms_per_step": r["ms_per_step"],
                          "scatter_ms": k.get("filter_scatter8_kernel", {}).get("ms_mean"),
                          "mask_ms": k.get("filter_mask_kernel", {}).get("ms_mean"),
                          "pool_cached_GB": round(pl._native.pool_cached() / 1e9, 2)
                          if hasattr(pl._native, "pool_cached") else None}), flush=True)

    hold = []
    for st in args.states.split(","):
        if st == "S":
            if stag is None:
                stag = staggered()
            r_frame = stag[0]
            run("S", r_frame)
            continue
        if st in ("A", "C"):
            torch.cuda.empty_cache()
            pl._native.release_cached()
        elif st.startswith("D"):
            # placement probe: the pool returned, then a held block of
            # st[1:] MiB + 4 KiB shifts where the outputs land
            hold.clear()
            torch.cuda.empty_cache()
            pl._native.release_cached()
            hold.append(torch.empty((int(st[1:]) << 20) + 4096, dtype=torch.uint8, device="cuda"))
        elif st == "B":
            bench.nulls_leg(torch, pl, sym, cols, 2, 1, 6.6)
            bench.keys_leg(torch, pl, sym, cols, 2, 1, 6.6)
            bench.many_groups_leg(torch, pl, cols, 2, 1, [1_000_000, 10_000_000], 0, 0.0, True)
        run(st)


if __name__ == "__main__":
    main()
