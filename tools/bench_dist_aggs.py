"""Cost of the composed multi-GPU group-by forms at 1e9 rows per rank
(run under torch.distributed.run; one JSON line per case from rank 0):
  sums      the headline partial-state exchange (bench.py's step)
  first_last  + first() / last() (run_first_last: values routed to owners)
  var_std   var / std (two partitioned passes + all-gathered means)
  two_keys  (symbol, day) packed into one code (plgpu_key_pack)
  float_key a Float64 key (canonical-bit codes + first() of the key)

    python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 \\
        tools/bench_dist_aggs.py [--rows 1e9 --steps 5]
"""

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=float, default=1e9)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    args = ap.parse_args()
    import torch
    import torch.distributed as dist

    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import bench
    import polaroid_amd as pl
    from polaroid_amd import distributed as D

    n = int(args.rows)
    sym, cols = bench.make_data(torch, n, 100, seed=1234 + dist.get_rank())
    day = (torch.arange(n, device="cuda", dtype=torch.int64) // (n // 250 + 1)).to(torch.int32)
    fk = (sym % 997).to(torch.float64) * 0.25
    df = pl.DataFrame([pl.Series.from_torch("symbol", sym), pl.Series.from_torch("day", day),
                       pl.Series.from_torch("fk", fk)] + [pl.Series.from_torch(k, v) for k, v in cols.items()])
    pred = pl.col("close") > bench.THRESHOLD
    sums = [pl.col(k).sum() for k in ("open", "high", "low", "close")]
    cases = {
        "sums": ("symbol", sums),
        "first_last": ("symbol", sums + [pl.col("open").first().alias("fo"), pl.col("close").last().alias("lc")]),
        "var_std": ("symbol", [pl.col("close").var().alias("v"), pl.col("open").std().alias("s")]),
        "two_keys": (("symbol", "day"), sums),
        "float_key": ("fk", sums),
    }
    for name, (key, aggs) in cases.items():
        for _ in range(args.warmup):
            D.group_by_agg(df, key, aggs, pred)
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            out = D.group_by_agg(df, key, aggs, pred)
        torch.cuda.synchronize()
        dist.barrier()
        ms = (time.perf_counter() - t0) / args.steps * 1e3
        if dist.get_rank() == 0:
            print(json.dumps({"case": name, "rows_per_rank": n, "world": dist.get_world_size(), "ms_per_step": round(ms, 3),
                              "groups_on_rank0": out.height}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
