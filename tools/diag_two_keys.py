"""(symbol, day) group-by at 1e9 rows: the single-GPU multi-key path and,
under torch.distributed.run, the multi-GPU packed-key path, with their info
dicts.  Without RANK in the environment only the single-GPU case runs (for
rocprofv3, which must not wrap a launcher)."""
import os, sys, time, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, torch.distributed as dist
torch.cuda.set_device(0)
DIST = "RANK" in os.environ
if DIST:
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
import bench, polaroid_amd as pl
from polaroid_amd import distributed as D
n = int(1e9)
sym, cols = bench.make_data(torch, n, 100, seed=1234)
day = (torch.arange(n, device="cuda", dtype=torch.int64) // (n // 250 + 1)).to(torch.int32)
df = pl.DataFrame([pl.Series.from_torch("symbol", sym), pl.Series.from_torch("day", day)] + [pl.Series.from_torch(k, v) for k, v in cols.items()])
pred = pl.col("close") > bench.THRESHOLD
sums = [pl.col(k).sum() for k in ("open", "high", "low", "close")]
for name, fn in [("single_gpu", lambda info: df.lazy().filter(pred).group_by("symbol", "day").agg(*sums).collect(info=info)),
                 ("dist", lambda info: D.group_by_agg(df, ("symbol", "day"), sums, pred, info=info))][:2 if DIST else 1]:
    for i in range(3):
        info = {}
        torch.cuda.synchronize(); t0 = time.perf_counter(); out = fn(info); torch.cuda.synchronize()
        print(name, round((time.perf_counter() - t0) * 1e3, 2), out.height, json.dumps({k: v for k, v in info.items()}), flush=True)
if DIST:
    dist.destroy_process_group()
