"""Phase times of the multi-GPU group-by protocol at world 1 (RCCL) next to the
single-GPU query, 1e9 rows."""
import os, sys, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch, torch.distributed as dist
os.environ.setdefault("MASTER_ADDR", "127.0.0.1"); os.environ.setdefault("MASTER_PORT", "29555")
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
import bench, polaroid_amd as pl
from polaroid_amd import distributed as D
from polaroid_amd.frame import _gb_lower
n = int(1e9)
sym, cols = bench.make_data(torch, n, 100, 1234)
df = pl.DataFrame([pl.Series.from_torch("symbol", sym)] + [pl.Series.from_torch(k, v) for k, v in cols.items()])
aggs = [pl.col(k).sum() for k in ("open", "high", "low", "close")]
pred = pl.col("close") > 250.0
dev = torch.device("cuda", 0)
def T(): torch.cuda.synchronize(); return time.perf_counter()
for it in range(5):
    t0 = T()
    g = _gb_lower(df, "symbol", aggs, pred)
    part = D.GpuPartial(g, 1)
    t1 = T()
    bottoms = part.begin()
    t2 = T()
    t3 = T()
    send, counts = part.export()
    t4 = T()
    recv, nrec, rows = D.exchange_records(send, counts, part.record_words, header=[0] + bottoms)
    t5 = T()
    out, mi = part.merge(recv, [r[0] for r in rows], [r[2:] for r in rows])
    t6 = T()
    q = df.lazy().filter(pred).group_by("symbol").agg(*aggs); info = {}
    q.collect(info=info)
    t7 = T()
    print(f"lower {1e3*(t1-t0):.3f} begin {1e3*(t2-t1):.3f} (kernel {part.info.main_kernel_ms:.3f}) export {1e3*(t4-t3):.3f} exch {1e3*(t5-t4):.3f} merge {1e3*(t6-t5):.3f} | single {1e3*(t7-t6):.3f} (kernel {info['main_kernel_ms']:.3f})", flush=True)
dist.destroy_process_group()
