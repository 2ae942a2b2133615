import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import torch
import polaroid_amd as pl
n = int(1e8)
g = torch.Generator(device="cuda"); g.manual_seed(9)
sym = torch.randint(0, 100, (n,), device="cuda", generator=g, dtype=torch.int64)
close = torch.rand(n, device="cuda", generator=g, dtype=torch.float64) * 500
df = pl.DataFrame([pl.Series.from_torch("symbol", sym), pl.Series.from_torch("close", close)])
for q in (pl.col("close").sum(), pl.col("close").std()):
    info = {}
    df.lazy().filter(pl.col("close") > 250.0).group_by("symbol").agg(q).collect(info=info)
    print(info, flush=True)
