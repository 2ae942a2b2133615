"""A/B of the many-groups partition passes (groupby.hip gb_part_count /
gb_part_scatter) on tools/bench_multikey.py's two workloads, price-like
values, 1e9 rows:

  (sym, day): filter(v0 > 255).group_by("sym", "day").agg(v0.sum(), v1.sum())  25,000 groups
  id        : filter(v0 > 255).group_by("id").agg(v0.sum(), v1.sum())          100,000 groups

    python tools/ab_many_groups.py [ROWS] [MODE ...]

A MODE is `K=V;K=V` over PLGPU_* switches without the prefix (PART_XCD=1:
XCD-aware chunk order; PART_G=N: partition workgroups), or `base`.  Modes
run interleaved, 4 rounds with the first discarded; every mode's result must
equal the base mode's exactly (the f64 sums are exact, so bit-identical)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import polaroid_amd as pl  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else int(1e9)
modes = sys.argv[2:] or ["base", "PART_XCD=1"]
KNOBS = ("PLGPU_PART_XCD", "PLGPU_PART_G", "PLGPU_PART_LDS_KB", "PLGPU_PART_WGS_PER_CU", "PLGPU_PART_RACC")


def set_mode(m):
    for k in KNOBS:
        os.environ.pop(k, None)
    if m != "base":
        for kv in m.split(";"):
            k, v = kv.split("=")
            os.environ["PLGPU_" + k] = v


g = torch.Generator(device="cuda")
g.manual_seed(5)


def ints(lo, hi):
    return torch.randint(lo, hi, (n,), device="cuda", generator=g, dtype=torch.int64)


def prices():
    return torch.rand(n, device="cuda", generator=g, dtype=torch.float64) * 490 + 10


def canon(df, keys):
    s = df.sort(*keys)
    return [s[c].to_torch() for c in s.columns]


for name, keys, card in (("(sym, day)", ["sym", "day"], None), ("id", ["id"], 100_000)):
    if card is None:
        cols = [pl.Series.from_torch("sym", ints(0, 100)), pl.Series.from_torch("day", ints(0, 250))]
    else:
        cols = [pl.Series.from_torch("id", ints(0, card))]
    df = pl.DataFrame(cols + [pl.Series.from_torch("v0", prices()), pl.Series.from_torch("v1", prices())])
    q = df.lazy().filter(pl.col("v0") > 255.0).group_by(*keys).agg(pl.col("v0").sum(), pl.col("v1").sum())
    ref = None
    res = {m: [] for m in modes}
    for rnd in range(4):
        for m in modes:
            set_mode(m)
            info = {}
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = q.collect(info=info)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) * 1e3
            if rnd > 0:
                res[m].append(dt)
            if rnd == 0:
                c = canon(out, keys)
                if ref is None:
                    ref = c
                    print(f"{name}: {out.height} groups, path {info.get('path')}", flush=True)
                else:
                    assert all(torch.equal(a, b) for a, b in zip(c, ref)), f"{name} mode {m}: result differs"
            del out
    for m in modes:
        print(f"{name:10s} mode {m:28s} median {np.median(res[m]):8.3f} ms  min {min(res[m]):8.3f}", flush=True)
    set_mode("base")
    del df, q, ref
    torch.cuda.empty_cache()
