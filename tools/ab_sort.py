"""A/B of the radix sort's downsweep shapes on configs[2]'s key column.

    python tools/ab_sort.py [ROWS] [MODE ...]

A MODE is `K=V;K=V` over the sort's PLGPU_SORT_* switches (today XCD:
PLGPU_SORT_XCD=0 = round-robin tiles in the downsweep; "XCD=1" is the
default).  Earlier switches measured with it and removed:
DT (512-thread downsweep shapes) and RANK (batched leader atomics).  Modes run interleaved in one process, 5 rounds with the first
discarded; every mode's permutation must equal the first mode's (stable sort:
the permutation is unique).  Key: shuffled timestamps < 2^40 as in
tools/bench_sort_rolling.py, so 5 radix passes run.  Prints per-mode median
arg_sort ms, then the whole 8-column df.sort of the default mode."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import polaroid_amd as pl  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else int(1e9)
modes = sys.argv[2:] or ["XCD=0", "XCD=1"]


def set_mode(m):
    for k in ("PLGPU_SORT_XCD",):
        os.environ.pop(k, None)
    for kv in filter(None, m.split(";")):
        k, v = kv.split("=")
        os.environ["PLGPU_SORT_" + k] = v


g = torch.Generator(device="cuda")
g.manual_seed(11)
ts = torch.empty(n, dtype=torch.int64, device="cuda")
chunk = 1 << 27
for s in range(0, n, chunk):
    e = min(n, s + chunk)
    ts[s:e] = torch.randint(0, 1 << 40, (e - s,), device="cuda", generator=g)
key = pl.Series.from_torch("ts", ts)
ref = None
res = {m: [] for m in modes}
for rnd in range(5):
    for m in modes:
        set_mode(m)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        p = key.arg_sort()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if rnd > 0:
            res[m].append(dt * 1e3)
        if rnd == 0:
            pt = p.to_torch()
            if ref is None:
                ref = pt.clone()
                srt = ts[ref.long()]
                assert bool((srt[1:] >= srt[:-1]).all()), "not sorted"
                eq = srt[1:] == srt[:-1]
                assert bool((ref[1:][eq] > ref[:-1][eq]).all()), "not stable"
            else:
                assert torch.equal(pt, ref), f"mode {m}: permutation differs"
        del p
for m in modes:
    print(f"arg_sort mode {m:16s} median {np.median(res[m]):8.3f} ms  min {min(res[m]):8.3f}", flush=True)
set_mode("")
del ref
cols = {"ts": ts}
for k in ("sym", "qty", "flags"):
    cols[k] = torch.randint(0, 1 << 20, (n,), device="cuda", generator=g, dtype=torch.int64)
for k in ("price", "bid", "ask", "vol"):
    cols[k] = 100 + torch.rand(n, device="cuda", generator=g, dtype=torch.float64) * 50
df = pl.DataFrame([pl.Series.from_torch(k, v) for k, v in cols.items()])
ts_ = []
for rnd in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = df.sort("ts")
    torch.cuda.synchronize()
    ts_.append((time.perf_counter() - t0) * 1e3)
    del out
print(f"df.sort (8 columns) ms: {[round(x, 2) for x in ts_]}", flush=True)
