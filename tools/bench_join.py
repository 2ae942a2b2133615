"""Join workload of BASELINE.json configs[3]: 1e9-row probe x 1e7-row build
hash inner join on an i64 key, one GPU, inputs resident in HBM.

    python tools/bench_join.py [--probe 1e9 --build 1e7 --steps 5 --warmup 1]

A step = `probe.join(build, on="k")` materialised: the build table, the
ordered probe and the gather of k, the probe payload and the build payload.
Build keys are a random 1e7-subset of [0, 2e7); probe keys are uniform on
[0, 2e7), so half of the probe rows match exactly one build row.
Prints one JSON line.

With --dist (under `python -m torch.distributed.run --nproc-per-node N`):
every rank holds --probe rows of the probe side and --build / N rows of the
build side, and the step is polaroid_amd.distributed.join (RCCL; "auto"
broadcasts the 1e7-row build side, so the probe never moves: weak scaling);
the time is the max over ranks between barriers and `value` counts the
probe rows of all ranks.
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
    ap.add_argument("--probe", type=float, default=1e9)
    ap.add_argument("--build", type=float, default=1e7)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--dist", action="store_true")
    ap.add_argument("--strategy", default="auto")
    ap.add_argument("--how", default="inner", help="inner / left / right / full / semi / anti")
    ap.add_argument("--order", default="none", help="maintain_order")
    ap.add_argument("--payloads", type=int, default=1, help="build payload columns (8-byte, null-free)")
    args = ap.parse_args()
    import torch

    import polaroid_amd as pl

    n, m = int(args.probe), int(args.build)
    if args.dist:
        return dist_main(args, n, m)
    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    pk = torch.empty(n, dtype=torch.int64, device="cuda")
    pv = torch.empty(n, dtype=torch.float64, device="cuda")
    chunk = 1 << 27
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        pk[s:e] = torch.randint(0, 2 * m, (e - s,), device="cuda", generator=g)
        pv[s:e] = torch.rand(e - s, device="cuda", generator=g, dtype=torch.float64)
    bk = torch.randperm(2 * m, device="cuda", generator=g)[:m].to(torch.int64)
    bvs = [torch.rand(m, device="cuda", generator=g, dtype=torch.float64) for _ in range(args.payloads)]
    probe = pl.DataFrame([pl.Series.from_torch("k", pk), pl.Series.from_torch("pv", pv)])
    build = pl.DataFrame([pl.Series.from_torch("k", bk)] +
                         [pl.Series.from_torch(f"bv{i}" if i else "bv", t) for i, t in enumerate(bvs)])
    out = None
    kw = dict(on="k", how=args.how, maintain_order=args.order)
    from polaroid_amd import _native as N

    for _ in range(args.warmup):
        out = probe.join(build, **kw)
    torch.cuda.synchronize()
    prev = N.set_option("ktime", 1)
    N.ktime_read(reset=True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = probe.join(build, **kw)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    kt = N.ktime_read(reset=True)
    N.set_option("ktime", prev)
    rows_out = out.height
    print(json.dumps({
        "metric": f"Mrows/sec hash {args.how}-join probe (1e9 probe x 1e7 build, i64 key), materialised",
        "value": round(n / dt / 1e6, 1), "unit": "Mrows/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(dt * 1e3, 3), "higher_is_better": True,
        "dtype": "int64", "data": "synthetic keys/payloads generated on device",
        "config": {"workload": f"probe.join(build, on='k', how='{args.how}', maintain_order='{args.order}'), "
                               "output every column", "probe_rows": n,
                   "build_rows": m, "output_rows": rows_out, "build_payloads": args.payloads},
        "kernels": {k: round(ms / args.steps, 4) for k, (ms, c) in kt.items()},
    }), flush=True)


def dist_main(args, n, m):
    import torch
    import torch.distributed as dist

    import polaroid_amd as pl
    from polaroid_amd import distributed as D

    rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", 0)))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    dist.init_process_group("nccl", rank=rank, world_size=world)
    g = torch.Generator(device="cuda")
    g.manual_seed(7)  # the same build-key permutation on every rank
    bk_all = torch.randperm(2 * m, device="cuda", generator=g)[:m].to(torch.int64)
    lo, hi = rank * m // world, (rank + 1) * m // world
    bk = bk_all[lo:hi].clone()
    del bk_all
    g.manual_seed(100 + rank)
    pk = torch.empty(n, dtype=torch.int64, device="cuda")
    pv = torch.empty(n, dtype=torch.float64, device="cuda")
    chunk = 1 << 27
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        pk[s:e] = torch.randint(0, 2 * m, (e - s,), device="cuda", generator=g)
        pv[s:e] = torch.rand(e - s, device="cuda", generator=g, dtype=torch.float64)
    bv = torch.rand(hi - lo, device="cuda", generator=g, dtype=torch.float64)
    probe = pl.DataFrame([pl.Series.from_torch("k", pk), pl.Series.from_torch("pv", pv)])
    build = pl.DataFrame([pl.Series.from_torch("k", bk), pl.Series.from_torch("bv", bv)])
    info = {}
    out = None
    for _ in range(args.warmup):
        out = D.join(probe, build, on="k", strategy=args.strategy, info=info)
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = D.join(probe, build, on="k", strategy=args.strategy, info=info)
    torch.cuda.synchronize()
    dt = torch.tensor([(time.perf_counter() - t0) / args.steps], dtype=torch.float64, device="cuda")
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    rows = torch.tensor([out.height], dtype=torch.int64, device="cuda")
    dist.all_reduce(rows)
    if rank == 0:
        t = float(dt.item())
        print(json.dumps({
            "metric": "Mrows/sec hash inner-join probe (1e9 probe x 1e7 build, i64 key), materialised",
            "value": round(world * n / t / 1e6, 1), "unit": "Mrows/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(t * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "dtype": "int64", "data": "synthetic keys/payloads generated on device",
            "config": {"workload": "distributed.join(probe, build, on='k') inner, output k, pv, bv",
                       "probe_rows_per_gpu": n, "build_rows_total": m, "strategy": info.get("strategy"),
                       "output_rows": int(rows.item())},
        }), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
