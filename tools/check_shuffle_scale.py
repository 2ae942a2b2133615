"""Scale check of the shuffle join's stages at world 1 (RCCL):
    python -m torch.distributed.run --nproc-per-node 1 tools/check_shuffle_scale.py [rows]
Compares row counts and key checksums after partition, pack, exchange and
unpack, and the join height against the single-GPU join."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist

    import polaroid_amd as pl
    from polaroid_amd import distributed as D

    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 500_000_000
    m = 10_000_000
    dist.init_process_group("nccl", rank=0, world_size=1)
    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    bk = torch.randperm(2 * m, device="cuda", generator=g)[:m].to(torch.int64)
    pk = torch.randint(0, 2 * m, (n,), device="cuda", generator=g)
    probe = pl.DataFrame([pl.Series.from_torch("k", pk)])
    build = pl.DataFrame([pl.Series.from_torch("k", bk)])
    ks = int(pk.sum().item())
    perm, counts = D.GpuJoinOps.partition(probe, ["k"], 1, False)
    print("partition", perm.len(), counts, flush=True)
    wire = D.GpuJoinOps.to_wire(probe, perm)
    print("pack sum ok", int(wire[0].values.sum().item()) == ks, flush=True)
    cols, nr = D.exchange_columns(wire, counts)
    print("exchange", nr, int(cols[0].values.sum().item()) == ks, flush=True)
    back = D.GpuJoinOps.from_wire(cols, nr)
    print("unpack", back.height, flush=True)
    member = torch.zeros(2 * m, dtype=torch.bool, device="cuda")
    member[bk] = True
    expect = int(member[pk].sum().item())
    a = back.join(build, on="k").height
    b = probe.join(build, on="k").height
    c = D.join(probe, build, on="k", strategy="shuffle").height
    print("expect", expect, "unpacked-join", a, "plain", b, "shuffle", c, flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
