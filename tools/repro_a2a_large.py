"""Standalone check of torch.distributed.all_to_all_single (RCCL) on large
messages -- no polaroid code involved:

    python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 \
        tools/repro_a2a_large.py 1 2 3 4 6

For each size (GiB) an int64 tensor of arange values is exchanged (world 1:
RCCL's self send/recv path) and the output is compared with the input on
the device; prints one line per size with the first mismatching element."""
import sys

import torch
import torch.distributed as dist


def main():
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    for gib in [float(a) for a in sys.argv[1:]] or [1, 2, 4]:
        n = int(gib * (1 << 30)) // 8
        x = torch.arange(n, device="cuda", dtype=torch.int64)
        y = torch.full_like(x, -1)
        dist.all_to_all_single(y, x)
        torch.cuda.synchronize()
        bad = torch.nonzero(y != x)
        first = int(bad[0].item()) if bad.numel() else -1
        print(f"{gib:g} GiB ({n} int64): {'OK' if first < 0 else 'MISMATCH'}"
              + ("" if first < 0 else f" first bad element {first} (byte {first * 8}), {bad.numel()} bad"),
              flush=True)
        del x, y, bad
        torch.cuda.empty_cache()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
