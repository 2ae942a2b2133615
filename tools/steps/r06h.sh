#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 120 python -u tools/dbg_radix.py > $O/r06h_dbg.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_join_radix.py > $O/r06h_radix.log 2>&1
for b in 4 8; do
PLGPU_JOIN_RADIX_BATCH=$b timeout -k 10 240 python -u tools/bench_legs.py --leg join --steps 5 --warmup 2 > $O/r06h_join_b$b.json 2> $O/r06h_join_b$b.err || exit 2
done
echo ok
