#!/bin/bash
# round 6: half-tile match pass (hash once, bucket staged), batch A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_join_radix.py > $O/r06i_radix.log 2>&1 || exit 1
for b in 8 4; do
PLGPU_JOIN_RADIX_BATCH=$b timeout -k 10 240 python -u tools/bench_legs.py --leg join --steps 5 --warmup 2 > $O/r06i_join_b$b.json 2> $O/r06i_join_b$b.err || exit 2
done
echo ok
