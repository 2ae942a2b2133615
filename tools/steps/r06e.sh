#!/bin/bash
# round 6: radix join (match pass + emit) and nulls on the fused / partitioned paths
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_join_radix.py > $O/r06e_radix.log 2>&1 || exit 1
timeout -k 10 240 python -u tools/bench_legs.py --leg join --steps 5 --warmup 2 > $O/r06e_join.json 2> $O/r06e_join.err || exit 2
PLGPU_JOIN_RADIX_BATCH=4 timeout -k 10 240 python -u tools/bench_legs.py --leg join --steps 5 --warmup 2 > $O/r06e_join_b4.json 2> $O/r06e_join_b4.err || exit 3
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_groupby_sweep.py > $O/r06e_sweep.log 2>&1 || exit 4
timeout -k 10 300 python -u tools/bench_legs.py --leg nulls --steps 5 --warmup 2 > $O/r06e_nulls.json 2> $O/r06e_nulls.err || exit 5
echo ok
