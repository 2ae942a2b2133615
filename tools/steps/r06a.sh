#!/bin/bash
# round 6: partitioned join, first GPU run
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_join_radix.py > $O/r06a_radix.log 2>&1 || exit 1
timeout -k 10 240 python -u tools/bench_legs.py --leg join --steps 5 --warmup 2 > $O/r06a_join.json 2> $O/r06a_join.err || exit 2
PLGPU_JOIN_RADIX=0 timeout -k 10 240 python -u tools/bench_legs.py --leg join --steps 5 --warmup 2 > $O/r06a_join_off.json 2> $O/r06a_join_off.err || exit 3
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_join.py tests/test_gpu_full_size.py -k "join" > $O/r06a_join_tests.log 2>&1 || exit 4
echo ok
