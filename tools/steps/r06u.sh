#!/bin/bash
# round 6: null-key sentinel, spread at level 2, slotted key-range atomics
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python -u tools/bench_legs.py --leg nulls --steps 5 --warmup 2 > $O/r06u_nulls.json 2> $O/r06u_nulls.err || exit 2
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_many_groups.py tests/test_gpu_groupby_sweep.py > $O/r06u_tests.log 2>&1 || exit 1
echo ok
