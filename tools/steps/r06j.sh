#!/bin/bash
# round 6: NULLS fused kernel with validity words shifted at consume time; oracle-checked sum_pos / var_pos
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python -u tools/bench_legs.py --leg nulls --steps 5 --warmup 2 > $O/r06j_nulls.json 2> $O/r06j_nulls.err || exit 2
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_groupby_sweep.py tests/test_gpu_fused_keys.py tests/test_gpu_var_std.py tests/test_gpu_sort_rolling.py -k "null or nonneg or ddof or sweep" > $O/r06j_tests.log 2>&1 || exit 1
echo ok
