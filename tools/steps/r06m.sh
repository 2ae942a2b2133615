#!/bin/bash
# round 6: rolling var/std numerators mod 2^128; hoisted validity words in the partition passes
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sort_rolling.py -k "var or std" > $O/r06m_var.log 2>&1 || exit 1
for v in 1 0; do
PLGPU_RL_VAR128=$v timeout -k 10 200 python -u tools/bench_rolling.py --kind std --steps 10 > $O/r06m_std_$v.json 2>&1 || exit 2
done
timeout -k 10 300 python -u tools/bench_legs.py --leg nulls --steps 5 --warmup 2 > $O/r06m_nulls.json 2> $O/r06m_nulls.err || exit 3
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_many_groups.py tests/test_gpu_groupby_sweep.py > $O/r06m_tests.log 2>&1 || exit 4
echo ok
