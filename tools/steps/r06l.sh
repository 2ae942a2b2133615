#!/bin/bash
# round 6: compact regions with an overflow table; value nulls as +0.0 in sum-only partition buffers
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_many_groups.py tests/test_gpu_groupby_sweep.py > $O/r06l_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_legs.py --leg many_groups --groups 10000000 --steps 5 --warmup 2 > $O/r06l_mg7.json 2> $O/r06l_mg7.err || exit 2
PLGPU_PART_COMPACT=0 timeout -k 10 300 python -u tools/bench_legs.py --leg many_groups --groups 10000000 --steps 5 --warmup 2 > $O/r06l_mg7_off.json 2> $O/r06l_mg7_off.err || exit 3
timeout -k 10 300 python -u tools/bench_legs.py --leg nulls --steps 5 --warmup 2 > $O/r06l_nulls.json 2> $O/r06l_nulls.err || exit 4
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fused_keys.py -k nonneg > $O/r06l_nonneg.log 2>&1 || exit 5
echo ok
