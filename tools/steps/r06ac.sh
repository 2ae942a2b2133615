#!/bin/bash
# round 6: partitioned aggregation with 4 rows per thread -- parity, then A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
PLGPU_PART_ROWS4=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_many_groups.py tests/test_gpu_groupby_sweep.py > $O/r06ac_tests.log 2>&1 || exit 1
for G in 10000000 1000000; do
for r in 0 1 0 1; do
  PLGPU_PART_ROWS4=$r timeout -k 10 300 python -u tools/bench_legs.py --leg many_groups --groups $G --steps 3 --warmup 1 >> $O/r06ac_mg_${G}_r$r.json 2>&1 || exit 2
done
done
echo ok
