#!/bin/bash
# round 6: partition scatter in 40.5 KiB of LDS, 4 waves per SIMD at level 2 / both -- parity, then A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06ah
mkdir -p $O
PLGPU_PART_SCATTER_WPE=2 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_many_groups.py tests/test_gpu_groupby_sweep.py tests/test_gpu_join_radix.py > $O/tests_wpe2.log 2>&1 || exit 1
for G in 10000000 1000000; do
for r in 0 1 2 0 1 2; do
  PLGPU_PART_SCATTER_WPE=$r timeout -k 10 300 python -u tools/bench_legs.py --leg many_groups --groups $G --steps 3 --warmup 1 >> $O/mg_${G}_w$r.json 2>&1 || exit 2
done
done
echo ok
