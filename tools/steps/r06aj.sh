#!/bin/bash
# round 6: rolling sum / mean common-block kernel -- parity, A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06aj
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sort_rolling.py -k "rolling" > $O/tests.log 2>&1 || exit 1
for cfg in "PLGPU_RL_MEAN_HOT=1" "PLGPU_RL_MEAN_HOT=0" "PLGPU_RL_MEAN_HOT=1" "PLGPU_RL_MEAN_HOT=0"; do
  env $cfg timeout -k 10 120 python -u tools/bench_rolling.py --kind mean --steps 5 >> $O/ab_mean.jsonl 2>&1 || exit 2
  env $cfg timeout -k 10 120 python -u tools/bench_rolling.py --kind sum --steps 5 >> $O/ab_sum.jsonl 2>&1 || exit 3
done
echo ok
