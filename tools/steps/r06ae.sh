#!/bin/bash
# round 6: rolling var / std common-block kernel -- parity, A/B, instruction mix
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06ae
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sort_rolling.py -k "rolling" > $O/tests.log 2>&1 || exit 1
for cfg in "PLGPU_RL_VAR_HOT=1" "PLGPU_RL_VAR_HOT=0" "PLGPU_RL_VAR_HOT=1 PLGPU_RL_STREAM=1" "PLGPU_RL_VAR_HOT=1" "PLGPU_RL_VAR_HOT=0"; do
  env $cfg timeout -k 10 120 python -u tools/bench_rolling.py --kind std --steps 5 >> $O/ab_std.jsonl 2>&1 || exit 2
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt_std -o kt -- python3 tools/bench_rolling.py --kind std --steps 3 > $O/kt_std.json 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY -d $O/pmc_std -o pmc -- python3 tools/bench_rolling.py --kind std --steps 1 > $O/pmc_std.log 2>&1 || exit 4
echo ok
