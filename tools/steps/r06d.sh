#!/bin/bash
# round 6: partitioned join as match pass + row-format emit; A/B + PMC
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_join_radix.py > $O/r06d_radix.log 2>&1 || exit 1
for cfg in "8 0" "4 0" "8 50" "8 25"; do
set -- $cfg
PLGPU_JOIN_RADIX_BATCH=$1 PLGPU_JOIN_RADIX_LOAD=$2 timeout -k 10 240 python -u tools/bench_legs.py --leg join --steps 5 --warmup 2 > $O/r06d_join_b$1_l$2.json 2> $O/r06d_join_b$1_l$2.err || exit 2
done
cd /tmp && export TMPDIR=/tmp
P=$GRAFT_REPO_ROOT/$O/prof_r06d
mkdir -p $P
L="python3 $GRAFT_REPO_ROOT/tools/bench_legs.py --leg join --steps 1 --warmup 1"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- $L > $P/trace.log 2>&1 || exit 3
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $P/pmc1 -o run -- $L > $P/pmc1.log 2>&1 || exit 4
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $P/pmc2 -o run -- $L > $P/pmc2.log 2>&1 || exit 5
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $P/pmc3 -o run -- $L > $P/pmc3.log 2>&1 || exit 6
timeout -k 10 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $P/pmc4 -o run -- $L > $P/pmc4.log 2>&1 || exit 7
echo ok
