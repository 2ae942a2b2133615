#!/bin/bash
# round 6: nulls word loads; join match-pass PMC
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_groupby_sweep.py > $O/r06f_sweep.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_legs.py --leg nulls --steps 5 --warmup 2 > $O/r06f_nulls.json 2> $O/r06f_nulls.err || exit 2
cd /tmp && export TMPDIR=/tmp
P=$GRAFT_REPO_ROOT/$O/prof_r06f
mkdir -p $P
L="python3 $GRAFT_REPO_ROOT/tools/bench_legs.py --leg join --steps 1 --warmup 1"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- $L > $P/trace.log 2>&1 || exit 3
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $P/pmc1 -o run -- $L > $P/pmc1.log 2>&1 || exit 4
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $P/pmc2 -o run -- $L > $P/pmc2.log 2>&1 || exit 5
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $P/pmc3 -o run -- $L > $P/pmc3.log 2>&1 || exit 6
timeout -k 10 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum --kernel-trace --output-format csv -d $P/pmc4 -o run -- $L > $P/pmc4.log 2>&1 || exit 7
echo ok
