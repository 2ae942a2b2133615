#!/bin/bash
# round 6: filter vs pool state; PMC of the many-groups aggregation at 1e7 groups
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 400 python -u tools/filter_pool_ab.py > $O/r06o_filter_ab.json 2> $O/r06o_filter_ab.err || exit 1
cd /tmp && export TMPDIR=/tmp
P=$GRAFT_REPO_ROOT/$O/prof_r06o
mkdir -p $P
L="python3 $GRAFT_REPO_ROOT/tools/bench_legs.py --leg many_groups --groups 10000000 --steps 2 --warmup 1"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- $L > $P/trace.log 2>&1 || exit 3
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $P/pmc1 -o run -- $L > $P/pmc1.log 2>&1 || exit 4
timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $P/pmc2 -o run -- $L > $P/pmc2.log 2>&1 || exit 5
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $P/pmc3 -o run -- $L > $P/pmc3.log 2>&1 || exit 6
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $P/pmc4 -o run -- $L > $P/pmc4.log 2>&1 || exit 7
echo ok
