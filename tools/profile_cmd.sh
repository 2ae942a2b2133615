#!/bin/bash
# rocprofv3 passes (trace + separate PMC passes) over any python command.
#   bash tools/profile_cmd.sh <tag> <script.py> [args...]
# Writes gpurun_out/prof_<tag>/{trace,pmc1..pmc4}; summarise with
# tools/pmc_summary.py gpurun_out/prof_<tag> <kernel-substring>.
set -o pipefail
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
SCRIPT=$R/$1; shift
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $SCRIPT "$@" > $OUT/trace.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc1 -o run -- python3 $SCRIPT "$@" > $OUT/pmc1.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc2 -o run -- python3 $SCRIPT "$@" > $OUT/pmc2.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace --output-format csv -d $OUT/pmc3 -o run -- python3 $SCRIPT "$@" > $OUT/pmc3.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $OUT/pmc4 -o run -- python3 $SCRIPT "$@" > $OUT/pmc4.log 2>&1 || exit 5
echo done
