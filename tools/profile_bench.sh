#!/bin/bash
# rocprofv3 passes over the headline bench (run on the GPU box via gpurun).
#   bash tools/profile_bench.sh <tag> [bench args...]
# Writes gpurun_out/prof_<tag>/{trace,pmc*}; summarise with tools/pmc_summary.py.
set -o pipefail
TAG=${1:-run}; shift
ARGS=${@:---rows 1e9 --steps 5 --warmup 1 --no-cpu}
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py $ARGS > $OUT/trace.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc1 -o run -- python3 $R/bench.py $ARGS > $OUT/pmc1.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc2 -o run -- python3 $R/bench.py $ARGS > $OUT/pmc2.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VMEM --kernel-trace --output-format csv -d $OUT/pmc3 -o run -- python3 $R/bench.py $ARGS > $OUT/pmc3.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS_ATOMIC SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/pmc4 -o run -- python3 $R/bench.py $ARGS > $OUT/pmc4.log 2>&1 || exit 5
echo done
