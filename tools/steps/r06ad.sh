#!/bin/bash
# round 6: rolling_std(20) instruction mix (PMC passes, one block set each) and kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06ad
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for kind in std mean; do
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt_$kind -o kt -- python3 tools/bench_rolling.py --kind $kind --steps 3 > $O/kt_$kind.json 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY -d $O/pmc_$kind -o pmc -- python3 tools/bench_rolling.py --kind $kind --steps 1 > $O/pmc_$kind.log 2>&1 || exit 2
done
echo ok
