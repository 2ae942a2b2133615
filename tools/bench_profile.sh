#!/bin/bash
# The bench line and the rocprofv3 evidence for it, in ONE lease (run on the
# GPU box via gpurun):
#   bash tools/bench_profile.sh <tag> [bench args...]
# 1. python bench.py <args>                       -> gpurun_out/<tag>/bench.json
# 2. the same command under rocprofv3 --kernel-trace --stats
#                                                 -> gpurun_out/<tag>/trace/
# 3. FETCH_SIZE and WRITE_SIZE passes (one counter group each, kernel trace
#    only: no runtime / sys trace next to counters)
#                                                 -> gpurun_out/<tag>/pmc{1,2}/
# Summarise with tools/bench_evidence.py gpurun_out/<tag>.
set -o pipefail
TAG=${1:-run}; shift
ARGS=${@:---steps 20 --warmup 5}
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 420 python3 -u $R/bench.py $ARGS > $OUT/bench.json 2> $OUT/bench.err || exit 1
# the profiled runs skip the CPU baselines and the host-link plugin leg (no
# GPU kernels of interest, minutes of host work under the tracer)
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 -u $R/bench.py $ARGS --no-cpu --no-plugin > $OUT/trace.json 2> $OUT/trace.err || exit 2
timeout -k 10 420 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc1 -o run -- \
    python3 -u $R/bench.py $ARGS --no-cpu --no-plugin > $OUT/pmc1.json 2> $OUT/pmc1.err || exit 3
timeout -k 10 420 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc2 -o run -- \
    python3 -u $R/bench.py $ARGS --no-cpu --no-plugin > $OUT/pmc2.json 2> $OUT/pmc2.err || exit 4
echo done
