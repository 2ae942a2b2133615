#!/bin/bash
# round 6: filter placement -- contiguous blocks A/B, alternating order
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
i=0
for k in 0 1 0 1; do
i=$((i+1))
PLGPU_ALLOC_CONTIG=$k timeout -k 10 400 python -u tools/filter_pool_ab.py --states A,C > $O/r06x_filter_${i}_c$k.json 2> $O/r06x_filter_${i}_c$k.err || exit 4
done
echo ok
