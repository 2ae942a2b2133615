#!/bin/bash
# round 6: filter placement -- physically contiguous large blocks A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
for k in 1 0; do
PLGPU_ALLOC_CONTIG=$k timeout -k 10 500 python -u tools/filter_pool_ab.py --states A,B,D3000,C > $O/r06w_filter_c$k.json 2> $O/r06w_filter_c$k.err || exit 4
done
echo ok
