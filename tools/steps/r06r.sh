#!/bin/bash
# round 6: same-box A/B -- per-workgroup vs per-wave status atomics; pool offset skew for the filter
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
for rep in 1 2; do
for w in 0 1; do
PLGPU_WAVE_REPORT=$w timeout -k 10 200 python -u tools/bench_legs.py --leg headline --steps 10 --warmup 3 > $O/r06r_head_w${w}_$rep.json 2>&1 || exit 2
done
done
for w in 0 1; do
PLGPU_WAVE_REPORT=$w timeout -k 10 300 python -u tools/bench_legs.py --leg many_groups --groups 10000000 --steps 3 --warmup 1 > $O/r06r_mg7_w$w.json 2>&1 || exit 3
done
for k in 0 1; do
PLGPU_ALLOC_SKEW=$k timeout -k 10 400 python -u tools/filter_pool_ab.py --states A,C,D1,D3000,D7001 > $O/r06r_filter_k$k.json 2> $O/r06r_filter_k$k.err || exit 4
done
echo ok
