#!/bin/bash
# round 6: many-groups LDS-miss rows; filter placement probe
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python -u tools/bench_legs.py --leg many_groups --groups 10000000 --steps 3 --warmup 1 > $O/r06p_mg7.json 2>&1 || exit 2
PLGPU_PART_LDS_KB=80 timeout -k 10 300 python -u tools/bench_legs.py --leg many_groups --groups 10000000 --steps 3 --warmup 1 > $O/r06p_mg7_80.json 2>&1 || exit 3
timeout -k 10 400 python -u tools/filter_pool_ab.py --states A,C,D1,D3000,D7001,C > $O/r06p_filter_ab.json 2> $O/r06p_filter_ab.err || exit 1
echo ok
