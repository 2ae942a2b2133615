#!/bin/bash
# round 6: per-workgroup status publication in the slim fused kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python -u tools/bench_legs.py --leg headline --steps 10 --warmup 3 > $O/r06q_head.json 2>&1 || exit 2
timeout -k 10 300 python -u tools/bench_legs.py --leg many_groups --groups 10000000 --steps 3 --warmup 1 > $O/r06q_mg7.json 2>&1 || exit 3
timeout -k 10 300 python -u tools/bench_legs.py --leg many_groups --groups 1000000 --steps 3 --warmup 1 > $O/r06q_mg6.json 2>&1 || exit 4
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_many_groups.py tests/test_gpu_groupby_sweep.py tests/test_gpu_parity.py tests/test_gpu_fused_keys.py > $O/r06q_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/filter_pool_ab.py --states A,C,D1,D3000,D7001,C > $O/r06q_filter_ab.json 2> $O/r06q_filter_ab.err || exit 5
echo ok
