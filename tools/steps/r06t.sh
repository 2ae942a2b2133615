#!/bin/bash
# round 6: null-key sentinel in sum-only partition buffers; wave_report A/B (now wired)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_many_groups.py tests/test_gpu_groupby_sweep.py > $O/r06t_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_legs.py --leg nulls --steps 5 --warmup 2 > $O/r06t_nulls.json 2> $O/r06t_nulls.err || exit 2
for w in 0 1; do
PLGPU_WAVE_REPORT=$w timeout -k 10 300 python -u tools/bench_legs.py --leg many_groups --groups 10000000 --steps 3 --warmup 1 > $O/r06t_mg7_w$w.json 2>&1 || exit 3
PLGPU_WAVE_REPORT=$w timeout -k 10 200 python -u tools/bench_legs.py --leg headline --steps 10 --warmup 3 > $O/r06t_head_w$w.json 2>&1 || exit 4
done
echo ok
