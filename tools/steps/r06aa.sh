#!/bin/bash
# round 6: sort A/B -- downsweep occupancy target, upsweep tiles per workgroup; parity first
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
PLGPU_SRT_W4=1 PLGPU_SRT_UP_TILES=4 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sort_rolling.py tests/test_gpu_sort_multi.py -k "sort" > $O/r06aa_sort_tests.log 2>&1 || exit 1
for cfg in "PLGPU_SRT_W4=0 PLGPU_SRT_UP_TILES=1" "PLGPU_SRT_W4=1 PLGPU_SRT_UP_TILES=1" "PLGPU_SRT_W4=0 PLGPU_SRT_UP_TILES=4" "PLGPU_SRT_W4=1 PLGPU_SRT_UP_TILES=4" "PLGPU_SRT_W4=0 PLGPU_SRT_UP_TILES=1"; do
  tag=$(echo $cfg | tr ' =' '__')
  env $cfg timeout -k 10 300 python -u tools/bench_legs.py --leg sort --steps 3 --warmup 1 > $O/r06aa_$tag.json 2>&1 || exit 2
done
echo ok
