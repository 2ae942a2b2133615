#!/bin/bash
# round 6: many-groups A/B -- partition LDS budget and workgroup size at 1e7 / 1e6 groups
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
for cfg in "X=0" "PLGPU_PART_LDS_KB=80" "PLGPU_PART_THREADS=1024" "PLGPU_PART_LDS_KB=80 PLGPU_PART_THREADS=1024"; do
  tag=$(echo $cfg | tr ' =' '__')
  env $cfg timeout -k 10 300 python -u tools/bench_legs.py --leg many_groups --groups 10000000 --steps 5 --warmup 2 > $O/r06n_mg7_$tag.json 2>&1 || exit 2
done
for cfg in "X=0" "PLGPU_PART_LDS_KB=80"; do
  tag=$(echo $cfg | tr ' =' '__')
  env $cfg timeout -k 10 300 python -u tools/bench_legs.py --leg many_groups --groups 1000000 --steps 5 --warmup 2 > $O/r06n_mg6_$tag.json 2>&1 || exit 3
done
echo ok
