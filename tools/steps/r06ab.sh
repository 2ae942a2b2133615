#!/bin/bash
# round 6: partition table budget A/B again, now with one status atomic per workgroup
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
for G in 10000000 1000000; do
for cfg in "X=0" "PLGPU_PART_LDS_KB=80" "X=0" "PLGPU_PART_LDS_KB=80"; do
  tag=$(echo $cfg | tr ' =' '__')
  env $cfg timeout -k 10 300 python -u tools/bench_legs.py --leg many_groups --groups $G --steps 3 --warmup 1 >> $O/r06ab_mg_${G}_$tag.json 2>&1 || exit 2
done
done
echo ok
