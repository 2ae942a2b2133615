#!/bin/bash
# A/B of the partitioned group-by's LDS budget and workgroups per CU on the
# (symbol, day) query at 1e9 rows (tools/diag_two_keys.py, single GPU).
set -o pipefail
cd $GRAFT_REPO_ROOT
for cfg in "80 2" "40 2" "80 8" "40 8" "160 4"; do
  set -- $cfg
  echo "== PLGPU_PART_LDS_KB=$1 PLGPU_PART_WGS_PER_CU=$2"
  PLGPU_PART_LDS_KB=$1 PLGPU_PART_WGS_PER_CU=$2 timeout -k 10 120 python tools/diag_two_keys.py || exit 1
done
