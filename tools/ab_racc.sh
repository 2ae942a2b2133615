#!/bin/bash
# A/B of the PART kernel's per-lane register accumulators (PLGPU_PART_RACC)
# on the time-ordered (symbol, day) query and the random many-groups ones.
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in 1 0; do
  echo "== PLGPU_PART_RACC=$v"
  PLGPU_PART_RACC=$v timeout -k 10 120 python tools/diag_two_keys.py || exit 1
done
timeout -k 10 400 python tools/ab_many_groups.py 1e9 base "PART_RACC=0" || exit 2
