#!/bin/bash
# A/B of the plan-selected register-accumulator variant of the fused kernel
# (PLGPU_RUNS) on random and symbol-sorted headline data.
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in auto 0; do
  echo "== PLGPU_RUNS=$v"
  if [ $v = auto ]; then timeout -k 10 200 python tools/diag_sorted_symbol.py || exit 1
  else PLGPU_RUNS=$v timeout -k 10 200 python tools/diag_sorted_symbol.py || exit 1; fi
done
