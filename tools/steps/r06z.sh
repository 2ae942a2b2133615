#!/bin/bash
# round 6: full GPU suite on the product library, then the checked build over the group-by sweep and many groups
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r06z_gpu_all.log 2>&1 || exit 1
PLGPU_LIB=$GRAFT_REPO_ROOT/polaroid_amd/libpolaroid_gpu_checked.so timeout -k 10 150 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_many_groups.py -k "compact or sentinel" > $O/r06z_checked.log 2>&1 || exit 2
echo ok
