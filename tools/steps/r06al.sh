#!/bin/bash
# round 6, final tree: full GPU suite, smoke, the default bench line, checked build over the group-by sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06al
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_all.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 2
PLGPU_LIB=$GRAFT_REPO_ROOT/polaroid_amd/libpolaroid_gpu_checked.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_many_groups.py tests/test_gpu_sort_rolling.py -k "compact or sentinel or rolling_var" > $O/checked.log 2>&1 || exit 3
echo ok
