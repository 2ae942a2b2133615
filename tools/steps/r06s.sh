#!/bin/bash
# round 6: host-side cost of the single-key and (symbol, day) queries
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 200 python -u tools/host_overhead.py --keys symbol --calls 300 > $O/r06s_host_sym.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/host_overhead.py --keys sym_day --calls 300 > $O/r06s_host_symday.txt 2>&1 || exit 2
timeout -k 10 200 python -u tools/host_overhead.py --keys sym_day --rows 1e8 --calls 30 > $O/r06s_host_symday_1e8.txt 2>&1 || exit 3
echo ok
