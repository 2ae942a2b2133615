#!/bin/bash
# round 6: input placement probe (separate column blocks vs staggered starts), three processes
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
for i in 1 2 3; do
timeout -k 10 400 python -u tools/stagger_probe.py > $O/r06y_stagger_$i.json 2> $O/r06y_stagger_$i.err || exit 4
done
echo ok
