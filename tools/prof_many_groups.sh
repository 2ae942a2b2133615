# Kernel trace of the two many-groups group-by workloads of
# tools/bench_multikey.py (1e9 rows): (sym, day) = 25,000 groups and
# id = 100,000 groups.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for w in groupby groupby_hc; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_mg_$w -o run -- python3 $R/tools/bench_multikey.py --only $w --steps 2 > $R/gpurun_out/prof_mg_$w.log 2>&1 || exit 1
done
