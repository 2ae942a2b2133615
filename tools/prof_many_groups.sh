# Kernel trace of the two many-groups group-by workloads of
# tools/bench_multikey.py (1e9 rows): (sym, day) = 25,000 groups and
# id = 100,000 groups; VALUES=prices|unit (default unit).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
V=${VALUES:-unit}
for w in groupby groupby_hc; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_mg_${w}_$V -o run -- python3 $R/tools/bench_multikey.py --only $w --steps 2 --values $V > $R/gpurun_out/prof_mg_${w}_$V.log 2>&1 || exit 1
done
