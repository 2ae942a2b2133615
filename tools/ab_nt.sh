# A/B of non-temporal loads / stores in the rolling wave kernel and the
# filter scatter (env switches), interleaved, one JSON line per run.
set -o pipefail
for rep in 1 2; do
  for nt in 0 1 2 3; do
    echo "rolling PLGPU_RL_NT=$nt"
    PLGPU_RL_NT=$nt timeout -k 10 120 python tools/bench_rolling.py --steps 10 || exit 1
  done
  for nt in 0 1; do
    echo "filter PLGPU_FILTER_NT=$nt"
    PLGPU_FILTER_NT=$nt timeout -k 10 120 python tools/bench_filter.py --steps 10 || exit 2
  done
done
