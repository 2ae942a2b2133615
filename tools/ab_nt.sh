# A/B of non-temporal loads / stores in the rolling wave kernel and the
# filter scatter.  PLGPU_RL_NT / PLGPU_FILTER_NT were temporary switches of
# the build measured in profiles/r02_nt_ab_rolling_filter.log (no gain, so
# they were removed again); kept as the record of that run.
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
