set -e
mkdir -p gpurun_out
for how in inner left semi anti full; do
  timeout -k 10 150 python -u tools/bench_join.py --how $how --steps 5 --warmup 1 >> gpurun_out/bench_join_types.jsonl
done
timeout -k 10 150 python -u tools/bench_join.py --how left --order right --steps 3 --warmup 1 >> gpurun_out/bench_join_types.jsonl
timeout -k 10 150 python -u tools/bench_join.py --how full --order left_right --steps 3 --warmup 1 >> gpurun_out/bench_join_types.jsonl
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_jt -o jt -- python3 tools/bench_join.py --how left --steps 3 --warmup 1 > gpurun_out/prof_jt.log 2>&1
