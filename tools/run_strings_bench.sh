set -e
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/bench_strings.py --rows 1e9 > gpurun_out/bench_strings.json 2> gpurun_out/bench_strings.err
export TMPDIR=/tmp
timeout -k 10 250 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_str -o str -- python3 tools/bench_strings.py --rows 1e9 --steps 3 > gpurun_out/prof_str.log 2>&1
