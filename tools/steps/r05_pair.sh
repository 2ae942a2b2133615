set -o pipefail
mkdir -p gpurun_out/pair
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_reduce.py tests/test_gpu_var_std.py tests/test_gpu_groupby_sweep.py -k "derived or var or vwap or std" > gpurun_out/pair/tests.log 2>&1 &&
for v in 1 0 1 0; do PLGPU_GB_PAIR=$v timeout -k 10 180 python -u tools/bench_legs.py --leg vwap --steps 10 --warmup 3 > gpurun_out/pair/vwap_$v.json 2>&1 && cat gpurun_out/pair/vwap_$v.json | tail -1 || exit 1; done
