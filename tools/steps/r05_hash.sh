set -o pipefail
mkdir -p gpurun_out/hash
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_groupby_sweep.py tests/test_gpu_parity.py tests/test_gpu_many_groups.py tests/test_gpu_plan_cache.py tests/test_gpu_fused_keys.py tests/test_gpu_reduce.py tests/test_gpu_var_std.py > gpurun_out/hash/tests.log 2>&1 || { tail -30 gpurun_out/hash/tests.log; exit 1; }
tail -2 gpurun_out/hash/tests.log
for leg in headline vwap std; do
  timeout -k 10 180 python -u tools/bench_legs.py --leg $leg --steps 10 --warmup 3 > gpurun_out/hash/$leg.json 2>&1 || exit 1
  tail -1 gpurun_out/hash/$leg.json
done
timeout -k 10 300 python -u tools/bench_legs.py --leg many_groups --groups 1000000 --steps 5 --warmup 2 > gpurun_out/hash/mg.json 2>&1 || exit 1
tail -1 gpurun_out/hash/mg.json
