set -o pipefail
mkdir -p gpurun_out/varpos
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_var_std.py tests/test_gpu_groupby_sweep.py > gpurun_out/varpos/tests.log 2>&1 || { tail -30 gpurun_out/varpos/tests.log; exit 1; }
tail -1 gpurun_out/varpos/tests.log
for rep in 1 2 3; do
for v in 1 0; do
  PLGPU_VAR_POS=$v timeout -k 10 180 python -u tools/bench_legs.py --leg std --steps 20 --warmup 3 > gpurun_out/varpos/std_${v}_$rep.json 2>&1 || exit 1
  echo "var_pos=$v $(tail -1 gpurun_out/varpos/std_${v}_$rep.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms"], d["frac"])')"
done
done
