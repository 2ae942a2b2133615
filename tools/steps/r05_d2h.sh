set -o pipefail
mkdir -p gpurun_out/d2h
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_var_std.py tests/test_gpu_plan_cache.py tests/test_gpu_fused_keys.py > gpurun_out/d2h/tests.log 2>&1 || { tail -30 gpurun_out/d2h/tests.log; exit 1; }
tail -1 gpurun_out/d2h/tests.log
for rep in 1 2; do
for lib in libpolaroid_gpu.so libpolaroid_gpu_ab1.so; do
  for leg in headline std; do
    PLGPU_LIB=$PWD/polaroid_amd/$lib timeout -k 10 180 python -u tools/bench_legs.py --leg $leg --steps 20 --warmup 3 > gpurun_out/d2h/${leg}_${lib}_$rep.json 2>&1 || exit 1
    echo "$lib $leg $(tail -1 gpurun_out/d2h/${leg}_${lib}_$rep.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms"])')"
  done
  PLGPU_LIB=$PWD/polaroid_amd/$lib timeout -k 10 300 python -u tools/bench_keys.py --only sym_day --steps 20 --warmup 3 > gpurun_out/d2h/symday_${lib}_$rep.json 2>&1 || exit 1
  echo "$lib symday $(tail -1 gpurun_out/d2h/symday_${lib}_$rep.json | cut -c1-200)"
done
done
