set -o pipefail
mkdir -p gpurun_out/sumpos
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fused_keys.py tests/test_gpu_full_size_groupby.py tests/test_gpu_groupby_sweep.py > gpurun_out/sumpos/tests.log 2>&1 || { tail -30 gpurun_out/sumpos/tests.log; exit 1; }
tail -1 gpurun_out/sumpos/tests.log
for rep in 1 2; do
for v in 1 0; do
  PLGPU_SUM_POS=$v timeout -k 10 180 python -u tools/bench_legs.py --leg headline --steps 20 --warmup 3 > gpurun_out/sumpos/h_${v}_$rep.json 2>&1 || exit 1
  echo "sum_pos=$v headline $(tail -1 gpurun_out/sumpos/h_${v}_$rep.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms"], d["frac"])')"
  PLGPU_SUM_POS=$v timeout -k 10 400 python -u tools/bench_keys.py --only categorical,string,sym_day --steps 10 --warmup 3 > gpurun_out/sumpos/k_${v}_$rep.json 2>&1 || exit 1
  grep '"case"' gpurun_out/sumpos/k_${v}_$rep.json | python -c 'import json,sys
for l in sys.stdin:
    d=json.loads(l); print("  ", d["case"], d["ms_per_step"], d.get("fused_kernel_ms"))'
done
done
