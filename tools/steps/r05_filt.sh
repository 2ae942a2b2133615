set -o pipefail
mkdir -p gpurun_out/filt
timeout -k 10 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "one_pass_lookback" > gpurun_out/filt/t1.log 2>&1 || { tail -30 gpurun_out/filt/t1.log; exit 1; }
tail -1 gpurun_out/filt/t1.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_dtypes.py tests/test_gpu_strings.py tests/test_gpu_groupby_multi.py -k "filter" > gpurun_out/filt/t2.log 2>&1 || { tail -30 gpurun_out/filt/t2.log; exit 1; }
tail -1 gpurun_out/filt/t2.log
for v in 1 0 1 0; do
  PLGPU_FILT_FUSED=$v timeout -k 10 180 python -u tools/bench_legs.py --leg filter --steps 10 --warmup 3 > gpurun_out/filt/f_$v.json 2>&1 || exit 1
  echo "fused=$v $(tail -1 gpurun_out/filt/f_$v.json | cut -c1-400)"
done
