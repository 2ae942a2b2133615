set -o pipefail
mkdir -p gpurun_out/rlfull
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sort_rolling.py tests/test_gpu_full_size.py > gpurun_out/rlfull/tests.log 2>&1 || { tail -30 gpurun_out/rlfull/tests.log; exit 1; }
tail -2 gpurun_out/rlfull/tests.log
for v in 1 0 1 0; do
  for k in mean std; do
    PLGPU_RL_FULL=$v timeout -k 10 120 python -u tools/bench_rolling.py --kind $k --steps 10 > gpurun_out/rlfull/${k}_$v.json 2>&1 || exit 1
    echo "full=$v $(tail -1 gpurun_out/rlfull/${k}_$v.json)"
  done
done
