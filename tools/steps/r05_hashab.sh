set -o pipefail
mkdir -p gpurun_out/hashab
for rep in 1 2; do
for lib in libpolaroid_gpu.so libpolaroid_gpu_ab1.so libpolaroid_gpu_ab2.so; do
  for leg in std headline vwap; do
    PLGPU_LIB=$PWD/polaroid_amd/$lib timeout -k 10 180 python -u tools/bench_legs.py --leg $leg --steps 10 --warmup 3 > gpurun_out/hashab/${leg}_${lib}_$rep.json 2>&1 || exit 1
    echo "$lib $leg $(tail -1 gpurun_out/hashab/${leg}_${lib}_$rep.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms"])')"
  done
done
done
