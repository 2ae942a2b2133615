set -o pipefail
mkdir -p gpurun_out/wpe
for rep in 1 2; do
for lib in libpolaroid_gpu_ab1.so libpolaroid_gpu.so; do
  PLGPU_LIB=$PWD/polaroid_amd/$lib timeout -k 10 180 python -u tools/bench_legs.py --leg headline --steps 20 --warmup 3 > gpurun_out/wpe/headline_${lib}_$rep.json 2>&1 || exit 1
  echo "$lib headline $(tail -1 gpurun_out/wpe/headline_${lib}_$rep.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms"])')"
  PLGPU_LIB=$PWD/polaroid_amd/$lib timeout -k 10 400 python -u tools/bench_keys.py --only categorical,string,sym_day --steps 10 --warmup 3 > gpurun_out/wpe/keys_${lib}_$rep.json 2>&1 || exit 1
  grep '"case"' gpurun_out/wpe/keys_${lib}_$rep.json | python -c 'import json,sys
for l in sys.stdin:
    d=json.loads(l); print("  ", d["case"], d["ms_per_step"], d.get("fused_kernel_ms"))'
done
done
