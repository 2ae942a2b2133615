set -o pipefail
mkdir -p gpurun_out/pload
for rep in 1 2; do
for ld in 50 70 80; do
  for g in 10000000 1000000; do
    PLGPU_PART_LOAD=$ld timeout -k 10 300 python -u tools/bench_legs.py --leg many_groups --groups $g --steps 5 --warmup 2 > gpurun_out/pload/mg_${g}_${ld}_$rep.json 2>&1 || exit 1
    echo "load=$ld G=$g $(tail -1 gpurun_out/pload/mg_${g}_${ld}_$rep.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); v=d[str(d["groups"])]; print(v["ms_per_step"], v["partition_bits"], v["scatter_passes"], v["scatter"]["kernel_ms"], v["aggregate"]["kernel_ms"])')"
  done
done
done
