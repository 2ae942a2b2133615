# Many-groups group-by (tools/bench_multikey.py groupby / groupby_hc, 1e9
# rows): step time against the partition pass's workgroup count
# (PLGPU_PART_G; default 8 per CU).
set -o pipefail
for g in 2048 1024 512 256; do
  for w in groupby groupby_hc; do
    echo "G=$g $w"
    PLGPU_PART_G=$g timeout -k 10 120 python tools/bench_multikey.py --only $w --steps 3 || exit 1
  done
done
