# PMC passes (L2 hit / miss, FETCH_SIZE, SQ) over tools/bench_join.py with the
# opt-in XCD-partitioned join probe.
set -o pipefail
export PLGPU_XP=1  # the opt-in XCD-partitioned probe
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_xp
mkdir -p $OUT
timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $OUT/p1 -o run -- python3 $R/tools/bench_join.py --steps 1 --warmup 0 > $OUT/p1.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/p2 -o run -- python3 $R/tools/bench_join.py --steps 1 --warmup 0 > $OUT/p2.log 2>&1 || exit 2
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU --kernel-trace --output-format csv -d $OUT/p3 -o run -- python3 $R/tools/bench_join.py --steps 1 --warmup 0 > $OUT/p3.log 2>&1 || exit 3
echo done
