# Profiles of the bench's timed window (t = 1..20, no warmup, no rest): kernel
# trace + stats, and PMC passes for attract_rows (HBM / L2 traffic and request
# counters, one block group per pass as MI355X_MICROARCH.md prescribes).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python bench.py --steps 20 --warmup 0 --no-rest --no-cpu-baseline --trace 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profw -o prof --output-format csv -- $B \
  > gpurun_out/profw.json 2> gpurun_out/profw.err || exit $?
for pass in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" \
            "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU"; do
  tag=$(echo $pass | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $pass --kernel-include-regex "attract_rows|bh_traverse|tile_apply|combine_update" \
    -d gpurun_out/pmcw_$tag -o pmc --output-format csv -- $B > gpurun_out/pmcw_$tag.log 2>&1 || exit $?
done
echo done > gpurun_out/prof_done.txt
