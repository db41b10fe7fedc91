# PMC passes on bh_traverse + tile_apply over t = 1..300 at 1M
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
  --kernel-include-regex "bh_traverse|tile_apply" -d gpurun_out/pmc3 -o pmc --output-format csv -- \
  python bench.py --steps 300 --warmup 0 --trace 0 --no-cpu-baseline > gpurun_out/pmc3.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH TCC_HIT_sum TCC_MISS_sum \
  --kernel-include-regex "bh_traverse|tile_apply" -d gpurun_out/pmc4 -o pmc --output-format csv -- \
  python bench.py --steps 300 --warmup 0 --trace 0 --no-cpu-baseline > gpurun_out/pmc4.log 2>&1 || exit $?
