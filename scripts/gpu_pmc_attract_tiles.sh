# PMC passes (SQ instruction mix / waits, LDS conflicts, L2) over the timed
# window's attraction launches: bench.py --steps 20 --warmup 5 (whole schedule), attract_tiles.
# Env: PMC_ARGS (extra bench arguments, e.g. --option attract_cfg=3).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
k=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS TCC_HIT_sum TCC_MISS_sum"; do
  k=$((k+1))
  timeout -s KILL 240 rocprofv3 --pmc $ctrs --kernel-include-regex 'attract_(rows|tiles)' \
    -d gpurun_out/pmc_at$k -o pmc --output-format csv -- \
    python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-cli-e2e --trace 0 ${PMC_ARGS:-} > gpurun_out/pmc_at$k.log 2>&1 || exit $?
done
