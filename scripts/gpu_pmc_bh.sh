# tests, rcp probe, timeline, and PMC passes on bh_traverse over t = 1..260 at 1M
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 60 ./scripts/rcp_accuracy > gpurun_out/rcp.log 2>&1 || exit $?
STEPS=300 bash scripts/gpu_timeline.sh || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
  --kernel-include-regex bh_traverse -d gpurun_out/pmc1 -o pmc --output-format csv -- \
  python bench.py --steps 260 --warmup 0 --trace 0 --no-cpu-baseline > gpurun_out/pmc1.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH TCC_HIT_sum TCC_MISS_sum \
  --kernel-include-regex bh_traverse -d gpurun_out/pmc2 -o pmc --output-format csv -- \
  python bench.py --steps 260 --warmup 0 --trace 0 --no-cpu-baseline > gpurun_out/pmc2.log 2>&1 || exit $?
