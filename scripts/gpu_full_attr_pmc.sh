# tests, full default bench, PMC passes on attract_rows (t = 1..300)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 900 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS \
  --kernel-include-regex attract_rows -d gpurun_out/apmc1 -o pmc --output-format csv -- \
  python bench.py --steps 300 --warmup 0 --trace 0 --no-cpu-baseline > gpurun_out/apmc1.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum \
  --kernel-include-regex attract_rows -d gpurun_out/apmc2 -o pmc --output-format csv -- \
  python bench.py --steps 300 --warmup 0 --trace 0 --no-cpu-baseline > gpurun_out/apmc2.log 2>&1 || exit $?
