# tests; rcp accuracy; PMC on bh_traverse (200k, 30 it); 200k + 1M full benches
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 60 ./scripts/rcp_accuracy > gpurun_out/rcp.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY \
  --kernel-include-regex bh_traverse -d gpurun_out/pmc2 -o pmc --output-format csv -- \
  python bench.py --n 200000 --steps 30 --warmup 0 --trace 0 --no-cpu-baseline > gpurun_out/pmc2.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --n 200000 --no-cpu-baseline > gpurun_out/bench_200k.log 2>&1 || exit $?
timeout -k 10 900 python bench.py > gpurun_out/bench_1m.log 2>&1 || exit $?
