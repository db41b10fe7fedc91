# GPU check of HEAD: parity tests, rocprofv3 kernel stats on a short 1M bench, full default bench
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o prof --output-format csv -- \
  python bench.py --steps 20 --warmup 2 --trace 0 --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1 || exit $?
timeout -k 10 900 python bench.py > gpurun_out/bench_1m.log 2>&1 || exit $?
