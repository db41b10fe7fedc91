# Iteration check: parity tests (all but the config-size ones), the default
# bench, and a rocprofv3 kernel trace of it with per-phase / per-kernel tables.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_spill.py tests/test_gpu_multi.py -m gpu -x -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/quick_tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o prof --output-format csv -- \
  python bench.py --no-cpu-baseline --trace 0 > gpurun_out/prof.json 2> gpurun_out/prof.err || exit $?
python scripts/trace_iters.py gpurun_out/prof/prof_kernel_trace.csv > gpurun_out/trace_phases.txt
python scripts/trace_kernels.py gpurun_out/prof/prof_kernel_trace.csv > gpurun_out/trace_kernels.txt
rm -f gpurun_out/prof/prof_kernel_trace.csv.gz
