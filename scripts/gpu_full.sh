# Full GPU test suite, then the default bench (headline) with a rocprof trace.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof
timeout -k 10 1100 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread \
  > gpurun_out/full_tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o prof --output-format csv -- \
  python bench.py --no-cpu-baseline --trace 0 > gpurun_out/prof.json 2> gpurun_out/prof.err || exit $?
python scripts/trace_iters.py gpurun_out/prof/prof_kernel_trace.csv > gpurun_out/trace_phases.txt
python scripts/trace_kernels.py gpurun_out/prof/prof_kernel_trace.csv > gpurun_out/trace_kernels.txt
rm -f gpurun_out/prof/prof_kernel_trace.csv.gz
