# Round-3 session-2 baseline: default bench, then a rocprofv3 kernel trace of it with the per-phase breakdown.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o prof --output-format csv -- \
  python bench.py --no-cpu-baseline --trace 0 > gpurun_out/prof.json 2> gpurun_out/prof.err || exit $?
python scripts/trace_iters.py gpurun_out/prof/prof_kernel_trace.csv > gpurun_out/trace_phases.txt
rm -f gpurun_out/prof/prof_kernel_trace.csv.gz
