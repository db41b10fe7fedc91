# rocprofv3 kernel trace + stats over the whole default schedule (C3, 1M)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o prof --output-format csv -- \
  python bench.py --trace 0 --no-cpu-baseline > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err || exit $?
