# rocprofv3 kernel-trace summary of a short 1M bench (kNN + setup + 4 iterations).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- \
  python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof1_bench.log 2>&1 || exit $?
find gpurun_out/prof1 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/prof1_kernel_stats.csv
