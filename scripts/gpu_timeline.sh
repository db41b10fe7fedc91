# dense timeline of the first iterations at 1M (trace every 5th step)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --steps ${STEPS:-300} --warmup 0 --trace 5 --no-cpu-baseline > gpurun_out/timeline.json 2> gpurun_out/timeline.err
