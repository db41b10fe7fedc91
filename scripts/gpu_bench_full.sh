# full default bench (whole 1000-iteration schedule at 1M x 128) with progress on stderr
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
