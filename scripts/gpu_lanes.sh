# tests (default L = 4 lanes per query), then t = 1..700 timelines for L = 1, 2, 4
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
for L in 4 2 1; do
  TSNE_BH_LANES=$L timeout -k 10 300 python bench.py --steps 700 --warmup 0 --trace 10 --no-cpu-baseline > gpurun_out/lanes_$L.json 2> gpurun_out/lanes_$L.err || exit $?
done
