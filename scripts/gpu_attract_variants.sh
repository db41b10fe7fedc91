# parity tests; attraction kernel variants (lanes per row x unroll) on 1M, 30 steps; full bench
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for v in 64x4 32x8 16x12; do
  TSNE_ATTRACT=$v timeout -k 10 300 python bench.py --steps 30 --warmup 0 --trace 5 --no-cpu-baseline > gpurun_out/attract_$v.json 2> gpurun_out/attract_$v.err || exit $?
done
timeout -k 10 1000 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
