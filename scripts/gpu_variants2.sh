# tests; attraction (persistent) variants; BH chunked-XCD variants; t = 1..300 at 1M
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
for v in 64x4 32x8 16x12; do
  TSNE_ATTRACT=$v timeout -k 10 300 python bench.py --steps 300 --warmup 0 --trace 10 --no-cpu-baseline > gpurun_out/av_$v.json 2> gpurun_out/av_$v.err || exit $?
done
for c in 4 16 64; do
  TSNE_BH_XCD=$c timeout -k 10 300 python bench.py --steps 300 --warmup 0 --trace 10 --no-cpu-baseline > gpurun_out/bx_$c.json 2> gpurun_out/bx_$c.err || exit $?
done
