# A/B of the attraction's placement over the whole C3 schedule (TSNE_OVERLAP:
# default = side stream beside the tree build / BH, none = serial on the
# context stream), then the GPU parity suite.  Outputs under gpurun_out/.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python bench.py --no-cpu-baseline"
timeout -k 10 300 $B > gpurun_out/ab_default.json 2> gpurun_out/ab_default.err || exit $?
TSNE_OVERLAP=none timeout -k 10 300 $B --trace 0 > gpurun_out/ab_none.json 2> gpurun_out/ab_none.err || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=3 -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1 || exit $?
echo done > gpurun_out/ab_done.txt
