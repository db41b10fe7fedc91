# Parity tests (all but the config-size ones) + the default bench.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_spill.py tests/test_gpu_multi.py -m gpu -x -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/quick_tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
echo done > gpurun_out/quick_done.txt
