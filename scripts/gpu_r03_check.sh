# Round-3 check: the default bench, its rocprof kernel trace + stats, then the
# config-size parity tests (C2/C3 first), then the spill tests.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o prof --output-format csv -- \
  python bench.py --no-cpu-baseline --trace 0 > gpurun_out/prof.json 2> gpurun_out/prof.err || exit $?
timeout -k 10 1200 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_spill.py -m gpu -v -p no:cacheprovider \
  --timeout 900 --timeout-method thread > gpurun_out/cfg_tests.log 2>&1 || exit $?
echo done > gpurun_out/check_done.txt
