# Round 3 session 14: 3-D update + centre in three launches (one rank) --
# 3-D tests and the C4 bench line.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_configs.py -m gpu -q \
  -p no:cacheprovider --timeout 600 --timeout-method thread -k "3 or c4" > gpurun_out/s14_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/s14_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --config c4 > gpurun_out/s14_c4.json 2> gpurun_out/s14_c4.err || exit $?
echo done > gpurun_out/s14_done.txt
