# Round 3 session 7: octree dense tiles with the next chunk prefetched --
# 3-D tests, the C4 loop, and the traversal counters through the transition.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_configs.py -m gpu -q \
  -p no:cacheprovider --timeout 600 --timeout-method thread -k "3 or c4" > gpurun_out/s7_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/s7_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/c4_probe.py --cap 120 > gpurun_out/s7_c4.jsonl 2> gpurun_out/s7_c4.err || exit $?
TSNE_DEBUG_OCT=1 timeout -k 10 300 python scripts/c4_probe.py --iterations 1000 --cap 25 > gpurun_out/s7_c4_dbg.jsonl \
  2> gpurun_out/s7_c4_dbg.err || exit $?
echo done > gpurun_out/s7_done.txt
