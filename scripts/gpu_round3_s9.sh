# Round 3 session 9: the 8-rank projection with heavy-wave spilling
# (TSNE_BH_SPILL=1) -- per-rank BH is bound by its heaviest waves.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_multi.py -m gpu -q -p no:cacheprovider --timeout 200 \
  --timeout-method thread > gpurun_out/s9_multi_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/s9_multi_tests.log; [ $rc -eq 0 ] || exit $rc
TSNE_BH_SPILL=1 timeout -k 10 600 python -u scripts/loop_projection.py --world 8 > gpurun_out/s9_spill2.json \
  2> gpurun_out/s9_spill2.err || exit $?
TSNE_BH_SPILL=1 TSNE_BH_BUDGET=0.5 timeout -k 10 600 python -u scripts/loop_projection.py --world 8 > gpurun_out/s9_spill05.json \
  2> gpurun_out/s9_spill05.err || exit $?
echo done > gpurun_out/s9_done.txt
