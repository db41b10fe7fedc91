# Round 3 session 6: loopback multi-rank tests (serial-turn timing mode added
# to LoopGroup), the 8-rank projection (default ownership, and TSNE_RECUT=1),
# the C4 bench line and its rocprofv3 kernel summary (csv).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_multi.py -m gpu -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/s6_multi_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/s6_multi_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/loop_projection.py > gpurun_out/s6_proj.json 2> gpurun_out/s6_proj.err || exit $?
TSNE_RECUT=1 timeout -k 10 600 python -u scripts/loop_projection.py --skip-single > gpurun_out/s6_proj_recut.json \
  2> gpurun_out/s6_proj_recut.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s6_c4_prof -o c4 -- \
  python bench.py --config c4 --trace 0 > gpurun_out/s6_c4_prof.json 2> gpurun_out/s6_c4_prof.err || exit $?
timeout -k 10 600 python bench.py --config c4 > gpurun_out/s6_c4.json 2> gpurun_out/s6_c4.err || exit $?
echo done > gpurun_out/s6_done.txt
