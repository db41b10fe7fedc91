# Round 3 session 5: the GPU suite (the centring mean finalised in
# combine_update's last block), the default bench line, the C4 bench line and
# its rocprofv3 kernel summary.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread \
  > gpurun_out/s5_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/s5_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/s5_bench.json 2> gpurun_out/s5_bench.err || exit $?
timeout -k 10 600 python bench.py --config c4 > gpurun_out/s5_c4.json 2> gpurun_out/s5_c4.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/s5_c4_prof -o c4 -- \
  python bench.py --config c4 --trace 0 > gpurun_out/s5_c4_prof.json 2> gpurun_out/s5_c4_prof.err || exit $?
echo done > gpurun_out/s5_done.txt
