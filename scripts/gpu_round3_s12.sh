# Round 3 session 12: final check of the tree -- the whole GPU suite, smoke(),
# and the default bench line.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread \
  > gpurun_out/s12_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/s12_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/s12_smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/s12_bench.json 2> gpurun_out/s12_bench.err || exit $?
echo done > gpurun_out/s12_done.txt
