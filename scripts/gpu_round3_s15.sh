# Round 3 session 15: the whole GPU suite and smoke() on the final tree.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread \
  > gpurun_out/s15_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/s15_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/s15_smoke.log 2>&1 || exit $?
echo done > gpurun_out/s15_done.txt
