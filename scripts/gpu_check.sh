# Round check on one MI355X: GPU parity suite, smoke(), the default bench
# (driver command), rocprofv3 kernel trace + stats of the same bench, PMC
# FETCH_SIZE / WRITE_SIZE passes over the bench's timed window (the attraction kernel),
# and the FETCH_SIZE width calibration (scripts/pmc_calib.hip).
# Outputs under gpurun_out/ (copied to profiles/rNN_* by hand).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS=${STEPS:-20}
WARM=${WARM:-5}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
    ${TESTS_K:+-k "$TESTS_K"} > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
  if [ $rc -ne 0 ]; then exit $rc; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  timeout -k 10 600 python bench.py --steps $STEPS --warmup $WARM > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
fi
if [ "${SKIP_PROF:-0}" != 1 ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o prof --output-format csv -- \
    python bench.py --steps $STEPS --warmup $WARM --no-cpu-baseline > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err || exit $?
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'attract_(rows|tiles)' -d gpurun_out/pmc_fetch -o pmc --output-format csv -- \
    python bench.py --steps $STEPS --warmup $WARM --no-rest --no-cpu-baseline --trace 0 > gpurun_out/pmc_fetch.log 2>&1 || exit $?
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'attract_(rows|tiles)' -d gpurun_out/pmc_write -o pmc --output-format csv -- \
    python bench.py --steps $STEPS --warmup $WARM --no-rest --no-cpu-baseline --trace 0 > gpurun_out/pmc_write.log 2>&1 || exit $?
  if [ -x scripts/pmc_calib ]; then
    timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_calib_fetch -o pmc --output-format csv -- \
      scripts/pmc_calib > gpurun_out/pmc_calib_fetch.log 2>&1 || exit $?
    timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_calib_write -o pmc --output-format csv -- \
      scripts/pmc_calib > gpurun_out/pmc_calib_write.log 2>&1 || exit $?
  fi
fi
echo done > gpurun_out/check_done.txt
