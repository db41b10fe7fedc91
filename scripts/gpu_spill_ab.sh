# Spill (dynamic splitting of heavy BH waves) on the GPU: its tests first,
# then the whole-schedule bench with spill on (default) and off, then the
# GPU parity suite.  Outputs under gpurun_out/.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_spill.py -m gpu -x -v -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/spill_tests.log 2>&1 || exit $?
B="python bench.py --no-cpu-baseline"
timeout -k 10 300 $B > gpurun_out/spill_on.json 2> gpurun_out/spill_on.err || exit $?
TSNE_BH_SPILL=0 timeout -k 10 300 $B --trace 0 > gpurun_out/spill_off.json 2> gpurun_out/spill_off.err || exit $?
TSNE_OVERLAP=none timeout -k 10 300 $B > gpurun_out/spill_on_serial.json 2> gpurun_out/spill_on_serial.err || exit $?
if [ "${RUN_SUITE:-1}" = 1 ]; then
  timeout -k 10 1200 python -u -m pytest tests -m gpu --maxfail=3 -v -p no:cacheprovider --timeout 600 \
    --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
fi
echo done > gpurun_out/spill_done.txt
