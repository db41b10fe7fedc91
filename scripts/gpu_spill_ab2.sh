# Spill tuning: tests, budget factors A/B over the whole C3 schedule, a rocprof
# kernel summary with spill on, then the C2/C3 config tests (optimizer-step
# parity).  Outputs under gpurun_out/.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_spill.py -m gpu -x -v -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/spill_tests.log 2>&1 || exit $?
B="python bench.py --no-cpu-baseline --trace 0"
TSNE_BH_SPILL=0 timeout -k 10 300 $B > gpurun_out/b_off.json 2> gpurun_out/b_off.err || exit $?
for f in 2 4 8; do
  TSNE_BH_BUDGET=$f timeout -k 10 300 $B > gpurun_out/b_f$f.json 2> gpurun_out/b_f$f.err || exit $?
done
TSNE_BH_BUDGET=4 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_spill -o prof --output-format csv -- \
  python bench.py --no-cpu-baseline --trace 0 > gpurun_out/prof_spill.json 2> gpurun_out/prof_spill.err || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py -m gpu -v -p no:cacheprovider --timeout 600 \
  --timeout-method thread -k "c2 or c3" > gpurun_out/cfg_tests.log 2>&1 || exit $?
echo done > gpurun_out/ab2_done.txt
