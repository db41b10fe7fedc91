# Spill tests, the default bench (headline) with a rocprof trace, then the
# chaotic-spread runs of the final KL (scripts/gpu_kl_spread.sh).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof
timeout -k 10 400 python -u -m pytest tests/test_gpu_spill.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/spill_tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o prof --output-format csv -- \
  python bench.py --no-cpu-baseline --trace 0 > gpurun_out/prof.json 2> gpurun_out/prof.err || exit $?
python scripts/trace_iters.py gpurun_out/prof/prof_kernel_trace.csv > gpurun_out/trace_phases.txt
python scripts/trace_kernels.py gpurun_out/prof/prof_kernel_trace.csv > gpurun_out/trace_kernels.txt
rm -f gpurun_out/prof/prof_kernel_trace.csv.gz
for s in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --trace 0 --y0-perturb 1e-15 --y0-perturb-seed $s \
    > gpurun_out/kl_$s.json 2> gpurun_out/kl_$s.err || exit $?
done
for s in 1 2; do
  TSNE_BH_NEAR_TOL=1e-6 TSNE_MOM_TOL=1e-14 timeout -k 10 300 python bench.py --no-cpu-baseline --trace 0 \
    --y0-perturb 1e-15 --y0-perturb-seed $s > gpurun_out/kl_old_$s.json 2> gpurun_out/kl_old_$s.err || exit $?
done
