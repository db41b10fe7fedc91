# Round-3 check: full GPU suite, headline bench + rocprof trace, the final KL
# for a second Y0 seed, and C4 probes at the default / relaxed 3-D tolerance.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof
timeout -k 10 1100 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread \
  > gpurun_out/full_tests.log 2>&1
echo "pytest rc=$?" >> gpurun_out/full_tests.log
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --trace 0 --y0-seed 1 > gpurun_out/bench_seed1.json 2> gpurun_out/bench_seed1.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o prof --output-format csv -- \
  python bench.py --no-cpu-baseline --trace 0 > gpurun_out/prof.json 2> gpurun_out/prof.err || exit $?
python scripts/trace_iters.py gpurun_out/prof/prof_kernel_trace.csv > gpurun_out/trace_phases.txt
python scripts/trace_kernels.py gpurun_out/prof/prof_kernel_trace.csv > gpurun_out/trace_kernels.txt
rm -f gpurun_out/prof/prof_kernel_trace.csv.gz
timeout -k 10 300 python scripts/c4_probe.py --cap 120 > gpurun_out/c4_default.jsonl 2> gpurun_out/c4_default.err || exit $?
TSNE_BH_NEAR_TOL3=5e-6 TSNE_MOM3_TOL=1e-12 timeout -k 10 300 python scripts/c4_probe.py --cap 120 \
  > gpurun_out/c4_nt5.jsonl 2> gpurun_out/c4_nt5.err || exit $?
