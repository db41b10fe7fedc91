# GPU session: parity tests, 1M bench, 200k end-to-end timeline.
set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --cpu-sample 64 > gpurun_out/bench_1m.log 2>&1 || exit $?
timeout -k 10 500 python bench.py --n 200000 --steps 5 --warmup 1 --full --trace 50 --no-cpu-baseline > gpurun_out/bench_200k.log 2> gpurun_out/trace_200k.log || exit $?
