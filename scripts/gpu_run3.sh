# GPU session: parity tests + default bench (full 1M schedule) + 200k full.
set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --n 200000 --no-cpu-baseline > gpurun_out/bench_200k.log 2>&1 || exit $?
timeout -k 10 900 python bench.py > gpurun_out/bench_1m.log 2>&1 || exit $?
