# 3-D (octree) tests and the C4 probe with the phase-split tolerance.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_configs.py -m gpu -q \
  -p no:cacheprovider --timeout 600 --timeout-method thread -k "3 or c4" > gpurun_out/c4_tests.log 2>&1
echo "pytest rc=$?" >> gpurun_out/c4_tests.log
timeout -k 10 300 python scripts/c4_probe.py --cap 120 > gpurun_out/c4_split.jsonl 2> gpurun_out/c4_split.err || exit $?
