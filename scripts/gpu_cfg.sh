# The config-size parity tests alone (optionally a -k filter as $1).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
K=${1:-}
timeout -k 10 1100 python -u -m pytest tests/test_gpu_configs.py -m gpu -v -p no:cacheprovider \
  ${K:+-k "$K"} --timeout 900 --timeout-method thread > gpurun_out/cfg_tests.log 2>&1
rc=$?
echo "rc=$rc" > gpurun_out/cfg_done.txt
exit $rc
