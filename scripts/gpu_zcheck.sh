set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/zcheck.py 300 > gpurun_out/zcheck.txt 2>&1 || exit $?
TSNE_TILE_CHUNK=0 timeout -k 10 300 python -u scripts/zcheck.py 300 > gpurun_out/zcheck_nochunk.txt 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py -m gpu -v -p no:cacheprovider \
  -k "c2 or c5_distance_matrix_50k" --timeout 600 --timeout-method thread > gpurun_out/cfg_tests.log 2>&1
