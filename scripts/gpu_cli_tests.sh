# GPU check of the native CLI: its host tests, the C1 / C5 CLI config tests,
# then bench.py (no CPU baseline) for the end_to_end_cli leg at C3.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r${ROUND:-6}${TAG:-x}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_host_cli.py tests/test_gpu_configs.py -m gpu -v -p no:cacheprovider \
    -k "cli or CLI" --timeout 300 --timeout-method thread > $O/cli_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/status.txt
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 600 python bench.py --no-cpu-baseline --detail-out $O/bench_detail.json > $O/bench.json 2> $O/bench.err || exit $?
echo done > $O/done.txt
