# Round 4 GPU session script: STEP selects what runs (each GPU step under its own time limit).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4${TAG:-x}
mkdir -p $O
run() { local lim=$1; shift; timeout -k 10 $lim "$@"; }
if [[ "${STEPS:-}" == *snap* ]]; then
  for v in ${SNAP_VARS:--}; do
    opt=""; [ "$v" != "-" ] && opt="--option $v"
    echo "# $v" >> $O/snap.jsonl
    run 300 python scripts/bh_snap.py snaps/Y_t250.npy snaps/Y_t450.npy snaps/Y_t650.npy $opt >> $O/snap.jsonl 2>> $O/snap.err || exit $?
  done
fi
if [[ "${STEPS:-}" == *tests_narrow* ]]; then
  run 900 python -u -m pytest tests/test_gpu_narrow.py tests/test_gpu_parity.py -x -v -p no:cacheprovider \
      --timeout 300 --timeout-method thread > $O/tests_narrow.log 2>&1 || exit $?
fi
if [[ "${STEPS:-}" == *bench* ]]; then
  for v in ${BENCH_VARS:--}; do
    opt=""; [ "$v" != "-" ] && opt="--option $v"
    echo "# $v" >> $O/bench.jsonl
    run 400 python bench.py --no-cpu-baseline $opt >> $O/bench.jsonl 2>> $O/bench.err || exit $?
  done
fi
if [[ "${STEPS:-}" == *tests3d* ]]; then
  run 900 python -u -m pytest tests/test_gpu_narrow.py tests/test_gpu_parity.py tests/test_gpu_multi.py -x -v \
      -p no:cacheprovider --timeout 300 --timeout-method thread -k "octal or gradient3 or optimize3" \
      > $O/tests3d.log 2>&1 || exit $?
fi
if [[ "${STEPS:-}" == *bench4* ]]; then
  for v in ${BENCH4_VARS:--}; do
    opt=""; [ "$v" != "-" ] && opt="--option $v"
    echo "# $v" >> $O/bench4.jsonl
    run 600 python bench.py --config c4 --no-cpu-baseline $opt >> $O/bench4.jsonl 2>> $O/bench4.err || exit $?
  done
fi
if [[ "${STEPS:-}" == *ktrace* ]]; then
  run 600 rocprofv3 --kernel-trace --output-format csv -d $O/ktrace -o kt -- python bench.py --no-cpu-baseline --trace 0 ${KTRACE_ARGS:-} > $O/ktrace_bench.json 2> $O/ktrace.err || exit $?
fi
if [[ "${STEPS:-}" == *tests_all* ]]; then
  run 1100 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 600 --timeout-method thread \
      > $O/tests_all.log 2>&1 || exit $?
fi
echo done > $O/done.txt
