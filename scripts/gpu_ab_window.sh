# A/B of environment-selected variants on the bench's timed window only
# (bench.py --no-rest: t = 1..K, value = window it/s; AB_FULL=1: the whole
# schedule too), one bench per entry.
# AB_VARS="A=1,B=2 C=3 -": entries separated by spaces, variables of one entry
# by commas; "-" = defaults.  Optional AB_TESTS: a pytest -k filter run first
# under each entry.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
k=0
for v in ${AB_VARS:--}; do
  k=$((k+1))
  if [ "$v" = "-" ]; then v="TSNE_AB_NONE=1"; fi
  vars=$(echo "$v" | tr ',' ' ')
  if [ -n "${AB_TESTS:-}" ]; then
    env $vars timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
      --timeout-method thread -k "$AB_TESTS" > gpurun_out/abw_tests_$k.log 2>&1 || exit $?
  fi
  rest="--no-rest"; if [ "${AB_FULL:-0}" = 1 ]; then rest=""; fi
  env $vars timeout -k 10 300 python bench.py $rest --no-cpu-baseline --trace 0 ${AB_BENCH_ARGS:-} \
    > gpurun_out/abw_$k.json 2> gpurun_out/abw_$k.err || exit $?
  echo "$k $v" >> gpurun_out/abw_index.txt
done
