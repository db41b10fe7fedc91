# parity tests, then the full bench once per variant: AB_VARS="NAME=VAL ..." ("-" = defaults)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
k=0
for v in ${AB_VARS:--}; do
  k=$((k+1))
  if [ "$v" = "-" ]; then
    timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/ab_$k.json 2> gpurun_out/ab_$k.err || exit $?
  else
    env "$v" timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/ab_$k.json 2> gpurun_out/ab_$k.err || exit $?
  fi
  echo "$k $v" >> gpurun_out/ab_index.txt
done
