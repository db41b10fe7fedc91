# A/B of environment-selected variants: GPU parity suite with defaults, the
# BH/optimizer parity tests under each AB_VARS entry, then the full bench per
# entry (AB_VARS="NAME=VAL ..."; "-" = defaults)
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
  if [ "$v" = "-" ]; then v="TSNE_AB_NONE=1"; fi
  env "$v" timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "${AB_TESTS:-gradient or optimize}" > gpurun_out/ab_tests_$k.log 2>&1 || exit $?
  env "$v" timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/ab_$k.json 2> gpurun_out/ab_$k.err || exit $?
  echo "$k $v" >> gpurun_out/ab_index.txt
done
