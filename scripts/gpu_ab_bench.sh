# A/B of environment-selected variants on the default bench only
# (AB_VARS="A=1,B=2 C=3 -": entries separated by spaces, variables within an
# entry by commas, "-" = defaults); each entry -> gpurun_out/ab_<k>.json.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab_index.txt
k=0
for v in ${AB_VARS:--}; do
  k=$((k+1))
  if [ "$v" = "-" ]; then v="TSNE_AB_NONE=1"; fi
  vars=$(echo "$v" | tr ',' ' ')
  env $vars timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_$k.json 2> gpurun_out/ab_$k.err || exit $?
  echo "$k $v" >> gpurun_out/ab_index.txt
done
