# BH traversal variants (records per batch x XCD block order) over t = 1..300 at 1M, then a
# rocprofv3 kernel-stats run of the default variant
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "4 0" "8 0" "4 1" "1 0"; do
  set -- $v
  TSNE_BH_KPOP=$1 TSNE_BH_XCD=$2 timeout -k 10 300 python bench.py --steps 300 --warmup 0 --trace 10 --no-cpu-baseline \
    > gpurun_out/bhv_$1_$2.json 2> gpurun_out/bhv_$1_$2.err || exit $?
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof300 -o prof --output-format csv -- \
  python bench.py --steps 300 --warmup 0 --trace 0 --no-cpu-baseline > gpurun_out/prof300.log 2>&1 || exit $?
