# BH repulsion on C3 schedule snapshots: the bench writes Y at the given
# iterations (to /tmp on the box), then scripts/bh_snap.py times
# tsne_dev_repulsion on each, per AB_VARS entry (as gpu_ab_window.sh), and
# once under rocprofv3 --kernel-trace --stats with the defaults.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out /tmp/snaps
SNAPS=${SNAPS:-200,250,300,400,500,700}
timeout -k 10 300 python bench.py --no-cpu-baseline --trace 0 --dump-y $SNAPS --dump-dir /tmp/snaps \
  > gpurun_out/snap_bench.json 2> gpurun_out/snap_bench.err || exit $?
files=$(for t in $(echo $SNAPS | tr ',' ' '); do echo /tmp/snaps/Y_t$t.npy; done)
k=0
for v in ${AB_VARS:--}; do
  k=$((k+1))
  if [ "$v" = "-" ]; then v="TSNE_AB_NONE=1"; fi
  vars=$(echo "$v" | tr ',' ' ')
  echo "# $v" > gpurun_out/snap_$k.jsonl
  env $vars timeout -k 10 300 python scripts/bh_snap.py $files >> gpurun_out/snap_$k.jsonl 2> gpurun_out/snap_$k.err || exit $?
done
if [ "${SNAP_PROF:-1}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/snapprof -o prof --output-format csv -- \
    python scripts/bh_snap.py $files --reps 2 > gpurun_out/snapprof.jsonl 2> gpurun_out/snapprof.err || exit $?
fi
echo done > gpurun_out/snap_done.txt
