# Kernel trace of the BH repulsion on C3 snapshots (bench.py --dump-y writes
# them first): per-kernel durations of the traversal, tile_apply,
# moment_apply, ... per call, plus the counting pass (bh_snap.py --stats).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r${ROUND:-6}${TAG:-x}
SN=/tmp/snaps
mkdir -p $O $SN
timeout -k 10 300 python bench.py --no-cpu-baseline --no-cli-e2e --trace 0 --dump-y 250,450,650 --dump-dir $SN \
    --detail-out "" > $O/mksnaps.json 2> $O/mksnaps.err || exit $?
for v in ${SNAP_VARS:--}; do
  opt=""; [ "$v" != "-" ] && opt="--option ${v//+/ --option }"
  k=$((${k:-0}+1))
  echo "# $v" >> $O/snap.jsonl
  timeout -k 10 300 python scripts/bh_snap.py $SN/Y_t250.npy $SN/Y_t450.npy $SN/Y_t650.npy --reps 3 --stats $opt \
      >> $O/snap.jsonl 2>> $O/snap.err || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$k -o kt -- \
      python scripts/bh_snap.py $SN/Y_t250.npy $SN/Y_t450.npy $SN/Y_t650.npy --reps 1 $opt > $O/kt_$k.log 2>&1 || exit $?
done
echo done > $O/done.txt
