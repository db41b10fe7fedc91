set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5g; mkdir -p $O
for v in - ab/libtsne_hip_atdiag1.so ab/libtsne_hip_atdiag2.so -; do
  lib=""; [ "$v" != "-" ] && lib=$v
  echo "# $v" >> $O/diag.jsonl
  TSNE_HIP_LIB="$lib" timeout -k 10 200 python bench.py --no-cpu-baseline --trace 0 --iterations 20 --steps 20 --warmup 1 --detail-out "" >> $O/diag.jsonl 2>> $O/diag.err || exit $?
done
for v in - bu_acqrel=1 - bu_acqrel=1; do
  opt=""; [ "$v" != "-" ] && opt="--option $v"
  echo "# $v" >> $O/bench.jsonl
  timeout -k 10 300 python bench.py --no-cpu-baseline --trace 0 $opt --detail-out "" >> $O/bench.jsonl 2>> $O/bench.err || exit $?
done
