# Round 3 session 10: pops per traversal step (TSNE_BH_KPOP 8 / 16 vs the
# default 4) at world 1 and in the 8-rank loopback projection.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TSNE_BH_KPOP=8 timeout -k 10 600 python -u scripts/loop_projection.py --world 8 > gpurun_out/s10_kp8.json \
  2> gpurun_out/s10_kp8.err || exit $?
TSNE_BH_KPOP=16 timeout -k 10 600 python -u scripts/loop_projection.py --world 8 > gpurun_out/s10_kp16.json \
  2> gpurun_out/s10_kp16.err || exit $?
echo done > gpurun_out/s10_done.txt
