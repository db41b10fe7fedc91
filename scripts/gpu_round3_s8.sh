# Round 3 session 8: the loopback projection with per-phase marks (tree /
# BH / attraction + Z) at 8, 4 and 2 ranks.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/loop_projection.py --world 8 > gpurun_out/s8_proj8.json 2> gpurun_out/s8_proj8.err || exit $?
timeout -k 10 600 python -u scripts/loop_projection.py --world 4 --skip-single > gpurun_out/s8_proj4.json \
  2> gpurun_out/s8_proj4.err || exit $?
timeout -k 10 600 python -u scripts/loop_projection.py --world 2 --skip-single > gpurun_out/s8_proj2.json \
  2> gpurun_out/s8_proj2.err || exit $?
echo done > gpurun_out/s8_done.txt
