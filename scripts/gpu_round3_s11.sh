# Round 3 session 11: kernel summary of the 8-rank loopback run (serial
# turns), to see which kernels make up a rank's BH stretch.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s11_prof -o w8 -- \
  python -u scripts/loop_projection.py --world 8 --skip-single > gpurun_out/s11_w8.json 2> gpurun_out/s11_w8.err || exit $?
rm -f gpurun_out/s11_prof/*kernel_trace.csv gpurun_out/s11_prof/*.db
echo done > gpurun_out/s11_done.txt
