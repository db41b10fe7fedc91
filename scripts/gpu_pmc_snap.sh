# PMC passes (one counter group per run, as MI355X_MICROARCH.md prescribes)
# over scripts/bh_snap.py on C3 snapshots: bh_traverse / tile_apply /
# moment_apply, plus GRBM_GUI_ACTIVE for the cycle base.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out /tmp/snaps
SNAPS=${SNAPS:-250,500}
timeout -k 10 300 python bench.py --no-cpu-baseline --trace 0 --dump-y $SNAPS --dump-dir /tmp/snaps \
  > gpurun_out/snap_bench.json 2> gpurun_out/snap_bench.err || exit $?
files=$(for t in $(echo $SNAPS | tr ',' ' '); do echo /tmp/snaps/Y_t$t.npy; done)
k=0
for pass in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
            "SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE" \
            "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"; do
  k=$((k+1))
  timeout -s KILL 180 rocprofv3 --pmc $pass --kernel-include-regex "bh_traverse|tile_apply|moment_apply" \
    -d gpurun_out/pmcs_$k -o pmc --output-format csv -- python scripts/bh_snap.py $files --reps 1 \
    > gpurun_out/pmcs_$k.log 2>&1 || exit $?
done
echo done > gpurun_out/pmcs_done.txt
