# PMC passes over the kNN filter (knn_filter_glds) of the C3 setup: MFMA busy,
# LDS bank conflicts and waits, instruction mix (one counter group per run).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python bench.py --steps 1 --warmup 0 --no-rest --no-cpu-baseline --trace 0"
k=0
for pass in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
            "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_MFMA SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"; do
  k=$((k+1))
  timeout -s KILL 240 rocprofv3 --pmc $pass --kernel-include-regex "knn_filter_glds" \
    -d gpurun_out/pmck_$k -o pmc --output-format csv -- $B > gpurun_out/pmck_$k.log 2>&1 || exit $?
done
echo done > gpurun_out/pmck_done.txt
