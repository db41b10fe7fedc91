# PMC passes over the default bench (timed region = the whole schedule), one
# counter group per run: FETCH_SIZE and WRITE_SIZE of attract_tiles (the
# roofline kernel's HBM traffic), and the BH traversal's VALU issue
# (SQ_INSTS_VALU, GRBM_GUI_ACTIVE).  Summarised by scripts/pmc_r03_summary.py.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'attract_tiles' -d gpurun_out/pmc_fetch -o pmc \
  --output-format csv -- python bench.py --no-cpu-baseline --trace 0 > gpurun_out/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'attract_tiles' -d gpurun_out/pmc_write -o pmc \
  --output-format csv -- python bench.py --no-cpu-baseline --trace 0 > gpurun_out/pmc_write.log 2>&1 || exit $?
timeout -s KILL 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
  --kernel-include-regex 'bh_traverse|tile_apply' -d gpurun_out/pmc_valu -o pmc \
  --output-format csv -- python bench.py --no-cpu-baseline --trace 0 > gpurun_out/pmc_valu.log 2>&1 || exit $?
