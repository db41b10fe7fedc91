# PMC passes over the default bench (timed region = the whole schedule), one
# counter group per run: FETCH_SIZE and WRITE_SIZE of the gradient kernels
# (attract_tiles -- the roofline kernel -- combine_update, center2),
# and the BH traversal's VALU issue (SQ_INSTS_VALU, GRBM_GUI_ACTIVE).
# Summarised by `python scripts/pmc_summary.py <tag>` into profiles/<tag>_*.json.
# Env: PMC_ARGS (extra bench arguments).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python bench.py --no-cpu-baseline --no-cli-e2e --trace 0 ${PMC_ARGS:-}"
R='attract_tiles|combine_update|center2'
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$R" -d gpurun_out/pmc_fetch -o pmc \
  --output-format csv -- $B > gpurun_out/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$R" -d gpurun_out/pmc_write -o pmc \
  --output-format csv -- $B > gpurun_out/pmc_write.log 2>&1 || exit $?
timeout -s KILL 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
  --kernel-include-regex 'bh_traverse|tile_apply' -d gpurun_out/pmc_valu -o pmc \
  --output-format csv -- $B > gpurun_out/pmc_valu.log 2>&1 || exit $?
