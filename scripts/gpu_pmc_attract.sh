# HBM traffic of attract_rows from PMC (separate FETCH_SIZE / WRITE_SIZE passes,
# MI355X_MICROARCH.md "HBM"), over the first 300 iterations at 1M
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex attract_rows -d gpurun_out/pmc_fetch -o pmc --output-format csv -- \
  python bench.py --steps 300 --warmup 0 --trace 0 --no-cpu-baseline > gpurun_out/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex attract_rows -d gpurun_out/pmc_write -o pmc --output-format csv -- \
  python bench.py --steps 300 --warmup 0 --trace 0 --no-cpu-baseline > gpurun_out/pmc_write.log 2>&1 || exit $?
