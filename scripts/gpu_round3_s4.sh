# 3-D check (tests + C4 probe), then the PMC passes of scripts/gpu_pmc_r03.sh.
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_c4_check.sh || exit $?
bash scripts/gpu_pmc_r03.sh || exit $?
