# Chaotic spread of the C3 final KL: the bench's schedule from Y0 perturbed by
# 1e-15 (relative, seeds 1..3) at the default near-exact tolerance, and at
# TSNE_BH_NEAR_TOL=1e-5 (seeds 0 = unperturbed, 1, 2).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for s in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --trace 0 --y0-perturb 1e-15 --y0-perturb-seed $s \
    > gpurun_out/kl_def_$s.json 2> gpurun_out/kl_def_$s.err || exit $?
done
for s in 1 2; do
  TSNE_BH_NEAR_TOL=1e-5 TSNE_MOM_TOL=1e-12 timeout -k 10 300 python bench.py --no-cpu-baseline --trace 0 \
    --y0-perturb 1e-15 --y0-perturb-seed $s > gpurun_out/kl_nt5_$s.json 2> gpurun_out/kl_nt5_$s.err || exit $?
done
