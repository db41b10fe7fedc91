# The native CLI (tsne_hip, Tsne.main's flags and formats) end to end at C3:
# 1M x 128 GMM written as the reference's COO input (128M "i,j,v" lines),
# parsed, kNN, affinities, joint, 1000 iterations, embedding CSV + loss file
# written.  Input generation is not timed.  Outputs under gpurun_out/.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
W=/tmp/tsne_cli_c3
mkdir -p $W
timeout -k 10 300 python -c "
import sys; sys.path.insert(0, 'tests')
import configs, torch
X = configs.c3_torch(1_000_000, 128, 2, torch.device('cuda', 0)).cpu().numpy()
X.astype('<f8').tofile('$W/x.bin')
" || exit $?
timeout -k 10 300 scripts/coo_write $W/x.bin 1000000 128 $W/c3.csv || exit $?
ls -la $W/c3.csv > gpurun_out/cli_c3_input.txt
t0=$(date +%s.%N); timeout -k 10 600 tsne-flink_amd/tsne_hip --input $W/c3.csv --output $W/y.csv --dimension 128 \
  --knnMethod bruteforce --metric sqeuclidean --perplexity 30 --iterations 1000 --theta 0.5 --loss $W/loss.txt \
  > gpurun_out/cli_c3.log 2>&1 || { tail -20 gpurun_out/cli_c3.log; exit 1; }
python3 -c "import sys; print('wall %.3f s' % (float(sys.argv[2]) - float(sys.argv[1])))" $t0 $(date +%s.%N) >> gpurun_out/cli_c3.log
head -c 300 $W/loss.txt > gpurun_out/cli_c3_loss_head.txt
wc -l $W/y.csv >> gpurun_out/cli_c3_input.txt
rm -rf $W
