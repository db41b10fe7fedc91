# GPU session script: STEPS (space-separated) selects what runs, each GPU step
# under its own time limit, outputs under gpurun_out/r${ROUND:-5}$TAG/:
#   driver      bench.py exactly as the driver runs it (--gpus 1 --steps 20 --warmup 5, CPU baseline included)
#   mksnaps     bench.py --dump-y 250,450,650 into /tmp/snaps (the snapshots the snap steps read)
#   snap        bh_snap.py on snaps/Y_t{250,450,650}.npy per SNAP_VARS entry ("-" = defaults, else KEY=VALUE;
#               SNAP_ARGS: more bh_snap arguments, e.g. --stats)
#   tests_narrow / tests_spill / tests_stream / tests_attr / tests3d / tests_all   GPU test subsets / the whole -m gpu suite
#   bench / bench4   bench.py (C3 / C4) per BENCH_VARS / BENCH4_VARS entry ("K1=V1+K2=V2": two options)
#   ktrace      rocprofv3 --kernel-trace --stats of the default bench (KTRACE_ARGS)
#   smoke       __graft_entry__.smoke()
#   pmc         scripts/gpu_pmc.sh (summarise with scripts/pmc_summary.py <tag>)
#   c4probe     scripts/c4_probe.py C4PROBE_ARGS
#   snap3       C4 snapshots (SNAP3_T) written by c4_probe, timed per SNAP3_VARS, debug counters, PMC
#   pmcsnap     PMC passes (SQ waits / LDS / VALU) over the BH kernels on snaps/Y_t{250,650}.npy
#   proj        scripts/loop_projection.py PROJ_ARGS per PROJ_VARS entry
#   valusnap    VALU / SALU / LDS instructions per wave pop of bh_traverse on snapshots t = 250, 450,
#               per VALU_LIBS library (scripts/valu_summary.py)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r${ROUND:-5}${TAG:-x}
SN=/tmp/snaps
mkdir -p $O
run() { local lim=$1; shift; timeout -k 10 $lim "$@"; }
# a test step's failures do not stop the session; a time limit, abort or crash does
tst() { run "$@"; local rc=$?; echo "tests rc=$rc" >> $O/status.txt; case $rc in 0|1) return 0;; *) return $rc;; esac; }
has() { [[ " ${STEPS:-} " == *" $1 "* ]]; }
if has driver; then
  run 600 python bench.py --gpus 1 --steps 20 --warmup 5 --detail-out $O/bench_detail.json > $O/driver_bench.json 2> $O/driver_bench.err || exit $?
fi
if has mksnaps; then
  mkdir -p $SN
  run 300 python bench.py --no-cpu-baseline --trace 0 --dump-y 250,450,650 --dump-dir $SN --detail-out "" > $O/mksnaps.json 2> $O/mksnaps.err || exit $?
fi
if has snap; then
  for v in ${SNAP_VARS:--}; do
    opt=""; [ "$v" != "-" ] && opt="--option ${v//+/ --option }"
    echo "# $v" >> $O/snap.jsonl
    run 300 python scripts/bh_snap.py $SN/Y_t250.npy $SN/Y_t450.npy $SN/Y_t650.npy $opt ${SNAP_ARGS:-} >> $O/snap.jsonl 2>> $O/snap.err || exit $?
  done
fi
if has tests_narrow; then
  TSNE_HIP_LIB="${TESTS_LIB:-}" tst 900 python -u -m pytest tests/test_gpu_csort.py tests/test_gpu_narrow.py tests/test_gpu_parity.py -v -p no:cacheprovider \
      --timeout 300 --timeout-method thread > $O/tests_narrow.log 2>&1 || exit $?
fi
if has tests_spill; then
  tst 900 python -u -m pytest tests/test_gpu_spill.py -v -p no:cacheprovider \
      --timeout 300 --timeout-method thread > $O/tests_spill.log 2>&1 || exit $?
fi
if has tests_stream; then
  tst 600 python -u -m pytest tests/test_gpu_stream.py -v -p no:cacheprovider \
      --timeout 300 --timeout-method thread > $O/tests_stream.log 2>&1 || exit $?
fi
if has tests_attr; then
  tst 600 python -u -m pytest tests/test_gpu_parity.py -v -p no:cacheprovider -k "tiled_attraction" \
      --timeout 300 --timeout-method thread > $O/tests_attr.log 2>&1 || exit $?
fi
if has tests_multi; then
  tst 900 python -u -m pytest tests/test_gpu_multi.py -v -p no:cacheprovider \
      --timeout 300 --timeout-method thread > $O/tests_multi.log 2>&1 || exit $?
fi
if has bench; then
  for v in ${BENCH_VARS:--}; do
    # "-": defaults; "lib=PATH": another build of the library (TSNE_HIP_LIB); else KEY=VALUE options
    opt=""; lib=""
    case "$v" in -) ;; lib=*) lib="${v#lib=}" ;; *) opt="--option ${v//+/ --option }" ;; esac
    bi=$((${bi:-0}+1))
    echo "# $v" >> $O/bench.jsonl
    TSNE_HIP_LIB="$lib" run 400 python bench.py --no-cpu-baseline --no-cli-e2e $opt --detail-out $O/bench_detail_$bi.json >> $O/bench.jsonl 2>> $O/bench.err || exit $?
  done
fi
if has tests3d; then
  tst 900 python -u -m pytest tests/test_gpu_narrow.py tests/test_gpu_parity.py tests/test_gpu_multi.py \
      tests/test_gpu_configs.py tests/test_gpu_csort.py -v -p no:cacheprovider --timeout 300 --timeout-method thread \
      -k "octal or gradient3 or optimize3 or c4 or C4 or 3d or csort or coherent" \
      > $O/tests3d.log 2>&1 || exit $?
fi
if has bench4; then
  for v in ${BENCH4_VARS:--}; do
    opt=""; lib=""
    case "$v" in -) ;; lib=*) lib="${v#lib=}" ;; *) opt="--option $v" ;; esac
    echo "# $v" >> $O/bench4.jsonl
    TSNE_HIP_LIB="$lib" run 600 python bench.py --config c4 --no-cpu-baseline $opt >> $O/bench4.jsonl 2>> $O/bench4.err || exit $?
  done
fi
if has ktrace; then
  run 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o kt -- python bench.py --no-cpu-baseline --no-cli-e2e --trace 0 ${KTRACE_ARGS:-} > $O/ktrace_bench.json 2> $O/ktrace.err || exit $?
fi
if has tests_all; then
  tst 1100 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread \
      > $O/tests_all.log 2>&1 || exit $?
fi
if has smoke; then
  run 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
fi
if has pmc; then
  run 1300 bash scripts/gpu_pmc.sh || exit $?
fi
if has c4probe; then
  for v in ${C4PROBE_VARS:--}; do
    opt=""; [ "$v" != "-" ] && opt="--option $v"
    echo "# $v" >> $O/c4probe.log
    run 300 python scripts/c4_probe.py ${C4PROBE_ARGS:-} $opt >> $O/c4probe.log 2>&1 || exit $?
  done
fi
if has snap3; then   # C4 snapshots in the transition, timed, counted and PMC-profiled
  S3=${SNAP3_T:-120,150,180}
  mkdir -p /tmp/snap3
  run 400 python scripts/c4_probe.py --stop ${S3##*,} --cap 200 --dump-y $S3 --dump-dir /tmp/snap3 > $O/snap3_probe.log 2>&1 || exit $?
  files=$(for t in $(echo $S3 | tr ',' ' '); do echo /tmp/snap3/Y3_t$t.npy; done)
  for v in ${SNAP3_VARS:--}; do
    opt=""; [ "$v" != "-" ] && opt="--option $v"
    echo "# $v" >> $O/snap3.jsonl
    run 300 python scripts/bh_snap.py $files --reps 3 $opt >> $O/snap3.jsonl 2>> $O/snap3.err || exit $?
  done
  TSNE_DEBUG_OCT=1 run 300 python scripts/bh_snap.py $files --reps 0 ${SNAP3_PMC_OPT:-} > $O/snap3_dbg.jsonl 2> $O/snap3_dbg.err || exit $?
  k=0
  for pass in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
              "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"; do
    k=$((k+1))
    timeout -s KILL 180 rocprofv3 --pmc $pass --kernel-include-regex "oct_" -d $O/pmc3_$k -o pmc --output-format csv -- \
      python scripts/bh_snap.py $files --reps 0 ${SNAP3_PMC_OPT:-} > $O/pmc3_$k.log 2>&1 || exit $?
  done
fi
if has pmcsnap; then   # PMC passes over the 2-D BH kernels on the committed C3 snapshots
  k=0
  for pass in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
              "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
    k=$((k+1))
    timeout -s KILL 180 rocprofv3 --pmc $pass --kernel-include-regex "bh_traverse|tile_apply" -d $O/pmcs_$k -o pmc \
      --output-format csv -- python scripts/bh_snap.py $SN/Y_t250.npy $SN/Y_t650.npy --reps 1 > $O/pmcs_$k.log 2>&1 || exit $?
  done
fi
if has valusnap; then   # fp64/VALU instructions per wave pop of bh_traverse<0> on the C3 snapshots,
  # per library build (VALU_LIBS, "-" = the in-tree one), narrow layout off so every group is a 64-query wave
  k=0
  for v in ${VALU_LIBS:--}; do
    lib=""; [ "$v" != "-" ] && lib="$v"
    k=$((k+1))
    echo "# $v" >> $O/valusnap.jsonl
    TSNE_HIP_LIB="$lib" run 300 python scripts/bh_snap.py $SN/Y_t250.npy $SN/Y_t450.npy --reps 3 --stats \
        --option narrow=0 >> $O/valusnap.jsonl 2>> $O/valusnap.err || exit $?
    TSNE_HIP_LIB="$lib" timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU \
        SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --kernel-include-regex "bh_traverse" -d $O/valu_$k -o pmc \
        --output-format csv -- python scripts/bh_snap.py $SN/Y_t250.npy $SN/Y_t450.npy --reps 1 --option narrow=0 \
        > $O/valu_$k.log 2>&1 || exit $?
  done
fi
if has proj; then
  for v in ${PROJ_VARS:--}; do
    opt=""; lib=""
    case "$v" in -) ;; lib=*) lib="${v#lib=}" ;; *) opt="--option ${v//+/ --option }" ;; esac
    echo "# $v" >> $O/proj.jsonl
    TSNE_HIP_LIB="$lib" run 600 python scripts/loop_projection.py ${PROJ_ARGS:-} $opt >> $O/proj.jsonl 2>> $O/proj.err || exit $?
  done
fi
echo done > $O/done.txt
