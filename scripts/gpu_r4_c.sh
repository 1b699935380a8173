# Round-4 step C: serpentine chunk order of the Winograd pass pipelines (F(4x4) input gradient,
# F(2x2) high-occupancy kernels) and XCD-ordered (channel block, split) workgroups of the bf16 / fp32
# weight-gradient kernels (3x3 and ConvT).  Parity of the touched kernels, then A/B against the
# previous code (PMU_LIB=prev) in time and PMC HBM bytes, then the c2 / c5 bench lines.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4c; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_wino4_gpu.py tests/test_wino2h_gpu.py tests/test_convT_gpu.py tests/test_unet_gpu.py \
  tests/test_bf16_gpu.py -k "not batch16" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for L in prev r4; do
  E=""; [ $L = prev ] && E="PMU_LIB=prev"
  env $E timeout -k 10 300 python tools/kbench.py --ops fwd_w2h,dgrad_w4,wgrad_wino --iters 5 > $O/kbench_c2_$L.txt 2>&1 || exit $?
  env $E timeout -k 10 300 python tools/kbench.py --c5 --ops wgrad_bf16 --iters 5 > $O/kbench_c5_$L.txt 2>&1 || exit $?
  env $E timeout -k 10 120 python tools/kbench_convt.py --c5 --ops wgrad_bf16 --iters 10 > $O/kbench_convT_c5_$L.txt 2>&1 || exit $?
  env $E timeout -k 10 120 python tools/kbench_convt.py --ops wgrad --iters 10 > $O/kbench_convT_c2_$L.txt 2>&1 || exit $?
  grep TOTAL $O/kbench_*_$L.txt
done
# PMC HBM bytes per dispatch of the same kernels (one pass per counter, kernel trace only)
cd /tmp && export TMPDIR=/tmp
for L in prev r4; do
  for C in FETCH_SIZE WRITE_SIZE; do
    if [ $L = prev ]; then export PMU_LIB=prev; else unset PMU_LIB; fi
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/pmc_${L}_c2_$C -o run -- python3 $R/tools/kbench.py --ops fwd_w2h,dgrad_w4,wgrad_wino --iters 1 > $O/pmc_${L}_c2_$C.log 2>&1 || exit $?
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/pmc_${L}_c5_$C -o run -- python3 $R/tools/kbench.py --c5 --ops wgrad_bf16 --iters 1 > $O/pmc_${L}_c5_$C.log 2>&1 || exit $?
  done
  unset PMU_LIB
  python3 $R/tools/pmc_traffic.py $O/pmc_${L}_c2_FETCH_SIZE $O/pmc_${L}_c2_WRITE_SIZE $O/pmc_${L}_c2.json > $O/pmc_${L}_c2.txt || exit $?
  python3 $R/tools/pmc_traffic.py $O/pmc_${L}_c5_FETCH_SIZE $O/pmc_${L}_c5_WRITE_SIZE $O/pmc_${L}_c5.json > $O/pmc_${L}_c5.txt || exit $?
  cat $O/pmc_${L}_c2.txt $O/pmc_${L}_c5.txt
done
cd $R
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || exit $?
timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline --no-eval > $O/bench_c5.json 2> $O/bench_c5.err || exit $?
cut -c 1-260 $O/bench_c2.json $O/bench_c5.json
