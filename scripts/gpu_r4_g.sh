# Round-4 step G: fp32 outputs of the LDS-DMA conv (z, dx) and of the F(2x2) / F(4x4) Winograd kernels
# stored as 8-byte channel pairs (a lane-pair shuffle; half the store instructions).  Touched-kernel
# tests, then kbench and bench A/B against PMU_LIB=prev (the library of commit 8d32157).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4g; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_wino4_gpu.py tests/test_wino2h_gpu.py tests/test_bnr_gpu.py tests/test_large_gpu.py \
  tests/test_unet_gpu.py tests/test_bf16_gpu.py tests/test_tee32_gpu.py -k "not batch16" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
for L in prev r4; do
  E=""; [ $L = prev ] && E="PMU_LIB=prev"
  env $E timeout -k 10 300 python tools/kbench.py --ops fwd_w2h,dgrad_w4 --iters 5 > $O/kbench_c2_$L.txt 2>&1 || exit $?
  env $E timeout -k 10 300 python tools/kbench.py --c5 --ops fwd_dma,dgrad_dma,dgrad_dmab --iters 5 > $O/kbench_c5_$L.txt 2>&1 || exit $?
  grep TOTAL $O/kbench_c2_$L.txt $O/kbench_c5_$L.txt
done
for L in prev r4; do
  E=""; [ $L = prev ] && E="PMU_LIB=prev"
  env $E timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c2_$L.json 2> $O/bench_c2_$L.err || exit $?
  env $E timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline --no-eval > $O/bench_c5_$L.json 2> $O/bench_c5_$L.err || exit $?
  cut -c 1-160 $O/bench_c2_$L.json $O/bench_c5_$L.json
done
