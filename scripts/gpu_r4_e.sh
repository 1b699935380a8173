# Round-4 step E: persistent LDS-DMA conv and F(2x2) / F(4x4) Winograd kernels (a workgroup per resident slot walks tiles, the next tile's
# first chunk under this tile's last MFMAs), co-block-parity serpentine order, first-layer kernels
# (multi-tile forward with the next patch prefetched; weight gradient da / z two pixels ahead),
# streaming max-pool backward (ping-pong windows) and the batched head forward.  Touched-kernel tests,
# then kbench and bench A/B against PMU_LIB=prev (the library of commit 29c9cac).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4e; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_bf16_gpu.py tests/test_bnr_gpu.py tests/test_first_layer_gpu.py tests/test_large_gpu.py \
  tests/test_wino4_gpu.py tests/test_wino2h_gpu.py tests/test_unet_gpu.py tests/test_blocks_gpu.py \
  tests/test_probunet_gpu.py -k "not batch16" > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; grep FAILED $O/tests.log
# a fault / abort / timeout ends the call; assertion failures are recorded and the A/B still runs
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for L in prev r4; do
  E=""; [ $L = prev ] && E="PMU_LIB=prev"
  env $E timeout -k 10 300 python tools/kbench.py --c5 --ops fwd_dma,dgrad_dma,dgrad_dmab --iters 5 > $O/kbench_c5_$L.txt 2>&1 || exit $?
  env $E timeout -k 10 300 python tools/kbench.py --ops fwd_w2h,dgrad_w4 --iters 5 > $O/kbench_c2_$L.txt 2>&1 || exit $?
  grep TOTAL $O/kbench_c5_$L.txt $O/kbench_c2_$L.txt
done
for L in prev r4; do
  E=""; [ $L = prev ] && E="PMU_LIB=prev"
  env $E timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline --no-eval > $O/bench_c5_$L.json 2> $O/bench_c5_$L.err || exit $?
  env $E timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c2_$L.json 2> $O/bench_c2_$L.err || exit $?
  env $E timeout -k 10 300 python bench.py --workload probunet --no-cpu-baseline > $O/bench_c4_$L.json 2> $O/bench_c4_$L.err || exit $?
  cut -c 1-200 $O/bench_c5_$L.json $O/bench_c2_$L.json $O/bench_c4_$L.json
done
