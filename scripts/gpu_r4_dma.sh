# A/B of the round-4 kernel-pipeline changes against the previous code (PMU_LIB=prev, built from the
# previous sources): LDS-DMA conv / ConvT chunk pipelines (next chunk's first operands read under this
# chunk's last MFMAs) on the c5 shapes and the Winograd epilogues (exchange reads ahead of the store
# branches) on the c2 shapes; then the full GPU suite, c2 and c5 bench lines, the MFMA counter
# calibration.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4dma; mkdir -p $O
cd $R
for L in exp rel; do
  E=""; [ $L = exp ] && E="PMU_LIB=prev"
  env $E timeout -k 10 300 python tools/kbench.py --c5 --ops fwd_dma,dgrad_dma,dgrad_dmab --iters 5 > $O/kbench_c5_$L.txt 2>&1 || exit $?
  env $E timeout -k 10 120 python tools/kbench_convt.py --c5 --ops fwd_dma,dgrad_dma --iters 10 > $O/kbench_convT_c5_$L.txt 2>&1 || exit $?
  env $E timeout -k 10 300 python tools/kbench.py --ops fwd_w2h,dgrad_w4,dgrad_w4b,dgrad_w2h --iters 5 > $O/kbench_c2_$L.txt 2>&1 || exit $?
  grep TOTAL $O/kbench_c5_$L.txt $O/kbench_convT_c5_$L.txt $O/kbench_c2_$L.txt
done
timeout -k 10 900 python -u -m pytest -q -p no:cacheprovider --timeout 600 --timeout-method thread -m gpu tests > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" $O/tests.log | head; exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || exit $?
timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline --no-eval > $O/bench_c5.json 2> $O/bench_c5.err || exit $?
cut -c 1-200 $O/bench_c2.json $O/bench_c5.json
bash scripts/gpu_mfma_calib.sh || exit $?
bash scripts/gpu_sq_dma.sh || exit $?
