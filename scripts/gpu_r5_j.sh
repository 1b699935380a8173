# Round 5: the transposed-epilogue DMA convs.  Seed spread of the c5 bf16 Dice-gap statistic for the
# previous build (PMU_LIB=prev) and this one, the debug-build DMA tests, then kbench and c5 bench A/B.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5j; mkdir -p $O
cd $R
for lib in prev cur; do
  L=""; [ $lib = prev ] && L=prev
  PMU_LIB=$L timeout -k 10 600 python tools/dice_gap_seeds.py --seeds 0,1,2,3,4,5 --out $O/dice_gap_seeds_$lib.json > $O/dice_gap_seeds_$lib.log 2>&1 || exit $?
  grep SUMMARY $O/dice_gap_seeds_$lib.log | cut -c1-400
done
PMU_LIB=debug timeout -k 10 900 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_bf16_gpu.py tests/test_dxb_gpu.py -k "dma or dxb" > $O/dma_tests_debug.log 2>&1; rc=$?
tail -2 $O/dma_tests_debug.log
[ $rc -ne 0 ] && exit $rc
for lib in prev cur; do
  L=""; [ $lib = prev ] && L=prev
  PMU_LIB=$L timeout -k 10 300 python tools/kbench.py --c5 --ops fwd_dma,dgrad_dma,dgrad_dmab > $O/kbench_dma_c5_$lib.txt 2>&1 || exit $?
  echo "lib=$lib"; grep TOTAL $O/kbench_dma_c5_$lib.txt
done
for lib in prev cur prev cur; do
  L=""; [ $lib = prev ] && L=prev
  PMU_LIB=$L timeout -k 10 600 python bench.py --workload c5 --no-cpu-baseline --no-eval > $O/bench_c5_$lib.json 2> $O/bench_c5_$lib.err || exit $?
  python -c "import json;d=json.load(open('$O/bench_c5_$lib.json'));print('$lib', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
done
echo r5j-done
