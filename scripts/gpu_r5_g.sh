# Round 5: L2-dropping (sc1) output stores in the LDS-DMA convs, A/B against the previous build
# (PMU_LIB=prev = the same tree before the change): c5 kbench of the DMA convs, DMA tests, c5 bench.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5g; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_bf16_gpu.py tests/test_dxb_gpu.py tests/test_bnr_gpu.py tests/test_dma_pers_gpu.py > $O/dma_tests.log 2>&1; rc=$?
tail -3 $O/dma_tests.log
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
echo r5g-done
