# Round 5: DMA weight gradient without the halo-row rotation copies.  Its tests, kbench A/B against the
# previous build (PMU_LIB=prev), c5 bench A/B.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5m; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_wgrad_dma_gpu.py > $O/wgrad_tests.log 2>&1; rc=$?
tail -2 $O/wgrad_tests.log
[ $rc -ne 0 ] && exit $rc
for lib in prev cur prev cur; do
  L=""; [ $lib = prev ] && L=prev
  PMU_LIB=$L timeout -k 10 300 python tools/kbench.py --c5 --ops wgrad_bf16d > $O/kbench_wgrad_c5_$lib.txt 2>&1 || exit $?
  echo "lib=$lib $(grep TOTAL $O/kbench_wgrad_c5_$lib.txt)"
done
for lib in prev cur prev cur; do
  L=""; [ $lib = prev ] && L=prev
  PMU_LIB=$L timeout -k 10 600 python bench.py --workload c5 --no-cpu-baseline --no-eval > $O/bench_c5_$lib.json 2> $O/bench_c5_$lib.err || exit $?
  python -c "import json;d=json.load(open('$O/bench_c5_$lib.json'));print('$lib', d['value'], d['ms_per_step'])"
done
echo r5m-done
