set -u
O=gpurun_out/r6r; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_wgrad_dma_gpu.py > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/tests.log | head -20; exit $rc; }
timeout -k 10 600 python tools/lib_bitcmp.py > $O/bitcmp.log 2>&1; rc=$?; cat $O/bitcmp.log; [ $rc -ne 0 ] && exit $rc
for lib in prev rel prev rel; do
  L=$lib; [ $lib = rel ] && L=""
  PMU_LIB=$L timeout -k 10 300 python tools/kbench.py --c5 --ops wgrad_bf16d --iters 10 > $O/kb_$lib.log 2>&1 || exit $?
  echo "$lib $(grep TOTAL $O/kb_$lib.log | tr '\n' ' ')"
done
for v in 2 1; do
  PMU_LIB=exp PMU_WGD_EXP=$v timeout -k 10 300 python tools/kbench.py --c5 --ops wgrad_bf16d --iters 10 > $O/kbw_exp$v.log 2>&1 || exit $?
  echo "wgd exp=$v $(grep TOTAL $O/kbw_exp$v.log)"
done
