set -u
O=gpurun_out/r7a; mkdir -p $O
timeout -k 10 600 env PMU_LIB=exp PMU_CONVT_PF2=1 python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_convT_gpu.py > $O/tests_pf2.log 2>&1; rc=$?; tail -2 $O/tests_pf2.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/tests_pf2.log | head; exit $rc; }
for v in 0 1 0 1; do
  PMU_LIB=exp PMU_CONVT_PF2=$v timeout -k 10 300 python tools/kbench_convt.py --ops fwd,dgrad --iters 20 > $O/kb_pf$v.log 2>&1 || exit $?
  echo "pf2=$v $(grep -i total $O/kb_pf$v.log | tr '\n' ' ')"
done
cat $O/kb_pf0.log $O/kb_pf1.log
