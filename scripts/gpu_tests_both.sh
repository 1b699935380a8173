# Full GPU test suite on the shipped library, then again on the bounds-checked debug library
# (PMU_LIB=debug: every GPU test fails if a kernel recorded an index-bound violation).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/tests; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 600 --timeout-method thread > $O/tests_gpu.log 2>&1; rc=$?
echo "tests exit=$rc" >> $O/tests_gpu.log
tail -3 $O/tests_gpu.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" $O/tests_gpu.log | head -20; exit $rc; fi
PMU_LIB=debug timeout -k 10 1000 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 600 --timeout-method thread > $O/tests_gpu_debug.log 2>&1; rc=$?
echo "tests exit=$rc" >> $O/tests_gpu_debug.log
tail -3 $O/tests_gpu_debug.log
grep -E "FAILED" $O/tests_gpu_debug.log | head -20
exit $rc
