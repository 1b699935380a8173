# Round 5 final: the whole GPU suite on the bounds-checked debug library (PMU_LIB=debug).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5dbg; mkdir -p $O
cd $R
PMU_LIB=debug timeout -k 10 1000 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests_gpu_debug.log 2>&1; rc=$?
tail -3 $O/tests_gpu_debug.log
exit $rc
