# Round 5: the LDS-DMA bf16 weight gradient after its DMA-issue rework: its tests, then kbench over the
# c5 shapes against the register-staged kernel.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5c; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_wgrad_dma_gpu.py > $O/tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|Error" $O/tests.log | tail -30
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/kbench.py --c5 --ops wgrad_bf16,wgrad_bf16d > $O/kbench_wgrad_c5.txt 2>&1 || exit $?
grep -E "wgrad" $O/kbench_wgrad_c5.txt
echo r5c-done
