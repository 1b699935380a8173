# Round 5: LDS-DMA bf16 weight gradient, per-segment source offsets (WS == 1): tests, kbench, SQ counters.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5d; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_wgrad_dma_gpu.py > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/kbench.py --c5 --ops wgrad_bf16,wgrad_bf16d > $O/kbench_wgrad_c5.txt 2>&1 || exit $?
grep -E "wgrad" $O/kbench_wgrad_c5.txt
bash scripts/gpu_sq_wgd.sh > $O/sq.log 2>&1 || exit $?
cp -r gpurun_out/sqwgd $O/ 2>/dev/null || true
echo r5d-done
