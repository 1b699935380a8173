# LDS-DMA bf16 conv: kernel parity tests, then c5-shape kbench against the register-staged kernel,
# then the full GPU suites (release + debug library).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/dma; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_bf16_gpu.py -q -k "dma" -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests_dma.log 2>&1; rc=$?
tail -3 $O/tests_dma.log
if [ $rc -ne 0 ]; then grep -E "FAILED|assert" $O/tests_dma.log | head -20; exit $rc; fi
timeout -k 10 300 python -u tools/kbench.py --c5 --ops fwd_dma,fwd_raw,dgrad_dma,dgrad_raw --iters 10 > $O/kbench_c5.txt 2>&1 || exit $?
grep TOTAL $O/kbench_c5.txt
bash scripts/gpu_tests_both.sh
