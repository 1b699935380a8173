# Round 5: persistent tile schedule of the LDS-DMA convs.  New tests (release, then the bounds-checked
# debug build), the DMA tests of test_bf16_gpu, the c5 kbench of the DMA convs with the persistent
# schedule on / off, and c5 bench A/B.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5f; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_dma_pers_gpu.py > $O/pers_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|Error|error" $O/pers_tests.log | tail -30
[ $rc -ne 0 ] && exit $rc
PMU_LIB=debug timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_dma_pers_gpu.py > $O/pers_tests_debug.log 2>&1; rc=$?
tail -3 $O/pers_tests_debug.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_bf16_gpu.py tests/test_dxb_gpu.py tests/test_bnr_gpu.py > $O/dma_tests.log 2>&1; rc=$?
tail -3 $O/dma_tests.log
[ $rc -ne 0 ] && exit $rc
for p in 1 0; do
  PMU_DMA_PERS=$p timeout -k 10 300 python tools/kbench.py --c5 --ops fwd_dma,dgrad_dma,dgrad_dmab > $O/kbench_dma_c5_pers$p.txt 2>&1 || exit $?
  echo "pers=$p"; grep TOTAL $O/kbench_dma_c5_pers$p.txt
done
for p in 0 1 0 1; do
  PMU_DMA_PERS=$p timeout -k 10 600 python bench.py --workload c5 --no-cpu-baseline --no-eval > $O/bench_c5_pers$p.json 2> $O/bench_c5_pers$p.err || exit $?
  python -c "import json;d=json.load(open('$O/bench_c5_pers$p.json'));print('pers=$p', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
done
echo r5f-done
