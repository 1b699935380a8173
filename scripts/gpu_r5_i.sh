# Round 5: transposed-accumulator epilogue of the LDS-DMA convs (16-B stores / z loads).  DMA-conv
# tests (release, then the bounds-checked debug build), kbench of the DMA convs A/B against the
# previous build (PMU_LIB=prev = HEAD before the change), then c5 bench A/B.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5i; mkdir -p $O
cd $R
T="tests/test_bf16_gpu.py tests/test_dxb_gpu.py tests/test_bnr_gpu.py tests/test_zb_gpu.py tests/test_pool_fuse_gpu.py"
timeout -k 10 900 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread $T > $O/dma_tests.log 2>&1; rc=$?
tail -3 $O/dma_tests.log
[ $rc -ne 0 ] && exit $rc
PMU_LIB=debug timeout -k 10 900 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_bf16_gpu.py tests/test_dxb_gpu.py -k "dma or dxb" > $O/dma_tests_debug.log 2>&1; rc=$?
tail -2 $O/dma_tests_debug.log
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
echo r5i-done
