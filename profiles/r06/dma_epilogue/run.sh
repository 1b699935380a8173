set -u
O=gpurun_out/r6o; mkdir -p $O
timeout -k 10 600 python tools/lib_bitcmp.py > $O/bitcmp.log 2>&1; rc=$?; cat $O/bitcmp.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 500 --timeout-method thread tests/test_dxb_gpu.py tests/test_bnr_gpu.py tests/test_convT_gpu.py tests/test_dma_pers_gpu.py tests/test_zb_gpu.py > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for lib in prev rel prev rel; do
  L=$lib; [ $lib = rel ] && L=""
  PMU_LIB=$L timeout -k 10 300 python tools/kbench.py --c5 --ops fwd_dma,dgrad_dmax,dgrad_dmabx --iters 10 > $O/kb_$lib.log 2>&1 || exit $?
  echo "$lib $(grep TOTAL $O/kb_$lib.log | tr '\n' ' ')"
done
for v in 0 1 2 3 0 1 2 3; do
  PMU_LIB=exp PMU_WGD_EXP=$v timeout -k 10 300 python tools/kbench.py --c5 --ops wgrad_bf16d --iters 10 > $O/kbw_exp$v.log 2>&1 || exit $?
  echo "wgd exp=$v $(grep TOTAL $O/kbw_exp$v.log)"
done
for lib in prev rel; do
  L=$lib; [ $lib = rel ] && L=""
  PMU_LIB=$L timeout -k 10 600 python bench.py --workload c5 --no-cpu-baseline --no-eval > $O/c5_$lib.json 2> $O/c5_$lib.err || exit $?
  python -c "import json;d=json.load(open('$O/c5_$lib.json'));print('c5 $lib', d['value'], d['ms_per_step'])"
done
