set -u
O=gpurun_out/r6m; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -m gpu -p no:cacheprovider --timeout 500 --timeout-method thread tests/test_pack_gpu.py tests/test_wino_b64_gpu.py tests/test_wino2h_gpu.py tests/test_train_gpu.py > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for lib in prev rel prev rel; do
  L=$lib; [ $lib = rel ] && L=""
  PMU_LIB=$L timeout -k 10 300 python tools/kbench.py --ops fwd_w2h,dgrad_w2h,dgrad_w2hb --iters 10 > $O/kb_$lib.log 2>&1 || exit $?
  echo "$lib $(grep TOTAL $O/kb_$lib.log | tr '\n' ' ')"
done
for lib in prev rel prev rel; do
  L=$lib; [ $lib = rel ] && L=""
  PMU_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c2_$lib.json 2> $O/c2_$lib.err || exit $?
  python -c "import json;d=json.load(open('$O/c2_$lib.json'));print('c2 $lib', d['value'], d['ms_per_step'])"
done
