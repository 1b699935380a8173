set -u
O=gpurun_out/r7b; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_convT_gpu.py tests/test_blocks_gpu.py > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/tests.log | head; exit $rc; }
timeout -k 10 600 python tools/lib_bitcmp.py > $O/bitcmp.log 2>&1; cat $O/bitcmp.log
for lib in prev rel prev rel; do
  L=$lib; [ $lib = rel ] && L=""
  PMU_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c2_$lib.json 2> $O/c2_$lib.err || exit $?
  python -c "import json;d=json.load(open('$O/c2_$lib.json'));print('c2 $lib', d['value'], d['ms_per_step'])"
done
for lib in prev rel; do
  L=$lib; [ $lib = rel ] && L=""
  PMU_LIB=$L timeout -k 10 300 python bench.py --workload probunet --no-cpu-baseline > $O/c4_$lib.json 2> $O/c4_$lib.err || exit $?
  python -c "import json;d=json.load(open('$O/c4_$lib.json'));print('c4 $lib', d['value'], d['ms_per_step'])"
done
