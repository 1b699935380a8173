# Round 5: the first layer's per-tile BN partial reduction over all threads.  First-layer / BN tests,
# kernel-trace stats prev vs current on c2 and c5, then c5 / c2 bench A/B.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5t; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_first_layer_gpu.py tests/test_bnr_gpu.py tests/test_train_gpu.py > $O/tests.log 2>&1; rc=$?
grep -E "FAILED|Error|passed|failed" $O/tests.log | tail -8
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
for lib in prev cur; do
  [ $lib = prev ] && export PMU_LIB=prev || unset PMU_LIB
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5_$lib -o bench -- python3 $R/bench.py --workload c5 --no-eval --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing > $O/prof_c5_$lib.log 2>&1 || exit $?
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2_$lib -o bench -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing > $O/prof_c2_$lib.log 2>&1 || exit $?
done
unset PMU_LIB
cd $R
for i in 1 2; do
  for lib in prev cur; do
    [ $lib = prev ] && L=prev || L=
    PMU_LIB=$L timeout -k 10 600 python bench.py --workload c5 --no-eval --no-cpu-baseline --steps 20 > $O/bench_c5_${lib}_$i.json 2> $O/bench_c5_${lib}_$i.err || exit $?
    python -c "import json;d=json.load(open('$O/bench_c5_${lib}_$i.json'));print('c5 $lib', d['value'], d['ms_per_step'])"
  done
done
echo r5t-done
