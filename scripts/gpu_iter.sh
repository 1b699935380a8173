# One development iteration: the named GPU test files (TESTS), then the c2 and (BENCH_C5=1) c5 bench
# lines without the CPU legs.  Every GPU step has its own time limit; the first failure ends the call.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/iter; mkdir -p $O
cd $R
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread $TESTS \
    > $O/tests.log 2>&1
  rc=$?; echo "tests exit=$rc" >> $O/tests.log; tail -3 $O/tests.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
if [ "${BENCH_C2:-1}" = "1" ]; then
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || exit $?
  cut -c 1-260 $O/bench_c2.json
fi
if [ "${BENCH_C5:-0}" = "1" ]; then
  timeout -k 10 400 python bench.py --workload c5 --no-cpu-baseline --no-eval > $O/bench_c5.json 2> $O/bench_c5.err || exit $?
  cut -c 1-260 $O/bench_c5.json
fi
echo iter-done
