# Full validation: every GPU test, smoke, and the c2 / c4 / c5 bench lines (no CPU legs).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/full; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests_gpu.log 2>&1
rc=$?; echo "tests exit=$rc" >> $O/tests_gpu.log; tail -3 $O/tests_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || exit $?
timeout -k 10 400 python bench.py --workload probunet --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err || exit $?
timeout -k 10 400 python bench.py --workload c5 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || exit $?
for f in c2 c4 c5; do cut -c 1-200 $O/bench_$f.json; done
echo full-done
