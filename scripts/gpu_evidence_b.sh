# Round evidence, part B: every GPU test, smoke, and the default c2 / c4 / c5 bench lines (CPU baselines,
# dice_vs_ref), citing the traffic files of part A (copied to the box's profiles/r03 first).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/round; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests_gpu.log 2>&1; rc=$?
echo "tests exit=$rc" >> $O/tests_gpu.log
tail -2 $O/tests_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 500 python bench.py --workload probunet > $O/bench_c4.json 2> $O/bench_c4.err || exit $?
timeout -k 10 500 python bench.py --workload c5 > $O/bench_c5.json 2> $O/bench_c5.err || exit $?
cut -c 1-200 $O/bench.json; cut -c 1-200 $O/bench_c4.json; cut -c 1-200 $O/bench_c5.json
echo evidence-b-done
