# Round 5 evidence, part A: the full GPU suite, smoke, the c2 / c4 / c5 bench lines with CPU baselines
# and dice_vs_ref, and c3's phantom line (with the slicer's own rate).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/round5; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests_gpu.log 2>&1; rc=$?
echo "tests exit=$rc" >> $O/tests_gpu.log
tail -2 $O/tests_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || exit $?
timeout -k 10 600 python bench.py --workload probunet > $O/bench_c4.json 2> $O/bench_c4.err || exit $?
timeout -k 10 900 python bench.py --workload c5 > $O/bench_c5.json 2> $O/bench_c5.err || exit $?
timeout -k 10 600 python bench.py --data phantom --no-cpu-baseline > $O/bench_c3_phantom.json 2> $O/bench_c3.err || exit $?
for f in c2 c4 c5 c3_phantom; do cut -c 1-220 $O/bench_$f.json; done
echo round-a-done
