# Round 5: the last layer's activation gradient left unstored (HeadDa).  New tests (release + debug),
# c2 / c5 bench A/B (PMU_HEAD_FUSE=0/1), then the full GPU suite.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5k; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_head_fuse_gpu.py tests/test_pool_fuse_gpu.py tests/test_bnr_gpu.py > $O/fuse_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|Error|error" $O/fuse_tests.log | tail -24
[ $rc -ne 0 ] && exit $rc
PMU_LIB=debug timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_head_fuse_gpu.py > $O/fuse_tests_debug.log 2>&1; rc=$?
tail -2 $O/fuse_tests_debug.log
[ $rc -ne 0 ] && exit $rc
for f in 0 1 0 1; do
  PMU_HEAD_FUSE=$f timeout -k 10 600 python bench.py --workload c5 --no-cpu-baseline --no-eval > $O/bench_c5_head$f.json 2> $O/bench_c5_head$f.err || exit $?
  python -c "import json;d=json.load(open('$O/bench_c5_head$f.json'));print('c5 head_fuse=$f', d['value'], d['ms_per_step'])"
done
for f in 0 1 0 1; do
  PMU_HEAD_FUSE=$f timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench_c2_head$f.json 2> $O/bench_c2_head$f.err || exit $?
  python -c "import json;d=json.load(open('$O/bench_c2_head$f.json'));print('c2 head_fuse=$f', d['value'], d['ms_per_step'], d['dice_vs_ref']['label_agreement'])"
done
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests_gpu.log 2>&1; rc=$?
tail -3 $O/tests_gpu.log
[ $rc -ne 0 ] && exit $rc
echo r5k-done
