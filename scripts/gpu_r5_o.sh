# Round 5: c2's pooled layers' gradient unstored (fp32 parts) and dz read in place by the fp32 input
# gradient.  Fusion tests (release + debug), c2 bench A/B (PMU_POOL_FUSE=0/1 and PMU_HEAD_FUSE), full suite.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5o; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_pool_fuse_gpu.py tests/test_head_fuse_gpu.py > $O/fuse_tests.log 2>&1; rc=$?
grep -E "FAILED|Error|error|passed|failed" $O/fuse_tests.log | tail -12
[ $rc -ne 0 ] && exit $rc
PMU_LIB=debug timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_pool_fuse_gpu.py tests/test_head_fuse_gpu.py > $O/fuse_tests_debug.log 2>&1; rc=$?
tail -2 $O/fuse_tests_debug.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for v in "PMU_POOL_FUSE=0 PMU_HEAD_FUSE=0" "PMU_POOL_FUSE=1 PMU_HEAD_FUSE=1"; do
    tag=$(echo $v | tr -d ' =_')
    env $v timeout -k 10 600 python bench.py --no-cpu-baseline --steps 20 > $O/bench_c2_${tag}_$i.json 2> $O/bench_c2_${tag}_$i.err || exit $?
    python -c "import json;d=json.load(open('$O/bench_c2_${tag}_$i.json'));print('$v', d['value'], d['ms_per_step'])"
  done
done
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests_gpu.log 2>&1; rc=$?
tail -3 $O/tests_gpu.log
[ $rc -ne 0 ] && exit $rc
echo r5o-done
